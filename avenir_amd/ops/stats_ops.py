"""K26 rank statistics on the device (csrc/kernels/stats.hip) with CPU twins.

Reference: P/mlextra/daexp.py (getSpearmanRankCorr, getKendalRankCorr, testTwoSampleMw,
testTwoSampleKw, :1093-1175 / :1458-1836) hands host arrays to scipy.stats.  Here the sample stays
on its device: one sort (rocPRIM via torch.sort), ONE ``rank_avg`` launch for tie-averaged ranks, the
tie-correction terms and per-group rank sums, and for Kendall ONE ``kendall_pairs`` launch counting
concordant / discordant / tied pairs exactly.  Only scalars reach the host, where the p-values are
closed-form functions of them (the same asymptotic formulas scipy uses; small tie-free samples, for
which scipy switches to exact null distributions, are delegated to scipy on those few values).
"""
from __future__ import annotations

import math

import torch

from .. import _native


def _dev(x) -> torch.Tensor:
    return torch.as_tensor(x).double().contiguous().view(-1)


def rank_avg(x: torch.Tensor, group: torch.Tensor | None = None, n_groups: int = 0):
    """(ranks f64 [n] — average over ties, 1-based; tie terms f64 [4] = sum (t^3 - t),
    sum t (t - 1), sum t (t - 1)(t - 2), sum t (t - 1)(2t + 5) over tie runs; rank sums f64
    [n_groups] of ``group`` int [n] or None)."""
    x = _dev(x)
    n = x.numel()
    sv, perm = torch.sort(x, stable=True)
    if x.is_cuda:
        g = group.to(x.device, torch.int32).contiguous() if group is not None else None
        r, tie, gs = _native.C().rank_avg(sv.contiguous(), perm.contiguous(), g, int(max(n_groups, 1)))
        return r, tie, (gs[:n_groups] if group is not None else None)
    # CPU twin: run bounds by searchsorted on the sorted copy
    lo = torch.searchsorted(sv, sv, right=False)
    hi = torch.searchsorted(sv, sv, right=True)
    ranks = torch.empty(n, dtype=torch.float64)
    ranks[perm] = 0.5 * (lo + 1 + hi).double()
    start = lo == torch.arange(n)
    t = (hi - lo)[start].double()
    tie = torch.stack([(t ** 3 - t).sum(), (t * (t - 1)).sum(), (t * (t - 1) * (t - 2)).sum(),
                       (t * (t - 1) * (2 * t + 5)).sum()]) if n else torch.zeros(4, dtype=torch.float64)
    gs = None
    if group is not None:
        gg = group.long()
        ok = (gg >= 0) & (gg < n_groups)
        gs = torch.zeros(n_groups, dtype=torch.float64).index_add_(0, gg[ok], ranks[ok])
    return ranks, tie, gs


KENDALL_PAIRS_MAX_N = 1 << 15   # above: the O(n log^2 n) merge count beats the O(n^2) pair kernel


def _tie_pairs(v: torch.Tensor) -> torch.Tensor:
    """sum over runs of equal values (v sorted; rows of a 2-D v) of t (t - 1) / 2."""
    _, c = torch.unique_consecutive(v, dim=0, return_counts=True)
    c = c.long()
    return (c * (c - 1) // 2).sum()


def _kendall_merge_counts(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """Knight's method on the device: order by (x, y), count the strict inversions of the y sequence
    level by level (blocks of 2s: every right-half value's count of larger left-half values by one
    batched searchsorted, then the blocks sorted for the next level) — the discordant pairs, since
    pairs tied in x are ordered by y and never inverted.  Tie pairs from run lengths; concordant =
    all - discordant - tied.  O(n log^2 n) work: on the GPU the merge-path kernels of stats.hip
    (1 + log2(n / 1024) launches), on the CPU a batched sort + searchsorted per level."""
    n = x.numel()
    o = torch.sort(y, stable=True).indices
    o = o[torch.sort(x[o], stable=True).indices]
    xs, ys = x[o], y[o]
    if ys.is_cuda:
        # stats.hip merge-path kernels: runs <= 1024 merged in LDS, then one launch per level
        inv = _native.C().inversion_count(ys.double().contiguous())[0]
    else:
        m = 1 << max(0, (n - 1).bit_length())
        cur = torch.cat([ys, torch.full((m - n,), float("inf"), dtype=ys.dtype, device=ys.device)])
        inv = torch.zeros((), dtype=torch.int64, device=x.device)
        s = 1
        while s < m:
            blk = cur.view(-1, 2, s)
            L, R = blk[:, 0, :].contiguous(), blk[:, 1, :].contiguous()
            inv += (s - torch.searchsorted(L, R, right=True)).sum()
            cur = torch.sort(cur.view(-1, 2 * s), dim=1).values.view(-1)
            s *= 2
    both = _tie_pairs(torch.stack([xs, ys], 1))
    tx = _tie_pairs(xs)
    ty = _tie_pairs(torch.sort(y).values)
    tot = torch.tensor(n * (n - 1) // 2, dtype=torch.int64, device=x.device)
    tx_only, ty_only = tx - both, ty - both
    return torch.stack([tot - inv - tx_only - ty_only - both, inv, tx_only, ty_only, both])


def kendall_counts(x: torch.Tensor, y: torch.Tensor, method: str = "auto") -> torch.Tensor:
    """int64 [5]: concordant, discordant, tied in x only, tied in y only, tied in both (pairs i < j).
    ``method``: "pairs" (GPU: the exact all-pairs kernel; CPU: tiled tensor comparisons), "merge"
    (sort-based inversion count) or "auto" (pairs up to KENDALL_PAIRS_MAX_N values on the GPU and
    4096 on the CPU, merge above)."""
    x, y = _dev(x), _dev(y).to(_dev(x).device)
    if method == "merge" or (method == "auto" and x.numel() > (KENDALL_PAIRS_MAX_N if x.is_cuda else 4096)):
        return _kendall_merge_counts(x, y)
    if x.is_cuda:
        return _native.C().kendall_pairs(x, y)
    n = x.numel()
    out = torch.zeros(5, dtype=torch.int64)
    step = max(1, (1 << 22) // max(n, 1))
    for i0 in range(0, n, step):
        xi, yi = x[i0:i0 + step].view(-1, 1), y[i0:i0 + step].view(-1, 1)
        a, b = torch.sign(xi - x.view(1, -1)), torch.sign(yi - y.view(1, -1))
        upper = torch.arange(i0, min(n, i0 + step)).view(-1, 1) < torch.arange(n).view(1, -1)
        s = a * b
        out += torch.stack([((s > 0) & upper).sum(), ((s < 0) & upper).sum(), ((a == 0) & (b != 0) & upper).sum(),
                            ((a != 0) & (b == 0) & upper).sum(), ((a == 0) & (b == 0) & upper).sum()])
    return out


def _pearson(a: torch.Tensor, b: torch.Tensor) -> float:
    ac, bc = a - a.mean(), b - b.mean()
    den = float(ac.norm() * bc.norm())
    return float(ac @ bc) / den if den > 0 else float("nan")


def spearman(x, y) -> tuple[float, float]:
    """(rho, two-sided p) as scipy.stats.spearmanr."""
    from scipy import stats
    rx, _, _ = rank_avg(x)
    ry, _, _ = rank_avg(torch.as_tensor(y).to(rx.device))
    n = rx.numel()
    rho = _pearson(rx, ry)
    if not math.isfinite(rho) or n < 3:
        return rho, float("nan")
    t = rho * math.sqrt((n - 2) / max(1e-300, (rho + 1.0) * (1.0 - rho)))
    return rho, float(2 * stats.t.sf(abs(t), n - 2))


def kendall_tau_b(x, y) -> tuple[float, float]:
    """(tau-b, two-sided p) as scipy.stats.kendalltau (variant b, method auto)."""
    from scipy import stats
    x, y = _dev(x), _dev(y).to(_dev(x).device)
    n = x.numel()
    if bool(torch.isnan(x).any() | torch.isnan(y).any()):
        return float("nan"), float("nan")          # scipy's nan_policy="propagate"
    cnt = kendall_counts(x, y).tolist()
    con, dis = cnt[0], cnt[1]
    _, tx, _ = rank_avg(x)
    _, ty, _ = rank_avg(y)
    tx, ty = tx.tolist(), ty.tolist()
    tot = n * (n - 1) // 2
    xtie, ytie = tx[1] / 2.0, ty[1] / 2.0
    if xtie == tot or ytie == tot:
        return float("nan"), float("nan")
    cmd = con - dis
    tau = cmd / math.sqrt(tot - xtie) / math.sqrt(tot - ytie)
    tau = min(1.0, max(-1.0, tau))
    if xtie == 0 and ytie == 0 and (n <= 33 or min(dis, tot - dis) <= 1):
        # scipy's exact null distribution for small tie-free samples (host, on the n values)
        return tau, float(stats.kendalltau(x.cpu().numpy(), y.cpu().numpy()).pvalue)
    m = n * (n - 1.0)
    var = ((m * (2 * n + 5) - tx[3] - ty[3]) / 18.0 + (2 * xtie * ytie) / m + tx[2] * ty[2] / (9 * m * (n - 2)))
    z = cmd / math.sqrt(var)
    return tau, float(2 * stats.norm.sf(abs(z)))


def mann_whitney_u(a, b) -> tuple[float, float]:
    """(U of the first sample, two-sided p) as scipy.stats.mannwhitneyu (continuity correction,
    method auto = scipy's ``_mwu_choose_method``: the exact null for tie-free samples unless BOTH
    hold more than 8 values)."""
    from scipy import stats
    a, b = _dev(a), _dev(b).to(_dev(a).device)
    n1, n2 = a.numel(), b.numel()
    z_all = torch.cat([a, b])
    grp = torch.cat([torch.zeros(n1, dtype=torch.int32), torch.ones(n2, dtype=torch.int32)]).to(z_all.device)
    _, tie, gs = rank_avg(z_all, grp, 2)
    r1 = float(gs[0])
    u1 = r1 - n1 * (n1 + 1) / 2.0
    t3 = float(tie[0])
    if (n1 <= 8 or n2 <= 8) and t3 == 0:
        return u1, float(stats.mannwhitneyu(a.cpu().numpy(), b.cpu().numpy()).pvalue)
    u2 = n1 * n2 - u1
    u = max(u1, u2)
    n = n1 + n2
    mu = n1 * n2 / 2.0
    s = math.sqrt(n1 * n2 / 12.0 * ((n + 1) - t3 / (n * (n - 1))))
    z = (u - mu - 0.5) / s if s > 0 else float("inf")
    return u1, float(min(1.0, max(0.0, 2 * stats.norm.sf(z))))


def kruskal_h(*samples) -> tuple[float, float]:
    """(H, p) as scipy.stats.kruskal."""
    from scipy import stats
    xs = [_dev(s) for s in samples]
    dev = xs[0].device
    z_all = torch.cat([s.to(dev) for s in xs])
    grp = torch.cat([torch.full((s.numel(),), k, dtype=torch.int32) for k, s in enumerate(xs)]).to(dev)
    _, tie, gs = rank_avg(z_all, grp, len(xs))
    N = z_all.numel()
    rs = gs.tolist()
    h = 12.0 / (N * (N + 1)) * sum(r * r / s.numel() for r, s in zip(rs, xs)) - 3 * (N + 1)
    tc = 1.0 - float(tie[0]) / (N ** 3 - N)
    if tc == 0:
        return float("nan"), float("nan")
    h /= tc
    return h, float(stats.chi2.sf(h, len(xs) - 1))


def wilcoxon_signed_rank(x, y) -> tuple[float, float]:
    """(statistic, two-sided p) as scipy.stats.wilcoxon(x, y) (zero_method "wilcox", no continuity
    correction, method auto).  The ranks of |x - y| over the non-zero differences and the positive
    / negative rank sums come from ONE rank_avg launch (group = sign); the tie term feeds the
    normal approximation.  Samples of <= 50 pairs (where scipy uses exact or permutation nulls)
    are delegated to scipy on those few values."""
    from scipy import stats
    x, y = _dev(x), _dev(y).to(_dev(x).device)
    if x.numel() != y.numel():
        raise ValueError("wilcoxon: x and y must have the same length")
    n_all = x.numel()
    if n_all <= 50:
        r = stats.wilcoxon(x.cpu().numpy(), y.cpu().numpy())
        return float(r.statistic), float(r.pvalue)
    d = x - y
    d = d[d != 0]
    n = d.numel()
    if n == 0:
        return 0.0, float("nan")
    _, tie, gs = rank_avg(d.abs(), (d > 0).to(torch.int32), 2)
    r_minus, r_plus = (float(v) for v in gs.tolist())
    mn = n * (n + 1.0) * 0.25
    se = math.sqrt((n * (n + 1.0) * (2.0 * n + 1.0) - float(tie[0]) / 2.0) / 24.0)
    z = (r_plus - mn) / se if se > 0 else float("nan")
    p = float(2 * stats.norm.sf(abs(z))) if math.isfinite(z) else float("nan")
    return min(r_plus, r_minus), min(1.0, p)


def cvm_2samp(x, y) -> tuple[float, float]:
    """(T, p) as scipy.stats.cramervonmises_2samp (method auto: asymptotic above 20 values per
    sample, else scipy's exact null on the host values).  Pooled ranks from one rank_avg launch;
    the ranks of each sample in ascending order are its pooled ranks sorted."""
    from scipy import stats
    x, y = _dev(x), _dev(y).to(_dev(x).device)
    nx, ny = x.numel(), y.numel()
    if nx < 2 or ny < 2:
        raise ValueError("x and y must contain at least two observations.")
    if max(nx, ny) <= 20:
        r = stats.cramervonmises_2samp(x.cpu().numpy(), y.cpu().numpy())
        return float(r.statistic), float(r.pvalue)
    r, _, _ = rank_avg(torch.cat([x, y]))
    rx = torch.sort(r[:nx]).values
    ry = torch.sort(r[nx:]).values
    dev = r.device
    u = (nx * ((rx - torch.arange(1, nx + 1, device=dev, dtype=torch.float64)) ** 2).sum()
         + ny * ((ry - torch.arange(1, ny + 1, device=dev, dtype=torch.float64)) ** 2).sum())
    u = float(u)
    k, N = nx * ny, nx + ny
    t = u / (k * N) - (4 * k - 1) / (6 * N)
    et = (1 + 1 / N) / 6
    vt = (N + 1) * (4 * k * N - 3 * (nx ** 2 + ny ** 2) - 2 * k) / (45 * N ** 2 * 4 * k)
    tn = 1 / 6 + (t - et) / math.sqrt(45 * vt)
    if tn < 0.003:
        return t, 1.0
    from scipy.stats._hypotests import _cdf_cvm_inf
    return t, max(0.0, 1.0 - float(_cdf_cvm_inf(tn)))


def anderson_ksamp(*samples) -> tuple[float, list[float], float]:
    """(standardised A2, critical values, significance level) as scipy.stats.anderson_ksamp
    (midrank variant, Scholz & Stephens 1987).  The A2akN sum runs on the samples' device: one sort of
    the pooled sample, its distinct values, and per sample one sort and two searchsorted passes; the
    normalisation and the p-value interpolation are host formulas on N and k."""
    import warnings

    import numpy as np
    xs = [_dev(s) for s in samples]
    k = len(xs)
    if k < 2:
        raise ValueError("anderson_ksamp needs at least two samples")
    dev = xs[0].device
    xs = [s.to(dev) for s in xs]
    n = [s.numel() for s in xs]
    if min(n) == 0:
        raise ValueError("anderson_ksamp encountered sample without observations")
    Z = torch.sort(torch.cat(xs)).values
    N = Z.numel()
    Zs = torch.unique_consecutive(Z)
    if Zs.numel() < 2:
        raise ValueError("anderson_ksamp needs more than one distinct observation")
    left = torch.searchsorted(Z, Zs, right=False).double()
    lj = torch.searchsorted(Z, Zs, right=True).double() - left
    Bj = left + lj / 2.0
    den = Bj * (N - Bj) - N * lj / 4.0
    a2 = torch.zeros((), dtype=torch.float64, device=dev)
    for s, ni in zip(xs, n):
        ss = torch.sort(s).values
        r = torch.searchsorted(ss, Zs, right=True).double()
        f = r - torch.searchsorted(ss, Zs, right=False).double()
        M = r - f / 2.0
        a2 = a2 + (lj / N * (N * M - Bj * ni) ** 2 / den).sum() / ni
    A2kN = float(a2) * (N - 1.0) / N
    # normalisation (scipy.stats.anderson_ksamp)
    H = sum(1.0 / v for v in n)
    hs_cs = np.cumsum(1.0 / np.arange(N - 1, 1, -1))
    h = hs_cs[-1] + 1
    g = (hs_cs / np.arange(2, N)).sum()
    a = (4 * g - 6) * (k - 1) + (10 - 6 * g) * H
    b = (2 * g - 4) * k ** 2 + 8 * h * k + (2 * g - 14 * h - 4) * H - 8 * h + 4 * g - 6
    c = (6 * h + 2 * g - 2) * k ** 2 + (4 * h - 4 * g + 6) * k + (2 * h - 6) * H + 4 * h
    d = (2 * h + 6) * k ** 2 - 4 * h * k
    sigmasq = (a * N ** 3 + b * N ** 2 + c * N + d) / ((N - 1.0) * (N - 2.0) * (N - 3.0))
    m = k - 1
    A2 = (A2kN - m) / math.sqrt(sigmasq)
    b0 = np.array([0.675, 1.281, 1.645, 1.96, 2.326, 2.573, 3.085])
    b1 = np.array([-0.245, 0.25, 0.678, 1.149, 1.822, 2.364, 3.615])
    b2 = np.array([-0.105, -0.305, -0.362, -0.391, -0.396, -0.345, -0.154])
    critical = b0 + b1 / math.sqrt(m) + b2 / m
    sig = np.array([0.25, 0.1, 0.05, 0.025, 0.01, 0.005, 0.001])
    if A2 < critical.min():
        p = float(sig.max())
        warnings.warn(f"p-value capped: true value larger than {p}.", stacklevel=2)
    elif A2 > critical.max():
        p = float(sig.min())
        warnings.warn(f"p-value floored: true value smaller than {p}.", stacklevel=2)
    else:
        pf = np.polyfit(critical, np.log(sig), 2)
        p = float(math.exp(np.polyval(pf, A2)))
    return float(A2), critical.tolist(), p
