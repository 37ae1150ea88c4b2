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


def kendall_counts(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """int64 [5]: concordant, discordant, tied in x only, tied in y only, tied in both (pairs i < j)."""
    x, y = _dev(x), _dev(y).to(_dev(x).device)
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
    method auto: exact for tie-free samples of <= 8 values each)."""
    from scipy import stats
    a, b = _dev(a), _dev(b).to(_dev(a).device)
    n1, n2 = a.numel(), b.numel()
    z_all = torch.cat([a, b])
    grp = torch.cat([torch.zeros(n1, dtype=torch.int32), torch.ones(n2, dtype=torch.int32)]).to(z_all.device)
    _, tie, gs = rank_avg(z_all, grp, 2)
    r1 = float(gs[0])
    u1 = r1 - n1 * (n1 + 1) / 2.0
    t3 = float(tie[0])
    if n1 <= 8 and n2 <= 8 and t3 == 0:
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
