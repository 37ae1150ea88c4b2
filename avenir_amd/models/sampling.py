"""Re-sampling, boosting and feature-relevance utilities (``J/explore``, ``S/explore``).

* ``smote`` — ClassBasedOverSampler: synthetic minority records interpolated between a record and
  one of its same-class neighbours; categorical attributes copied from either side with uniform or
  exponentially distributed pick (``J/explore/ClassBasedOverSampler.java:125-200``).
* ``undersample`` — UnderSamplingBalancer: keep majority-class records with probability
  minCount/count (``J/explore/UnderSamplingBalancer.java:95-166``).
* ``bagging_indices`` — BaggingSampler: bootstrap within batches (``J/explore/BaggingSampler.java``).
* ``AdaBoost`` — weighted error and weight update, alpha = 1/2 ln((1-e)/e), reset when e >= 0.5
  (``J/explore/AdaBoostError.java``, ``AdaBoostUpdate.java``).
* ``relief`` — Relief scores from neighbourhoods: hits lower, misses raise the score, numeric diffs
  normalised by range (``J/explore/ReliefFeatureRelevance.java``, ``S/explore/FeatureRelevanceByRelief``).
"""
from __future__ import annotations

import math

import torch

from ..ops import distance as dist
from ..parallel.comm import Comm, get_comm
from .similarity import top_matches_by_class


def _row_base(n: int, comm) -> tuple[int, list[int]]:
    """(global index of this rank's first row, every rank's row count)."""
    if comm is None or not comm.is_distributed:
        return 0, [n]
    sizes = [int(x) for x in comm.all_gather_object(int(n))]
    return sum(sizes[: comm.rank]), sizes


def smote(X: torch.Tensor, y: torch.Tensor, minority: int, n_new: int, k: int = 5, seed: int = 0,
          cat_cols: torch.Tensor | None = None, pick: str = "uniform", exp_mean: float = 1.0,
          comm: Comm | None = None) -> tuple[torch.Tensor, torch.Tensor | None]:
    """SMOTE over this rank's rows (ClassBasedOverSampler, J/explore/ClassBasedOverSampler.java:
    125-200): ``n_new`` synthetic minority records over ALL ranks.  Minority record g (global order)
    seeds ``n_new // m + (g < n_new % m)`` synthetic records; its k same-class neighbours are found
    among every rank's minority records (distributed_knn ring, no all-gather of X) and their rows
    fetched by id; pick / gap / categorical coin come from the K25 kernel's Philox draws keyed by
    (seed, record, copy).  The rank-ordered concatenation of the outputs does not depend on the world
    size.  Returns (new_X [*, D], new_cat [*, Fc] or None)."""
    from ..ops import resample_ops as RS
    comm = comm or get_comm()
    dist_mode = comm.is_distributed
    idx = torch.nonzero(y == minority).squeeze(1)
    Xm = X[idx].float().contiguous()
    m_loc = Xm.shape[0]
    gbase, sizes = _row_base(m_loc, comm if dist_mode else None)
    m = sum(sizes)
    D = X.shape[1]
    if m == 0 or n_new <= 0:
        return X.new_zeros((0, D)).float(), (None if cat_cols is None else cat_cols.new_zeros((0, cat_cols.shape[1])))
    kk = max(1, min(k, m - 1))
    gid = torch.arange(gbase, gbase + m_loc, device=X.device)
    _, nb = dist.distributed_knn(Xm, Xm, kk + 1, comm if dist_mode else _SelfComm(), r_ids=gid)
    keep = (nb != gid.view(-1, 1)) & (nb >= 0)                              # drop self
    slot = keep.long().cumsum(1) - 1
    nbk = torch.full((m_loc, kk), -1, dtype=torch.long, device=X.device)
    rr, cc = torch.nonzero(keep & (slot < kk), as_tuple=True)
    nbk[rr, slot[rr, cc]] = nb[rr, cc]
    nn = (nbk >= 0).sum(1).int()
    tables = [Xm] + ([cat_cols[idx].int().contiguous()] if cat_cols is not None else [])
    if dist_mode:
        fetched = comm.fetch_rows(nbk.view(-1), tables, gbase, sizes)
    else:
        fetched = [t[nbk.view(-1).clamp_min(0)] for t in tables]
    Xn = fetched[0].view(m_loc, kk, D).contiguous()
    Cs = Cn = None
    if cat_cols is not None:
        Cs = tables[1]
        Cn = fetched[1].view(m_loc, kk, -1).contiguous()
    mult = -(-n_new // m)
    newX, newC, _ = RS.smote_rows(Xm, Xn, nn, Cs, Cn, mult, gbase, seed, pick == "exponential", exp_mean)
    # record g keeps copies j < n_new // m + (g < n_new % m)
    gi = torch.arange(gbase, gbase + m_loc, device=newX.device).repeat_interleave(mult)
    j = torch.arange(mult, device=newX.device).repeat(m_loc)
    take = j < (n_new // m + (gi < n_new % m).long())
    return newX[take], (newC[take] if cat_cols is not None else None)


class _SelfComm:
    is_distributed = False
    world = 1
    rank = 0


def undersample(y: torch.Tensor, seed: int = 0, comm: Comm | None = None) -> torch.Tensor:
    """Boolean keep-mask balancing classes down to the minority count: record g of class c is kept
    when u(seed, g) < min_count / count_c (global counts; K25 Philox keyed by the GLOBAL record
    index, so the mask does not depend on the world size)."""
    from ..ops import resample_ops as RS
    comm = comm or get_comm()
    C = int(y.max()) + 1 if y.numel() else 1
    cnt = torch.bincount(y.long(), minlength=C).double()
    if comm.is_distributed:
        C2 = torch.tensor([float(C)], device=cnt.device)
        comm.all_reduce(C2, "max")
        if int(C2) > C:
            cnt = torch.cat([cnt, torch.zeros(int(C2) - C, dtype=cnt.dtype, device=cnt.device)])
        comm.all_reduce(cnt)
    base, _ = _row_base(y.shape[0], comm)
    minc = float(cnt[cnt > 0].min()) if bool((cnt > 0).any()) else 0.0
    keep_p = (minc / cnt.clamp_min(1))[y.long()].float()
    u = RS.uniform(seed, RS.STREAM_UNDERSAMPLE, base, y.shape[0], y.device).to(y.device)
    return u <= keep_p


def bagging_indices(n: int, batch_size: int | None = None, seed: int = 0, base: int = 0,
                    total: int | None = None, device="cpu") -> torch.Tensor:
    """Bootstrap positions (with replacement) drawn within consecutive batches of the GLOBAL record
    order (BaggingSampler, J/explore/BaggingSampler.java:117-122): output slot g of batch
    [b0, b1) takes record b0 + floor(u(seed, g) * (b1 - b0)).  Slots [base, base + n) of ``total``
    records; returns GLOBAL record ids (a rank fetches the ones it does not hold)."""
    from ..ops import resample_ops as RS
    total = n if total is None else total
    bs = batch_size or total
    dev = torch.device(device)
    g = torch.arange(base, base + n, dtype=torch.long, device=dev)
    b0 = (g // bs) * bs
    b1 = torch.clamp(b0 + bs, max=total)
    # the draws on the target device (resample_uniform_kernel: the same Philox values as the host
    # twin; the numpy twin took ~0.1 s of a 2^21-record job)
    u = RS.uniform(seed, RS.STREAM_BAGGING, base, n, dev).double()
    return b0 + torch.minimum((u * (b1 - b0).double()).long(), (b1 - b0 - 1).clamp_min(0))


class AdaBoost:
    def __init__(self, comm: Comm | None = None):
        self.comm = comm

    def error(self, pred: torch.Tensor, actual: torch.Tensor, weight: torch.Tensor) -> float:
        w = weight.double()
        num = (w * (pred != actual).double()).sum().view(1)
        den = w.sum().view(1)
        comm = self.comm or get_comm()
        if comm.is_distributed:
            comm.all_reduce(num)
            comm.all_reduce(den)
        return float(num / den)

    @staticmethod
    def alpha(err: float) -> float:
        err = min(max(err, 1e-12), 1 - 1e-12)
        return 0.5 * math.log((1 - err) / err)

    def update(self, pred: torch.Tensor, actual: torch.Tensor, weight: torch.Tensor, err: float) -> torch.Tensor:
        if err >= 0.5:
            return torch.ones_like(weight) / weight.numel()
        a = self.alpha(err)
        wrong = (pred != actual).to(weight.dtype)
        return weight * torch.exp(a * (2 * wrong - 1))


def relief(X: torch.Tensor, y: torch.Tensor, k: int = 1, ranges: torch.Tensor | None = None,
           comm: Comm | None = None) -> torch.Tensor:
    """Relief feature relevance [D]: sum over records of (miss diff - hit diff) / (n k), diffs
    normalised by the attribute range (J/explore/ReliefFeatureRelevance.java:119-232).  Sharded:
    the hits (nearest same-class, self excluded) and misses (nearest other-class) of this rank's
    rows are searched over ALL ranks' records by the distributed_knn ring (class subsets travel
    with their global ids), the neighbour rows are fetched by id with two all-to-alls, and the
    ranges are one min / max all-reduce — no rank ever holds more than its shard plus n*k fetched
    rows (the previous design all-gathered X)."""
    comm = comm or get_comm()
    X = X.float().contiguous()
    y = y.long()
    dist_mode = comm.is_distributed
    cm = comm if dist_mode else _SelfComm()
    base, sizes = _row_base(X.shape[0], comm if dist_mode else None)
    if ranges is None:
        lo = X.min(0).values if X.shape[0] else torch.full((X.shape[1],), float("inf"), device=X.device)
        hi = X.max(0).values if X.shape[0] else torch.full((X.shape[1],), float("-inf"), device=X.device)
        if dist_mode:
            comm.all_reduce(lo, "min")
            comm.all_reduce(hi, "max")
        rng = hi - lo
    else:
        rng = ranges.float().to(X.device)
    rng = rng.clamp_min(1e-12)
    C = torch.tensor([float(int(y.max()) + 1 if y.numel() else 0)], device=X.device)
    if dist_mode:
        comm.all_reduce(C, "max")
    n = X.shape[0]
    gid = torch.arange(base, base + n, device=X.device)
    hit = torch.full((n, k), -1, dtype=torch.long, device=X.device)
    miss = torch.full((n, k), -1, dtype=torch.long, device=X.device)
    for c in range(int(C.item())):          # every rank walks the same classes (collective ring)
        qi = torch.nonzero(y == c).squeeze(1)
        oi = torch.nonzero(y != c).squeeze(1)
        _, hh = dist.distributed_knn(X[qi], X[qi], k + 1, cm, r_ids=gid[qi])
        keep = (hh != gid[qi].view(-1, 1)) & (hh >= 0)
        slot = keep.long().cumsum(1) - 1
        rr, cc = torch.nonzero(keep & (slot < k), as_tuple=True)
        hit[qi[rr], slot[rr, cc]] = hh[rr, cc]
        _, mm = dist.distributed_knn(X[qi], X[oi], k, cm, r_ids=gid[oi])
        miss[qi] = mm
    if dist_mode:
        Xh, Xmiss = (comm.fetch_rows(hit.view(-1), [X], base, sizes)[0].view(n, k, -1),
                     comm.fetch_rows(miss.view(-1), [X], base, sizes)[0].view(n, k, -1))
    else:
        Xh, Xmiss = X[hit.clamp_min(0)], X[miss.clamp_min(0)]
    dh = ((X.unsqueeze(1) - Xh).abs() / rng).double() * (hit >= 0).unsqueeze(2)
    dm = ((X.unsqueeze(1) - Xmiss).abs() / rng).double() * (miss >= 0).unsqueeze(2)
    score = (dm.sum((0, 1)) - dh.sum((0, 1)))
    cnt = torch.tensor([float(n * k)], dtype=torch.float64, device=X.device)
    if dist_mode:
        comm.all_reduce(score)
        comm.all_reduce(cnt)
    return (score / cnt).float()
