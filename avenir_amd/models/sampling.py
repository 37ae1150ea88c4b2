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


def smote(X: torch.Tensor, y: torch.Tensor, minority: int, n_new: int, k: int = 5, seed: int = 0,
          cat_cols: torch.Tensor | None = None, pick: str = "uniform") -> tuple[torch.Tensor, torch.Tensor]:
    """Return (new_X [n_new, D], new_cat [n_new, Fc] or None) for the minority class."""
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    idx = torch.nonzero(y == minority).squeeze(1)
    Xm = X[idx].float()
    _, nb = dist.knn(Xm, Xm, min(k, max(1, Xm.shape[0] - 1)), "euclidean", exclude_self=True)
    src = torch.randint(0, Xm.shape[0], (n_new,), generator=g).to(X.device)
    col = torch.randint(0, nb.shape[1], (n_new,), generator=g).to(X.device)
    nbr = nb[src, col].clamp_min(0)
    gap = torch.rand((n_new, 1), generator=g).to(X.device)
    newX = Xm[src] + gap * (Xm[nbr] - Xm[src])
    newC = None
    if cat_cols is not None:
        Cm = cat_cols[idx]
        if pick == "exponential":
            u = torch.rand(n_new, generator=g).to(X.device)
            take_src = (-torch.log(u.clamp_min(1e-12))) < 1.0
        else:
            take_src = torch.rand(n_new, generator=g).to(X.device) < 0.5
        newC = torch.where(take_src.unsqueeze(1), Cm[src], Cm[nbr])
    return newX, newC


def undersample(y: torch.Tensor, seed: int = 0, comm: Comm | None = None) -> torch.Tensor:
    """Boolean keep-mask balancing classes down to the minority count (global counts)."""
    comm = comm or get_comm()
    C = int(y.max()) + 1 if y.numel() else 1
    cnt = torch.bincount(y.long(), minlength=C).double()
    if comm.is_distributed:
        C2 = torch.tensor([float(C)], device=cnt.device)
        comm.all_reduce(C2, "max")
        if int(C2) > C:
            cnt = torch.cat([cnt, torch.zeros(int(C2) - C, dtype=cnt.dtype, device=cnt.device)])
        comm.all_reduce(cnt)
    minc = float(cnt[cnt > 0].min())
    keep_p = (minc / cnt.clamp_min(1))[y.long()]
    g = torch.Generator(device="cpu")
    g.manual_seed(seed + 7919 * comm.rank)
    return torch.rand(y.shape[0], generator=g).to(y.device) < keep_p


def bagging_indices(n: int, batch_size: int | None = None, seed: int = 0) -> torch.Tensor:
    """Bootstrap indices (with replacement) drawn within consecutive batches."""
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    bs = batch_size or n
    out = []
    for s in range(0, n, bs):
        m = min(bs, n - s)
        out.append(s + torch.randint(0, m, (m,), generator=g))
    return torch.cat(out) if out else torch.zeros(0, dtype=torch.long)


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
    """Relief feature relevance [D]: sum over records of (miss diff - hit diff) / n, diffs normalised
    by the attribute range.  With row shards on several ranks the neighbours are searched over ALL
    ranks' records (one all-gather of the shard, as TopMatchesByClass joins every pair) and the
    ranges are global, so the score equals the single-process one."""
    comm = comm or get_comm()
    X = X.float()
    dist_mode = comm.is_distributed
    if dist_mode:
        dev = comm.device if comm.backend == "nccl" else torch.device("cpu")
        Xa = comm.all_gather_v(X.to(dev)).to(X.device)
        ya = comm.all_gather_v(y.to(dev).long()).to(X.device)
        sizes = comm.all_gather(torch.tensor([X.shape[0]], dtype=torch.long, device=dev)).view(-1).tolist()
        base = int(sum(sizes[:comm.rank]))
    else:
        Xa, ya, base = X, y, 0
    rng = (Xa.max(0).values - Xa.min(0).values) if ranges is None else ranges.float().to(X.device)
    rng = rng.clamp_min(1e-12)
    if dist_mode:
        hit, miss = _global_matches(X, y.long(), Xa, ya, base, k)
    else:
        _, hit = top_matches_by_class(X, y, k, same_class=True)
        _, miss = top_matches_by_class(X, y, k, same_class=False)
    score = torch.zeros(X.shape[1], dtype=torch.float64, device=X.device)
    for j in range(k):
        h, m = hit[:, j], miss[:, j]
        okh, okm = h >= 0, m >= 0
        score -= ((X[okh] - Xa[h[okh]]).abs() / rng).double().sum(0)
        score += ((X[okm] - Xa[m[okm]]).abs() / rng).double().sum(0)
    n = torch.tensor([float(X.shape[0] * k)], dtype=torch.float64, device=X.device)
    if dist_mode:
        comm.all_reduce(score)
        comm.all_reduce(n)
    return (score / n).float()


def _global_matches(X, y, Xa, ya, base: int, k: int):
    """Nearest same-class (hits, self excluded by global id) and other-class (misses) records of
    this rank's rows among all records: global row ids [n, k] (-1 when fewer)."""
    from ..ops import distance as dist
    n = X.shape[0]
    hit = torch.full((n, k), -1, dtype=torch.long, device=X.device)
    miss = torch.full((n, k), -1, dtype=torch.long, device=X.device)
    for c in torch.unique(ya).tolist():
        qi = torch.nonzero(y == c).squeeze(1)
        if qi.numel() == 0:
            continue
        ri = torch.nonzero(ya == c).squeeze(1)
        if ri.numel():
            _, i = dist.knn(X[qi], Xa[ri], min(k + 1, ri.numel()))
            gi = torch.where(i >= 0, ri[i.clamp_min(0)], i)
            keep = (gi != (qi + base).view(-1, 1)) & (gi >= 0)                  # drop self
            slot = keep.long().cumsum(1) - 1
            rr, cc = torch.nonzero(keep & (slot < k), as_tuple=True)
            hit[qi[rr], slot[rr, cc]] = gi[rr, cc]
        ro = torch.nonzero(ya != c).squeeze(1)
        if ro.numel():
            _, i = dist.knn(X[qi], Xa[ro], k)
            miss[qi] = torch.where(i >= 0, ro[i.clamp_min(0)], i)
    return hit, miss
