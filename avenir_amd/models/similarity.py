"""Record similarity family (Spark ``S/similarity/*``, MR ``J/explore/TopMatchesByClass``).

* ``RecordSimilarity`` — all pairs within one dataset or between two (reference: bucket-pair
  replication + groupByKey, ``RecordSimilarity.scala:80-188``); here a tiled MFMA distance kernel
  with fused top-k, or the full matrix when every pair is wanted.
* ``GroupedRecordSimilarity`` — pairwise distances within each key group (``:59-80``).
* ``NearestRecords`` — per record the top-k (by count or distance threshold) (``:97-125``).
* ``TopMatchesByClass`` — same-class (or other-class) top-N neighbours for Relief / SMOTE
  (``J/explore/TopMatchesByClass.java:133-399``).
"""
from __future__ import annotations

import math

import torch

from ..ops import distance as dist


class RecordSimilarity:
    def __init__(self, metric: str = "euclidean", scale: float = 1.0):
        self.metric = metric
        self.scale = scale

    def all_pairs(self, A: torch.Tensor, B: torch.Tensor | None = None, chunk: int = 8192):
        """Yield (i, j, distance) triples as tensors, chunked (upper triangle when B is None)."""
        same = B is None
        B = A if same else B
        for s in range(0, A.shape[0], chunk):
            d = dist.pairwise(A[s:s + chunk], B, self.metric) * self.scale
            ii = torch.arange(s, s + d.shape[0], device=d.device).view(-1, 1).expand_as(d)
            jj = torch.arange(B.shape[0], device=d.device).view(1, -1).expand_as(d)
            m = (jj > ii) if same else torch.ones_like(d, dtype=torch.bool)
            yield ii[m], jj[m], d[m]

    def top_k(self, A: torch.Tensor, B: torch.Tensor | None = None, k: int = 5):
        same = B is None
        return dist.knn(A, A if same else B, k, self.metric, exclude_self=same)


class NearestRecords:
    def __init__(self, k: int = 5, metric: str = "euclidean", max_distance: float | None = None):
        self.k, self.metric, self.max_distance = k, metric, max_distance

    def __call__(self, A: torch.Tensor, B: torch.Tensor | None = None):
        d, i = dist.knn(A, A if B is None else B, self.k, self.metric, exclude_self=B is None)
        if self.max_distance is not None:
            far = d > self.max_distance
            d = torch.where(far, torch.full_like(d, math.inf), d)
            i = torch.where(far, torch.full_like(i, -1), i)
        return d, i


class GroupedRecordSimilarity:
    def __init__(self, metric: str = "euclidean"):
        self.metric = metric

    def __call__(self, X: torch.Tensor, groups: torch.Tensor) -> dict[int, torch.Tensor]:
        """Full distance matrix per group id."""
        out = {}
        for g in torch.unique(groups).tolist():
            idx = torch.nonzero(groups == g).squeeze(1)
            out[g] = dist.pairwise(X[idx], X[idx], self.metric)
        return out


def top_matches_by_class(X: torch.Tensor, y: torch.Tensor, k: int, same_class: bool = True,
                         metric: str = "euclidean"):
    """For every record, the k nearest records of the same class (or of the other classes):
    (dist [n, k], idx [n, k] global)."""
    n = X.shape[0]
    out_d = torch.full((n, k), math.inf, device=X.device)
    out_i = torch.full((n, k), -1, dtype=torch.long, device=X.device)
    for c in torch.unique(y).tolist():
        qi = torch.nonzero(y == c).squeeze(1)
        ri = qi if same_class else torch.nonzero(y != c).squeeze(1)
        if ri.numel() == 0 or qi.numel() == 0:
            continue
        d, i = dist.knn(X[qi], X[ri], k, metric, exclude_self=same_class)
        gi = torch.where(i >= 0, ri[i.clamp_min(0)], i)
        out_d[qi], out_i[qi] = d, gi
    return out_d, out_i
