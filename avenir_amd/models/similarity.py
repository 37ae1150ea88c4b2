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
    """Pairwise distances within each key group, all groups at once: records are sorted by group,
    groups are bucketed by size (powers of two) and each bucket is ONE batched distance launch over
    a zero-padded [groups, L, D] block — no per-group loop, whatever the number of groups."""

    def __init__(self, metric: str = "euclidean"):
        self.metric = metric

    def pairs(self, X: torch.Tensor, groups: torch.Tensor):
        """Every within-group pair i < j (original row indices): (i, j, distance) tensors, ordered
        by group then (i, j)."""
        n = X.shape[0]
        dev = X.device
        groups = groups.to(dev)
        order = torch.argsort(groups, stable=True)
        g_sorted = groups[order]
        _, counts = torch.unique_consecutive(g_sorted, return_counts=True)
        starts = torch.cumsum(counts, 0) - counts
        cnt_h = counts.cpu()
        out_i, out_j, out_d, out_key = [], [], [], []
        G = int(cnt_h.numel())
        if n == 0 or G == 0:
            e = torch.zeros(0, dtype=torch.long, device=dev)
            return e, e, torch.zeros(0, device=dev)
        lvl = torch.ceil(torch.log2(cnt_h.clamp_min(1).double())).long()
        for L2 in torch.unique(lvl).tolist():
            gsel = torch.nonzero(lvl == L2).view(-1)
            L = 1 << int(L2)
            if L < 2:
                continue                                           # singleton groups: no pairs
            gd = gsel.to(dev)
            pos = torch.arange(L, device=dev)
            valid = pos.view(1, -1) < counts[gd].view(-1, 1)          # [Gb, L]
            src = (starts[gd].view(-1, 1) + pos.view(1, -1)).clamp_max(n - 1)
            rows = order[src]                                         # [Gb, L] original row ids
            B = X[rows] * valid.unsqueeze(-1)
            Dm = self._batched(B)                                     # [Gb, L, L]
            ii, jj = torch.triu_indices(L, L, 1, device=dev)
            ok = valid[:, ii] & valid[:, jj]                          # [Gb, P]
            gb, pidx = torch.nonzero(ok, as_tuple=True)
            out_i.append(rows[gb, ii[pidx]])
            out_j.append(rows[gb, jj[pidx]])
            out_d.append(Dm[gb, ii[pidx], jj[pidx]])
            out_key.append(gd[gb] * (n + 1) + starts[gd[gb]])         # stable group order
        if not out_i:
            e = torch.zeros(0, dtype=torch.long, device=dev)
            return e, e, torch.zeros(0, device=dev)
        i, j, d, key = torch.cat(out_i), torch.cat(out_j), torch.cat(out_d), torch.cat(out_key)
        # group order, then (i, j) in the group's sorted-row order
        rank = torch.empty(n, dtype=torch.long, device=dev)
        rank[order] = torch.arange(n, device=dev)
        o = torch.argsort(rank[i] * (n + 1) + rank[j])
        return i[o], j[o], d[o]

    def _batched(self, B: torch.Tensor) -> torch.Tensor:
        if self.metric in ("euclidean", "sqeuclidean"):
            d = torch.cdist(B, B)
            return d * d if self.metric == "sqeuclidean" else d
        if self.metric == "manhattan":
            return torch.cdist(B, B, p=1)
        if self.metric == "cosine":
            nb = torch.nn.functional.normalize(B, dim=-1)
            return 1 - nb @ nb.transpose(1, 2)
        raise ValueError(f"unknown metric {self.metric}")

    def __call__(self, X: torch.Tensor, groups: torch.Tensor) -> dict[int, torch.Tensor]:
        """Full distance matrix per group id (small outputs; ``pairs`` is the bulk path)."""
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
