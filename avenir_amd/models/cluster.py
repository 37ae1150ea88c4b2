"""Clustering: batched / distributed k-means (+ k-means++ and knuckle selection), agglomerative
graphical clustering, DBSCAN, Hopkins statistic.

Reference: ``J/cluster/KmeansCluster.java`` (one MR job per Lloyd iteration over many cluster
groups: mapper finds the nearest centroid with the mixed-type record distance, reducer recomputes
numeric means + categorical modes, movement / status / SSE, :57-297), ``S/cluster/KmeansCluster.scala``
(many (k, init-group) runs, min-SSE run per k, knuckle k by the max second difference of SSE,
:103-172), ``S/cluster/KMeansPlusPlusCluster.scala`` (commons-math k-means++), ``P/unsupv/cluster.py``
(sklearn kmeans / agglomerative / dbscan, Hopkins statistic), ``J/cluster/AgglomerativeGraphical.java``.

MI355X: assignment is the k = 1 case of the fused MFMA distance + top-k kernel, the update is one
LDS-privatised accumulation kernel, and ONE all-reduce of [K, D] sums + [K] counts per iteration
replaces the shuffle; the convergence test runs on device.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch

from .. import _native
from ..ops import distance as dist
from ..parallel.comm import Comm, get_comm


@dataclass
class KMeansRun:
    k: int
    seed: int
    centroids: torch.Tensor
    sse: float = math.inf
    iterations: int = 0
    counts: torch.Tensor | None = None
    converged: bool = False
    history: list = field(default_factory=list)


class KMeans:
    def __init__(self, n_clusters: int | list[int] = 3, n_init: int = 1, max_iter: int = 300,
                 tol: float = 1e-4, init: str = "k-means++", seed: int = 0, comm: Comm | None = None):
        self.ks = [n_clusters] if isinstance(n_clusters, int) else list(n_clusters)
        self.n_init = n_init
        self.max_iter = max_iter
        self.tol = tol
        self.init = init
        self.seed = seed
        self.comm = comm
        self.runs: list[KMeansRun] = []
        self.best: dict[int, KMeansRun] = {}

    # ------------------------------------------------------------------------------------------
    def _init_centroids(self, X: torch.Tensor, k: int, seed: int) -> torch.Tensor:
        """k-means++ (D^2 sampling) on a gathered sample; identical on every rank (broadcast)."""
        comm = self.comm or get_comm()
        g = torch.Generator(device="cpu")
        g.manual_seed(seed)
        # sample up to 64k points overall for seeding
        m = min(X.shape[0], max(1, 65536 // max(comm.world, 1)))
        # sample without a full permutation of the data (O(m), not O(n)); duplicates are harmless
        sel = (torch.randperm(X.shape[0], generator=g)[:m] if X.shape[0] <= 4 * m
               else torch.randint(0, X.shape[0], (m,), generator=g)).to(X.device)
        S = X[sel].float()
        if comm.is_distributed:
            S = comm.all_gather_v(S)
        if self.init == "random":
            C = S[torch.randperm(S.shape[0], generator=g)[:k].to(S.device)]
        else:
            first = int(torch.randint(0, S.shape[0], (1,), generator=g))
            C = S[first:first + 1]
            d2 = ((S - C) ** 2).sum(1)
            for _ in range(1, k):
                p = (d2 / d2.sum().clamp_min(1e-30)).double().cpu()
                nxt = int(torch.multinomial(p, 1, generator=g)) if float(p.sum()) > 0 else 0
                C = torch.cat([C, S[nxt:nxt + 1]])
                d2 = torch.minimum(d2, ((S - S[nxt]) ** 2).sum(1))
        if comm.is_distributed:
            C = comm.broadcast(C.contiguous(), 0)
        return C.contiguous()

    def _step(self, X: torch.Tensor, Xp: torch.Tensor | None, Cs: list[torch.Tensor]):
        """One Lloyd pass for a GROUP of runs -> per run (sums f64 [k, D], counts [k], sse f64 [1]).
        GPU: ONE launch of the fused K16 kernel for all runs (data read once); CPU: oracle."""
        if Xp is not None:
            D = X.shape[1]
            ks = [c.shape[0] for c in Cs]
            Cp = torch.zeros((sum(ks), Xp.shape[1]), dtype=torch.float32, device=X.device)
            Cp[:, :D] = torch.cat(Cs)
            sums, counts, sse, _ = _native.C().kmeans_step(Xp, Cp.contiguous(), ks, False)
            out, o = [], 0
            for r, k in enumerate(ks):
                out.append((sums[o:o + k, :D].contiguous(), counts[o:o + k].round().long(), sse[r:r + 1]))
                o += k
            return out
        res = []
        for C in Cs:
            d, idx = dist.knn(X, C, 1, "sqeuclidean")
            sums, counts = dist.cluster_accumulate(X, idx[:, 0].int(), C.shape[0])
            res.append((sums, counts, d[:, 0].double().sum().view(1)))
        return res

    @staticmethod
    def _padded(X: torch.Tensor) -> torch.Tensor | None:
        if not X.is_cuda or not _native.available():
            return None
        D = X.shape[1]
        Dp = next((p for p in (2, 4, 8, 16, 32, 64) if p >= D), None)
        if Dp is None:
            return None
        if Dp == D:
            return X
        Xp = torch.zeros((X.shape[0], Dp), dtype=torch.float32, device=X.device)
        Xp[:, :D] = X
        return Xp

    def _groups(self, specs: list[tuple[int, int]], Dp: int | None) -> list[list[int]]:
        """Pack runs into launch groups: <= 16 runs and total centroids within the LDS budget."""
        groups, cur, tot = [], [], 0
        cap = (64 * 1024) // (4 * (2 * Dp + 2)) if Dp else 1 << 30
        for i, (k, _) in enumerate(specs):
            if Dp is not None and k > cap:
                raise ValueError(f"k={k} too large for the LDS-resident k-means kernel at D={Dp}")
            if cur and (len(cur) == 16 or tot + k > cap or Dp is None):
                groups.append(cur)
                cur, tot = [], 0
            cur.append(i)
            tot += k
        if cur:
            groups.append(cur)
        return groups

    def fit(self, X: torch.Tensor) -> "KMeans":
        """All (k, init) runs advance together (S/cluster/KmeansCluster.scala keys by
        (numClusters, initGroup)): one kernel launch per iteration per group of runs."""
        comm = self.comm or get_comm()
        X = X.float().contiguous()
        Xp = self._padded(X)
        specs = [(k, self.seed * 1009 + k * 31 + r) for k in self.ks for r in range(self.n_init)]
        runs = [KMeansRun(k, sd, self._init_centroids(X, k, sd)) for k, sd in specs]
        self.best = {}
        for grp in self._groups(specs, Xp.shape[1] if Xp is not None else None):
            active = list(grp)
            for it in range(self.max_iter):
                res = self._step(X, Xp, [runs[i].centroids for i in active])
                if comm.is_distributed:
                    flat = torch.cat([torch.cat([s.view(-1), c.double().view(-1), e]) for s, c, e in res])
                    flat = comm.all_reduce(flat)
                    o, red = 0, []
                    for s, c, e in res:
                        a, b = s.numel(), c.numel()
                        red.append((flat[o:o + a].view_as(s), flat[o + a:o + a + b].round().long(),
                                    flat[o + a + b:o + a + b + 1]))
                        o += a + b + 1
                    res = red
                moves = []
                for i, (sums, counts, sse) in zip(active, res):
                    C = runs[i].centroids
                    newC = torch.where(counts.view(-1, 1) > 0, sums / counts.clamp_min(1).view(-1, 1),
                                       C.double()).float()
                    moves.append(((newC - C) ** 2).sum(1).sqrt().max())
                    runs[i].centroids = newC
                    runs[i].history.append(sse)
                    runs[i].iterations = it + 1
                mv = torch.stack(moves).cpu().tolist()          # one host sync per iteration per group
                still = []
                for i, m in zip(active, mv):
                    if m <= self.tol:
                        runs[i].converged = True
                    else:
                        still.append(i)
                active = still
                if not active:
                    break
            final = self._step(X, Xp, [runs[i].centroids for i in grp])
            for i, (sums, counts, sse) in zip(grp, final):
                if comm.is_distributed:
                    sse = comm.all_reduce(sse)
                    counts = comm.all_reduce(counts)
                runs[i].sse, runs[i].counts = float(sse), counts
                runs[i].history = [float(h) for h in runs[i].history]
        self.runs = runs
        for r in runs:
            if r.k not in self.best or r.sse < self.best[r.k].sse:
                self.best[r.k] = r
        return self

    @property
    def cluster_centers_(self) -> torch.Tensor:
        return self.best[self.ks[0]].centroids

    def predict(self, X: torch.Tensor, k: int | None = None) -> torch.Tensor:
        C = self.best[k or self.ks[0]].centroids
        return dist.knn(X.float(), C.to(X.device), 1, "sqeuclidean")[1][:, 0]

    def knuckle_k(self) -> int:
        """k at the maximum second difference of min-SSE vs k (MathUtils.getMaxSecondDiff)."""
        ks = sorted(self.best)
        if len(ks) < 3:
            return ks[0]
        sse = [self.best[k].sse for k in ks]
        best, arg = -math.inf, ks[1]
        for i in range(1, len(ks) - 1):
            sd = sse[i - 1] - 2 * sse[i] + sse[i + 1]
            if sd > best:
                best, arg = sd, ks[i]
        return arg


def categorical_modes(codes: torch.Tensor, n: int, bins: list[int], assign: torch.Tensor, k: int,
                      comm: Comm | None = None) -> torch.Tensor:
    """Per-cluster mode of every categorical attribute ([k, F]) via the K2 histogram kernel with the
    cluster id as the class (CategoricalHistogramStat in the reference reducer)."""
    from ..ops.histogram import class_histogram
    lab = torch.full((codes.shape[1],), 255, dtype=torch.uint8, device=codes.device)
    lab[:n] = assign[:n].clamp(0, 254).to(torch.uint8)
    h = class_histogram(codes, n, bins, lab, k)
    if comm is not None and comm.is_distributed:
        comm.all_reduce(h)
    out, o = [], 0
    for b in bins:
        out.append(h[:, o:o + b].argmax(1))
        o += b
    return torch.stack(out, 1)


# ----------------------------------------------------------------------------------------------
def dbscan(X: torch.Tensor, eps: float, min_samples: int = 5, chunk: int = 8192) -> torch.Tensor:
    """DBSCAN labels (-1 = noise) with GPU neighbourhood queries and label propagation."""
    n = X.shape[0]
    X = X.float()
    nbr_counts = torch.zeros(n, dtype=torch.long, device=X.device)
    for s in range(0, n, chunk):
        d = torch.cdist(X[s:s + chunk], X)
        nbr_counts[s:s + chunk] = (d <= eps).sum(1)
    core = nbr_counts >= min_samples
    labels = torch.where(core, torch.arange(n, device=X.device), torch.full((n,), n, device=X.device))
    # min-label propagation over core-core edges until fixpoint
    for _ in range(n):
        changed = False
        for s in range(0, n, chunk):
            d = torch.cdist(X[s:s + chunk], X)
            adj = (d <= eps) & core.unsqueeze(0)
            nb = torch.where(adj, labels.unsqueeze(0), torch.full_like(d, n, dtype=labels.dtype)).min(1).values
            blk = labels[s:s + chunk]
            upd = core[s:s + chunk] & (nb < blk)
            if bool(upd.any()):
                labels[s:s + chunk] = torch.where(upd, nb, blk)
                changed = True
        if not changed:
            break
    # border points: label of a core neighbour
    out = torch.full((n,), -1, dtype=torch.long, device=X.device)
    for s in range(0, n, chunk):
        d = torch.cdist(X[s:s + chunk], X)
        adj = (d <= eps) & core.unsqueeze(0)
        nb = torch.where(adj, labels.unsqueeze(0), torch.full_like(d, n, dtype=labels.dtype)).min(1).values
        out[s:s + chunk] = torch.where(nb < n, nb, torch.full_like(nb, -1))
    # relabel to 0..m-1
    uniq = torch.unique(out[out >= 0])
    remap = torch.full((n + 1,), -1, dtype=torch.long, device=X.device)
    remap[uniq] = torch.arange(uniq.numel(), device=X.device)
    return torch.where(out >= 0, remap[out.clamp_min(0)], out)


def hopkins(X: torch.Tensor, sample: int = 100, seed: int = 0) -> float:
    """Hopkins statistic (P/unsupv/cluster.py): ~0.5 random, -> 1 clustered."""
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    n = X.shape[0]
    m = min(sample, n - 1)
    X = X.float()
    idx = (torch.randperm(n, generator=g)[:m] if n <= 4 * m else torch.randint(0, n, (m,), generator=g)).to(X.device)
    lo, hi = X.min(0).values, X.max(0).values
    U = lo + (hi - lo) * torch.rand((m, X.shape[1]), generator=g).to(X.device)
    ud, _ = dist.knn(U, X, 1, "euclidean")
    # nearest OTHER data point of each sampled data point (k = 2, drop the point itself)
    wd, _ = dist.knn(X[idx], X, 2, "euclidean")
    u, w = float(ud.sum()), float(wd[:, 1].sum())
    return u / (u + w)


class AgglomerativeGraphical:
    """Greedy graph clustering over an edge-distance structure (``J/cluster/AgglomerativeGraphical``):
    each entity joins the existing cluster with the best average edge weight when it exceeds
    ``min_avg_weight``, otherwise starts a new cluster."""

    def __init__(self, min_avg_weight: float = 0.5):
        self.min_avg_weight = min_avg_weight

    def fit(self, W: torch.Tensor) -> torch.Tensor:
        """W: dense [n, n] edge weights (similarity; 0 = no edge)."""
        n = W.shape[0]
        labels = torch.full((n,), -1, dtype=torch.long)
        Wc = W.double().cpu()
        members: list[list[int]] = []
        for i in range(n):
            best, arg = -math.inf, -1
            for c, mem in enumerate(members):
                avg = float(Wc[i, mem].mean())
                if avg > best:
                    best, arg = avg, c
            if arg >= 0 and best >= self.min_avg_weight:
                members[arg].append(i)
                labels[i] = arg
            else:
                members.append([i])
                labels[i] = len(members) - 1
        return labels
