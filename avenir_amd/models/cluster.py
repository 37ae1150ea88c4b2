"""Clustering: batched / distributed k-means (+ k-means++ and knuckle selection), agglomerative
graphical clustering, DBSCAN, Hopkins statistic.

Reference: ``J/cluster/KmeansCluster.java`` (one MR job per Lloyd iteration over many cluster
groups: mapper finds the nearest centroid with the mixed-type record distance, reducer recomputes
numeric means + categorical modes, movement / status / SSE, :57-297), ``S/cluster/KmeansCluster.scala``
(many (k, init-group) runs, min-SSE run per k, knuckle k by the max second difference of SSE,
:103-172), ``S/cluster/KMeansPlusPlusCluster.scala`` (commons-math k-means++), ``P/unsupv/cluster.py``
(sklearn kmeans / agglomerative / dbscan, Hopkins statistic), ``J/cluster/AgglomerativeGraphical.java``.

MI355X: a group of up to 16 runs shares ONE pass over the data per iteration (K16: packed-FMA
scoring against SGPR-resident centroid pairs, one-hot x rows on the matrix cores for the partial
sums), a deterministic device reduction, ONE all-reduce of the flat [K (D+1) + R] statistics
replaces the shuffle, and the centroid update + movement test run on the device.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch

from .. import _native
from ..ops import distance as dist
from ..parallel.comm import Comm, get_comm
from ..utils.resilience import IterationLoop, RecoveryConfig


def kmeanspp_seed_batch(samples: list[torch.Tensor], ks: list[int], us: list[torch.Tensor],
                        max_elems: int = 1 << 26) -> list[torch.Tensor]:
    """Greedy k-means++ (Arthur & Vassilvitskii 2007, as scikit-learn) for several runs at once.
    Run r seeds ``ks[r]`` centres from its sample ``samples[r]`` [m, D]; per centre it draws
    L = ``us[r].shape[1]`` candidates by D^2 inverse-CDF sampling (the uniforms ``us[r]`` [k, L],
    row 0's first entry picks the first centre) and keeps the one that lowers the potential most.
    Runs with samples of one shape advance together: per centre index one cumsum, one batched
    searchsorted, one batched distance and one argmin over [R, L, m] — chunked so R L m stays
    under ``max_elems`` — with finished runs (k reached) frozen by a mask.  No host round trip."""
    out: list[torch.Tensor | None] = [None] * len(samples)
    by_key: dict[tuple, list[int]] = {}
    for r, S in enumerate(samples):
        by_key.setdefault((S.shape[1], us[r].shape[1], S.device), []).append(r)
    for (D, L, dev), rs in by_key.items():
        # samples of different sizes (the key groups of a job) share a launch, zero-padded to the
        # chunk's largest: a padded row has D^2 weight 0, so it is never drawn and adds 0 to every
        # potential; the first centre and the candidate clamp use the run's own size
        rs = sorted(rs, key=lambda r: samples[r].shape[0])
        step = max(1, max_elems // max(1, L * samples[rs[-1]].shape[0]))
        for c0 in range(0, len(rs), step):
            grp = rs[c0:c0 + step]
            ms = [samples[r].shape[0] for r in grp]
            m, R, kmax = max(ms), len(grp), max(ks[r] for r in grp)
            if min(ms) == m:
                S = torch.stack([samples[r] for r in grp]).float()                   # [R, m, D]
            else:
                S = torch.zeros((R, m, D), dtype=torch.float32, device=dev)
                for j, r in enumerate(grp):
                    S[j, : ms[j]] = samples[r]
            U = torch.zeros((R, kmax, L), dtype=torch.float64)
            for j, r in enumerate(grp):
                U[j, : ks[r]] = us[r]
            U = U.to(dev)
            kk = torch.tensor([ks[r] for r in grp], device=dev)
            mr = torch.tensor(ms, device=dev)
            ar = torch.arange(R, device=dev)
            Sd = S.double()
            i0 = torch.minimum((U[:, 0, 0] * mr.double()).long(), mr - 1)
            idx = torch.zeros((R, kmax), dtype=torch.long, device=dev)
            idx[:, 0] = i0
            d2 = ((S - S[ar, i0].unsqueeze(1)) ** 2).sum(2).double()                # [R, m]
            if min(ms) != m:
                d2 = d2 * (torch.arange(m, device=dev) < mr.unsqueeze(1))
            for i in range(1, kmax):
                cum = torch.cumsum(d2, 1)
                cand = torch.minimum(torch.searchsorted(cum, cum[:, -1:] * U[:, i], right=True),
                                     (mr - 1).unsqueeze(1))                          # [R, L]
                dc = torch.cdist(Sd[ar.unsqueeze(1), cand], Sd).square()            # [R, L, m]
                pot = torch.minimum(dc, d2.unsqueeze(1))
                best = pot.sum(2).argmin(1)                                          # [R]
                live = kk > i
                idx[:, i] = torch.where(live, cand[ar, best], 0)
                d2 = torch.where(live.unsqueeze(1), pot[ar, best], d2)
            for j, r in enumerate(grp):
                out[r] = S[j, idx[j, : ks[r]]]
    return out


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


class _PairLayout:
    """Device state of one launch group in the K16 pair layout: runs padded to an even centroid
    count (padding centroids have norm +inf and are never chosen), stored as C2 [Kp/2, Dp, 2]."""

    def __init__(self, Cs: list[torch.Tensor], Dp: int):
        dev = Cs[0].device
        self.ks = [c.shape[0] for c in Cs]
        self.h_roff = [0]
        for k in self.ks:
            self.h_roff.append(self.h_roff[-1] + k + (k & 1))
        K = self.h_roff[-1]
        self.K, self.Dp = K, Dp
        Cf = torch.zeros((K, Dp), dtype=torch.float32, device=dev)
        self.Cn = torch.full((K,), math.inf, dtype=torch.float32, device=dev)
        run_of = torch.full((K,), -1, dtype=torch.int32)
        for r, C in enumerate(Cs):
            o, k = self.h_roff[r], self.ks[r]
            Cf[o:o + k, :C.shape[1]] = C.float()
            self.Cn[o:o + k] = (C.float() ** 2).sum(1)
            run_of[o:o + k] = r
        self.C2 = Cf.view(K // 2, 2, Dp).transpose(1, 2).contiguous()
        self.run_of = run_of.to(dev)
        self.roff = torch.tensor(self.h_roff, dtype=torch.int32, device=dev)

    def centroids(self, r: int, D: int) -> torch.Tensor:
        Cf = self.C2.transpose(1, 2).reshape(self.K, self.Dp)
        o = self.h_roff[r]
        return Cf[o:o + self.ks[r], :D].contiguous()

    def stats(self, flat: torch.Tensor, r: int, D: int):
        """(sums f64 [k, D], counts f64 [k], sse f64 scalar) of run r from the reduced vector."""
        blk = flat[: self.K * (self.Dp + 1)].view(self.K, self.Dp + 1)
        o, k = self.h_roff[r], self.ks[r]
        return blk[o:o + k, :D], blk[o:o + k, self.Dp], flat[self.K * (self.Dp + 1) + r]


def kmeans_step(X: torch.Tensor, Cs: list[torch.Tensor], want_assign: bool = False):
    """One fused K16 Lloyd pass of several runs over ``X`` (GPU, D padded to 2/4/8/16/32/64):
    per run (sums f64 [k, D], counts f64 [k], sse f64, assignment int32 [n] or None)."""
    Dp = X.shape[1]
    lay = _PairLayout(Cs, Dp)
    C = _native.C()
    partial, ssep, assign = C.kmeans_assign(X.float().contiguous(), lay.C2, lay.Cn, lay.roff, lay.h_roff,
                                            want_assign)
    flat = C.kmeans_reduce(partial, ssep)
    out = []
    for r in range(len(Cs)):
        sums, counts, sse = lay.stats(flat, r, Dp)
        out.append((sums, counts, sse, assign[r] if want_assign else None))
    return out


class KMeans:
    def __init__(self, n_clusters: int | list[int] = 3, n_init: int = 1, max_iter: int = 300,
                 tol: float = 1e-4, init: str = "k-means++", seed: int = 0, comm: Comm | None = None,
                 recovery: RecoveryConfig | None = None, tol_mode: str = "shift"):
        self.ks = [n_clusters] if isinstance(n_clusters, int) else list(n_clusters)
        self.n_init = n_init
        self.max_iter = max_iter
        self.tol = tol
        # "shift": a run converges when every centroid moves <= tol (J/cluster/ClusterData.java:
        # movement > centroidShiftThreshold keeps a cluster active); "sklearn": when the summed
        # squared centroid shift <= tol x the mean per-feature variance of the data (P/unsupv/
        # cluster.py uses scikit-learn's KMeans and its tol)
        if tol_mode not in ("shift", "sklearn"):
            raise ValueError(f"unknown tol_mode {tol_mode}")
        self.tol_mode = tol_mode
        self.init = init
        self.seed = seed
        self.comm = comm
        self.recovery = recovery           # checkpoint / resume per Lloyd iteration (utils/resilience)
        self.runs: list[KMeansRun] = []
        self.best: dict[int, KMeansRun] = {}

    # ------------------------------------------------------------------------------------------
    def _seed_sample(self, X: torch.Tensor, g: torch.Generator, comm) -> torch.Tensor:
        """A run's seeding sample: up to 64k points overall, in O(m) and on X's device: every row
        when the shard fits; m distinct rows of a random affine permutation i -> (a i + b) mod n
        (gcd(a, n) = 1) up to 4 m rows; m uniform draws above (duplicates are harmless).  Only
        scalars come from the host generator, so CPU and GPU sample the same rows (a host randperm
        per run was 27 ms of kMeansPlusPlusCluster's 69: profiles/r6_slow_jobs.jsonl)."""
        n = X.shape[0]
        m = min(n, max(1, 65536 // max(comm.world, 1)))
        if m >= n:
            sel = None
        elif n <= 4 * m:
            a = int(torch.randint(1, n, (1,), generator=g))
            while math.gcd(a, n) != 1:
                a = a % (n - 1) + 1
            b = int(torch.randint(0, n, (1,), generator=g))
            sel = (torch.arange(m, device=X.device, dtype=torch.long) * a + b) % n
        else:
            sel = torch.randint(0, n, (m,), generator=g).to(X.device)
        S = (X if sel is None else X[sel]).float()
        if comm.is_distributed:
            S = comm.all_gather_v(S)
        return S

    def _init_centroids_all(self, X: torch.Tensor, specs: list[tuple[int, int]]) -> list[torch.Tensor]:
        """Initial centroids of every (k, seed) run, identical on every rank (rank 0's, broadcast).
        k-means++ seeding runs for ALL runs of the fit together (:func:`kmeanspp_seed_batch`): one
        set of batched tensor ops per centre index instead of one per centre per run (63 runs of
        the kMeansPlusPlusCluster sweep spent 29 of its 46 ms in per-run seeding loops)."""
        return KMeans.init_many([self], [X])[0]

    def run_specs(self) -> list[tuple[int, int]]:
        """(k, seed) of every run of a fit, in run order."""
        return [(k, self.seed * 1009 + k * 31 + r) for k in self.ks for r in range(self.n_init)]

    @staticmethod
    def init_many(models: list["KMeans"], Xs: list[torch.Tensor]) -> list[list[torch.Tensor]]:
        """Initial centroids of every run of several independent fits (model i on Xs[i]), the
        k-means++ seeding of all of them in ONE :func:`kmeanspp_seed_batch` pass (the
        kMeansPlusPlusCluster job seeds all its key groups together)."""
        per_model, kpp = [], []
        for km, X in zip(models, Xs):
            comm = km.comm or get_comm()
            specs = km.run_specs()
            X = X.float().contiguous()
            gens = [torch.Generator(device="cpu").manual_seed(sd) for _, sd in specs]
            samples = [km._seed_sample(X, g, comm) for g in gens]
            if km.init == "random":
                per_model.append([S[torch.randperm(S.shape[0], generator=g)[:k].to(S.device)]
                                  for (k, _), S, g in zip(specs, samples, gens)])
            else:
                ks = [k for k, _ in specs]
                us = [torch.rand((k, 2 + int(math.log(max(k, 2)))), generator=g, dtype=torch.float64)
                      for k, g in zip(ks, gens)]
                per_model.append(None)
                kpp.append((len(per_model) - 1, samples, ks, us))
        if kpp:
            flat = kmeanspp_seed_batch([S for _, ss, _, _ in kpp for S in ss], [k for _, _, ks, _ in kpp for k in ks],
                                       [u for _, _, _, us in kpp for u in us])
            o = 0
            for i, ss, _, _ in kpp:
                per_model[i] = flat[o:o + len(ss)]
                o += len(ss)
        out = []
        for km, Cs in zip(models, per_model):
            comm = km.comm or get_comm()
            if comm.is_distributed:
                Cs = [comm.broadcast(C.contiguous(), 0) for C in Cs]
            out.append([C.contiguous() for C in Cs])
        return out

    def _step(self, X: torch.Tensor, Cs: list[torch.Tensor]):
        """CPU oracle of one Lloyd pass -> per run (sums f64 [k, D], counts [k], sse f64 [1])."""
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
        """Pack runs into launch groups: <= 16 runs and at most as many padded centroids as one
        launch holds (the kernel picks its MFMA or LDS variant from the group's size); CPU: one run
        per group."""
        groups, cur, tot = [], [], 0
        # MFMA variant: <= 16 blocks of 16 centroids x 16 dims; LDS variant: K (2 Dp + 2) floats <= 64 KiB
        cap = max(256 // max(1, Dp // 16), (65536 // (8 * Dp + 8)) & ~1) if Dp else 1 << 30
        for i, (k, _) in enumerate(specs):
            kp = k + (k & 1)
            if kp > cap:
                raise ValueError(f"k={k} exceeds the {cap} centroids one k-means launch holds at D={Dp}")
            if cur and (len(cur) == 16 or tot + kp > cap or Dp is None):
                groups.append(cur)
                cur, tot = [], 0
            cur.append(i)
            tot += kp
        if cur:
            groups.append(cur)
        return groups

    def fit(self, X: torch.Tensor, init_centroids: list[torch.Tensor] | None = None) -> "KMeans":
        """All (k, init) runs advance together (S/cluster/KmeansCluster.scala keys by
        (numClusters, initGroup)).  GPU: per iteration ONE fused assignment launch for a group of
        runs, one reduction launch, one RCCL all-reduce of the flat [K (D+1) + R] statistics when
        distributed, one update launch and a 4-byte-per-run host read of the centroid movement."""
        comm = self.comm or get_comm()
        X = X.float().contiguous()
        self._tol_eff = self._effective_tol(X, comm)
        Xp = self._padded(X)
        specs = self.run_specs()
        if init_centroids is None:                 # (``init_centroids``: from init_many)
            init_centroids = self._init_centroids_all(X, specs)
        runs = [KMeansRun(k, sd, C) for (k, sd), C in zip(specs, init_centroids)]
        self.best = {}
        for gi, grp in enumerate(self._groups(specs, Xp.shape[1] if Xp is not None else None)):
            with IterationLoop(f"kmeans.g{gi}", self.recovery, comm, device=X.device) as lp:
                if Xp is not None:
                    self._fit_gpu_group(X.shape[1], Xp, [runs[i] for i in grp], comm, lp)
                else:
                    self._fit_cpu_group(X, [runs[i] for i in grp], comm, lp)
        self.runs = runs
        for r in runs:
            if r.k not in self.best or r.sse < self.best[r.k].sse:
                self.best[r.k] = r
        return self

    def _effective_tol(self, X: torch.Tensor, comm) -> float:
        if self.tol_mode == "shift":
            return self.tol
        # global mean of per-feature variances (sums / squares / count all-reduced)
        st = torch.stack([X.double().sum(0), (X.double() ** 2).sum(0)])
        n = torch.tensor([float(X.shape[0])], dtype=torch.float64, device=X.device)
        if comm.is_distributed:
            comm.all_reduce(st)
            comm.all_reduce(n)
        mean = st[0] / n
        var = (st[1] / n - mean * mean).clamp_min(0)
        return float(var.mean()) * self.tol

    def _converged(self, max_shift: float, sq_shift: float) -> bool:
        if self.tol_mode == "shift":
            return max_shift <= self.tol
        return sq_shift <= self._tol_eff

    def _fit_gpu_group(self, D: int, Xp: torch.Tensor, grp: list[KMeansRun], comm,
                       lp: IterationLoop) -> None:
        C = _native.C()
        lay = _PairLayout([r.centroids for r in grp], Xp.shape[1])
        R = len(grp)
        frozen_h = [0] * R
        frozen = torch.zeros(R, dtype=torch.uint8, device=Xp.device)
        hist: list[tuple[int, torch.Tensor]] = []
        it0, st, _ = lp.restore(Xp.device)
        if st is not None:                              # resume: centroids, status, SSE history
            lay.C2.copy_(st["C2"])
            lay.Cn.copy_(st["Cn"])
            frozen_h = [int(v) for v in st["frozen"].tolist()]
            frozen.copy_(st["frozen"])
            hist = [(i, st["hist"][i]) for i in range(st["hist"].shape[0])]
            for r, run in enumerate(grp):
                run.iterations = int(st["iters"][r])
                run.converged = bool(frozen_h[r])
        nbytes = float(Xp.numel() * 4)
        for it in range(it0, self.max_iter):
            if all(frozen_h):
                break
            with lp.step(it, nbytes=nbytes):
                partial, ssep, _ = C.kmeans_assign(Xp, lay.C2, lay.Cn, lay.roff, lay.h_roff, False)
                flat = C.kmeans_reduce(partial, ssep)
                if comm.is_distributed:
                    flat = comm.all_reduce(flat)
                moves = C.kmeans_update(flat, lay.C2, lay.Cn, lay.run_of, frozen, lay.Dp)
                hist.append((it, flat[-R:]))
                mv = moves.cpu().tolist()                  # the one host sync of the iteration
            changed = False
            for r, run in enumerate(grp):
                if frozen_h[r]:
                    continue
                run.iterations = it + 1
                if self._converged(mv[r], mv[R + r]):
                    run.converged = True
                    frozen_h[r] = 1
                    changed = True
            if changed:
                frozen.copy_(torch.tensor(frozen_h, dtype=torch.uint8))
            if lp.enabled:
                lp.commit(it, {"C2": lay.C2, "Cn": lay.Cn, "frozen": frozen,
                               "iters": torch.tensor([r.iterations for r in grp]),
                               "hist": torch.stack([h for _, h in hist])})
        sse_hist = torch.stack([h for _, h in hist]).cpu() if hist else torch.zeros((0, R), dtype=torch.float64)
        for r, run in enumerate(grp):
            run.history = [float(sse_hist[i, r]) for i in range(run.iterations)]
            run.centroids = lay.centroids(r, D)
        partial, ssep, _ = C.kmeans_assign(Xp, lay.C2, lay.Cn, lay.roff, lay.h_roff, False)
        flat = C.kmeans_reduce(partial, ssep)
        if comm.is_distributed:
            flat = comm.all_reduce(flat)
        for r, run in enumerate(grp):
            _, counts, sse = lay.stats(flat, r, D)
            run.sse, run.counts = float(sse), counts.round().long()

    def _fit_cpu_group(self, X: torch.Tensor, grp: list[KMeansRun], comm, lp: IterationLoop) -> None:
        active = list(range(len(grp)))
        it0, st, _ = lp.restore(X.device)
        if st is not None:
            for r, run in enumerate(grp):
                run.centroids = st[f"c{r}"].to(X.device)
                run.iterations = int(st["iters"][r])
                run.converged = bool(st["done"][r])
                run.history = st[f"h{r}"].tolist()
            active = [r for r in range(len(grp)) if not grp[r].converged]
        for it in range(it0, self.max_iter):
            if not active:
                break
            with lp.step(it):
                res = self._step(X, [grp[i].centroids for i in active])
            if comm.is_distributed:
                flat = torch.cat([torch.cat([s.view(-1), c.double().view(-1), e]) for s, c, e in res])
                flat = comm.all_reduce(flat)
                o, red = 0, []
                for s_, c, e in res:
                    a, b = s_.numel(), c.numel()
                    red.append((flat[o:o + a].view_as(s_), flat[o + a:o + a + b].round().long(),
                                flat[o + a + b:o + a + b + 1]))
                    o += a + b + 1
                res = red
            still = []
            for i, (sums, counts, sse) in zip(active, res):
                run = grp[i]
                Cc = run.centroids
                newC = torch.where(counts.view(-1, 1) > 0, sums / counts.clamp_min(1).view(-1, 1),
                                   Cc.double()).float()
                sh2 = ((newC - Cc) ** 2).sum(1)
                mv, sq = float(sh2.sqrt().max()), float(sh2.sum())
                run.centroids = newC
                run.history.append(float(sse))
                run.iterations = it + 1
                if self._converged(mv, sq):
                    run.converged = True
                else:
                    still.append(i)
            active = still
            if lp.enabled:
                state = {f"c{r}": run.centroids for r, run in enumerate(grp)}
                state.update({f"h{r}": torch.tensor(run.history, dtype=torch.float64) for r, run in enumerate(grp)})
                state["iters"] = torch.tensor([run.iterations for run in grp])
                state["done"] = torch.tensor([run.converged for run in grp])
                lp.commit(it, state)
        final = self._step(X, [r.centroids for r in grp])
        for run, (sums, counts, sse) in zip(grp, final):
            if comm.is_distributed:
                sse = comm.all_reduce(sse)
                counts = comm.all_reduce(counts)
            run.sse, run.counts = float(sse), counts

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
