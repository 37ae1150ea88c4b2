"""Batched stochastic optimisers (K22): simulated annealing, genetic algorithm (island model),
evolutionary strategy, random multi-start search with local search, tabu search, Bayesian
optimisation, and hyper-parameter search.

Reference behaviour:
* Spark SA — one chain per partition, Metropolis acceptance, geometric/linear cooling every
  ``temp.update.interval`` moves, accumulators, optional local search of each chain's best
  (S/optimize/SimulatedAnnealing.scala:111-234; config R/opt.conf).
* Spark GA — island model, each partition an independent GA (S/optimize/GeneticAlgorithm.scala:70-163).
* Spark random search — random multi-start then ``focussed`` (neighbours of the best) or
  ``trajectory`` local search (S/optimize/RandomSearch.scala:105-250).
* Python optimisers — ``EvolutionaryOptimizer`` / ``GeneticAlgorithmOptimizer`` (P/mlextra/optpopu.py:32-187,
  pool / mating / replacement / purge-by-cost-and-age), ``SimulatedAnnealingOptimizer`` and
  ``BayesianOptimizer`` (P/mlextra/optsolo.py:34-182); parameter search (P/supv/pasearch.py:17-242);
  ``TabuSearchDomain`` tenure purge (J/optimize/TabuSearchDomain.java:54-66).

MI355X design: the population / the set of chains / the set of islands is the batch axis of
device tensors.  Simulated annealing over an :class:`AssignmentDomain` runs entirely inside one
K22 kernel launch (one chain per lane, solution tile in LDS), and so does the island genetic
algorithm (optimize/ga.py: one workgroup per island, pool / costs / children in LDS, all
generations of a migration interval per launch; its numpy twin is the CPU path, bit-equal).
Other domains take batched tensor ops per generation; the GA over them runs one generation per
ISLAND (each island draws from its own generator, keyed by global island index, so that results do
not depend on the world size): ~12 small launches per island per generation.  Measured on one
MI355X (profiles/r6_ga_islands.jsonl): 8 / 64 / 512 islands x 50 generations at 3.9 k / 20.5 k /
110 k island-generations/s end to end with the kernel, 316 / 310 with the per-island path.
Chains and islands are indexed GLOBALLY (their random streams
are keyed by global index, not by rank): rank r runs its block of them, the W-rank run equals one
process running all of them, the global best is one tiny all-gather, and checkpoints re-deal the
chains / islands over any world size on resume.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, Sequence

import numpy as np
import torch

from .. import _native
from ..ops.random import philox4x32, u32_to_unit
from ..parallel.comm import Comm, get_comm
from ..utils.resilience import IterationLoop, RecoveryConfig
from .domain import AssignmentDomain, SearchDomain


@dataclass
class OptResult:
    best: torch.Tensor                 # [L] best solution (value indices)
    best_cost: float
    costs: torch.Tensor                # [n] best cost per chain / island (local rank)
    solutions: torch.Tensor            # [n, L]
    history: list = field(default_factory=list)
    stats: dict = field(default_factory=dict)


def _gen(device, seed: int) -> torch.Generator:
    return torch.Generator(device=torch.device(device)).manual_seed(int(seed))


def _global_best(comm: Comm, cost: torch.Tensor, sol: torch.Tensor) -> tuple[torch.Tensor, float]:
    if cost.numel() == 0:                  # a rank left without chains / islands after a re-deal
        c, s = torch.full((1,), math.inf, device=cost.device), torch.zeros(sol.shape[-1], dtype=torch.long,
                                                                            device=sol.device)
    else:
        i = int(torch.argmin(cost))
        c, s = cost[i:i + 1].float(), sol[i].long()
    if comm.is_distributed:
        dev = comm.device if comm.backend == "nccl" else torch.device("cpu")
        cs = comm.all_gather(c.to(dev)).view(-1)
        ss = comm.all_gather(s.to(dev))
        j = int(torch.argmin(cs))
        return ss[j].to(sol.device), float(cs[j])
    return s, float(c)


# ================================================================================================
# simulated annealing
# ================================================================================================
class SimulatedAnnealing:
    """Batched SA chains.  The one-launch K22 kernel (``sa_assign_kernel``) takes assignment domains
    with single-position moves (``max.step.size`` = 1) and L <= 512 positions (the [L][64]
    solution tile of a wave lives in LDS).  Multi-position steps, larger L and other domains run
    the batched generic path: every chain of the rank advances together, one set of tensor ops
    per move (documented limit; the reference's task-schedule configurations all use step 1 and
    tens of positions)."""

    def __init__(self, domain: SearchDomain, n_chains: int = 8, iters: int = 300, t0: float = 30.0,
                 cooling: float = 0.99, geometric: bool = True, interval: int = 2, step: int = 1,
                 max_retry: int = 3, seed: int = 0, locally_optimize: bool = False, local_iters: int = 50,
                 comm: Comm | None = None, use_kernel: bool | None = None,
                 recovery: RecoveryConfig | None = None, segment: int | None = None):
        self.domain = domain
        self.recovery = recovery        # checkpoint / resume (utils/resilience)
        self.segment = segment          # moves per checkpointed segment (default iters / 10)
        self.n_chains, self.iters, self.t0, self.cooling = n_chains, iters, t0, cooling
        self.geometric, self.interval, self.step, self.max_retry = geometric, interval, step, max_retry
        self.seed, self.locally_optimize, self.local_iters = seed, locally_optimize, local_iters
        self.comm = comm
        self.use_kernel = use_kernel

    @classmethod
    def from_config(cls, domain, cfg, **kw) -> "SimulatedAnnealing":
        """HOCON block of R/opt.conf (``simulatedAnnealing``)."""
        return cls(domain, n_chains=cfg.get_int("num.optimizers"), iters=cfg.get_int("max.num.iterations"),
                   t0=cfg.get_float("initial.temp", 30.0), cooling=cfg.get_float("cooling.rate.value", 0.99),
                   geometric=cfg.get_bool("cooling.rate.geometric", True),
                   interval=cfg.get_int("temp.update.interval", 2), step=cfg.get_int("max.step.size", 1),
                   locally_optimize=cfg.get_bool("locally.optimize", False),
                   local_iters=cfg.get_int("max.num.local iterations", cfg.get_int("max.num.local.iterations", 50)),
                   **kw)

    def run(self, init: torch.Tensor | None = None) -> OptResult:
        comm = self.comm or get_comm()
        d = self.domain
        kernel_ok = isinstance(d, AssignmentDomain) and self.step == 1 and d.L <= 512
        use_kernel = kernel_ok if self.use_kernel is None else (self.use_kernel and kernel_ok)
        chain_base = None
        if use_kernel:
            best, bc, stats, gen, chain_base = self._run_kernel(comm, init)
        else:
            seed = self.seed + 1_000_003 * comm.rank
            gen = _gen(d.device, seed)
            sol = d.random(self.n_chains, gen)[0] if init is None else init.to(d.device).long().clone()
            # generic path: one torch generator per rank drives every chain of the rank -> sharded
            # state, resumable at the world size that wrote it
            with IterationLoop("simulatedAnnealing.generic", self.recovery, comm, sharded=True,
                               device=d.device) as lp:
                best, bc, stats = self._generic(sol, d.evaluate(sol), gen, lp)
        if self.locally_optimize:
            if chain_base is None:      # generic path: the rank's generator (as its chains)
                best, bc = local_focussed(d, best, bc, self.local_iters, gen)
            else:                       # kernel path: one generator per GLOBAL chain, so the result
                outs = [local_focussed(d, best[p:p + 1], bc[p:p + 1], self.local_iters,  # does not depend on W
                                       _gen(d.device, self.seed + 1_000_003 + chain_base + p))
                        for p in range(best.shape[0])]
                if outs:
                    best = torch.cat([o[0] for o in outs])
                    bc = torch.cat([o[1] for o in outs])
        b, c = _global_best(comm, bc, best)
        return OptResult(b, c, bc, best, stats=stats)

    def _run_kernel(self, comm, init):
        """K22 path.  Chains are GLOBAL: chain ``g`` draws Philox stream ``(seed, g)`` and starts from
        row ``g`` of one population drawn from ``seed`` alone, rank ``r`` runs chains
        ``[r * n_chains, (r + 1) * n_chains)``.  The W-rank result therefore equals one process
        running ``W * n_chains`` chains, and the checkpoint (rank 0 writes every chain) resumes at
        ANY world size: the restored chains are re-dealt by global index.  Under checkpointing the
        run is split into segments of ``segment`` moves (one launch each, same Philox counters and
        cooling schedule as one launch)."""
        from ..data.table import shard_range
        d = self.domain
        W, r = comm.world, comm.rank
        gen = None                                               # local search: per global chain (run)
        stats = {"better": 0, "worse_accepted": 0, "rejected": 0}
        best = bc = temp = None
        b0 = 0
        with IterationLoop("simulatedAnnealing", self.recovery, comm, device=d.device) as lp:
            _, st, meta = lp.restore(d.device)
            if st is not None:
                total = int(meta["chains"])
                a, e = shard_range(total, r, W)
                sol, cost, best, bc = (st[k][a:e].to(d.device) for k in ("sol", "cost", "best", "best_cost"))
                temp, b0 = float(meta["temp"]), int(meta["moves"])
                if r == 0:                                       # global counters: summed over ranks at the end
                    stats = dict(meta["stats"])
            else:
                if init is None:
                    total = self.n_chains * W
                    sol = d.random(total, _gen(d.device, self.seed))[0][r * self.n_chains:(r + 1) * self.n_chains]
                    a = r * self.n_chains
                else:
                    sol = init.to(d.device).long().clone()
                    counts = comm.all_gather(torch.tensor([sol.shape[0]])).view(-1).tolist()
                    total, a = sum(counts), sum(counts[:r])
                cost = d.evaluate(sol)
            seg = max(1, self.segment or -(-self.iters // 10)) if lp.enabled else max(1, self.iters)
            for b in range(b0, self.iters, seg):
                n = min(seg, self.iters - b)
                with lp.step(b // seg):
                    best, bc, s, sol, cost, temp = sa_assign(d, sol, cost, n, self.t0, self.cooling, self.interval,
                                                             self.geometric, self.max_retry, self.seed, 0, it_begin=b,
                                                             temp_start=temp, best=best, best_cost=bc,
                                                             return_state=True, chain_base=a)
                for k in stats:
                    stats[k] += s[k]
                if lp.enabled:
                    full = [comm.all_gather_v(x.contiguous()) for x in (sol, cost, best, bc)]
                    lp.commit(b // seg, dict(zip(("sol", "cost", "best", "best_cost"), full)),
                              {"temp": temp, "moves": b + n, "stats": self._global_stats(comm, stats),
                               "chains": total}, force=True)
        if best is None:                                   # no moves at all
            best, bc = sol.clone(), cost.clone()
        return best.long(), bc, self._global_stats(comm, stats), gen, a

    @staticmethod
    def _global_stats(comm, stats: dict) -> dict:
        if not comm.is_distributed:
            return dict(stats)
        v = torch.tensor([stats[k] for k in ("better", "worse_accepted", "rejected")], dtype=torch.float64)
        comm.all_reduce(v)
        return dict(zip(("better", "worse_accepted", "rejected"), (int(x) for x in v.tolist())))

    def _generic(self, sol, cost, gen, lp: IterationLoop | None = None):
        d = self.domain
        best, bc = sol.clone(), cost.clone()
        temp = self.t0
        stats = {"better": 0, "worse_accepted": 0, "rejected": 0}
        it0 = 0
        if lp is not None:
            it0, st, meta = lp.restore(d.device)
            if st is not None:
                sol, cost, best, bc = st["sol"], st["cost"], st["best"], st["best_cost"]
                gen.set_state(st["rng"])
                temp, stats = float(meta["temp"]), dict(meta["stats"])
        for it in range(it0, self.iters):
            if lp is not None:
                with lp.step(it):
                    pass
            cand, _ = d.mutate(sol, self.step, gen, self.max_retry)
            cc = d.evaluate(cand)
            delta = cc - cost
            u = torch.rand(cost.shape, generator=gen, device=cost.device)
            acc = (delta <= 0) | (u < torch.exp(-delta / max(temp, 1e-12)))
            stats["better"] += int((delta <= 0).sum())
            stats["worse_accepted"] += int((acc & (delta > 0)).sum())
            stats["rejected"] += int((~acc).sum())
            sol = torch.where(acc.view(-1, 1), cand, sol)
            cost = torch.where(acc, cc, cost)
            imp = cost < bc
            best[imp] = sol[imp]
            bc = torch.minimum(bc, cost)
            if self.interval > 0 and (it + 1) % self.interval == 0:
                temp = temp * self.cooling if self.geometric else max(self.t0 - (it + 1) * self.cooling, 1e-12)
            if lp is not None and lp.enabled:
                lp.commit(it, {"sol": sol, "cost": cost, "best": best, "best_cost": bc, "rng": gen.get_state()},
                          {"temp": temp, "stats": stats})
        return best, bc, stats


def sa_assign(d: AssignmentDomain, sol: torch.Tensor, cost: torch.Tensor, iters: int, t0: float, cool: float,
              interval: int, geometric: bool, max_retry: int, seed: int, offset: int, it_begin: int = 0,
              temp_start: float | None = None, best: torch.Tensor | None = None, best_cost: torch.Tensor | None = None,
              return_state: bool = False, chain_base: int = 0):
    """Run ``sol.shape[0]`` SA chains over an assignment domain: K22 kernel on GPU, the bit-exact
    numpy mirror (same Philox stream, float32 arithmetic) on CPU.  Returns (best_sol, best_cost, stats)
    or, with ``return_state``, also (current_sol, current_cost, temperature) so a run split into
    segments [it_begin, it_begin + iters) (checkpoint / resume) equals one uninterrupted launch.
    Row ``p`` is global chain ``chain_base + p``: its Philox stream does not depend on the launch."""
    ts = float(t0 if temp_start is None else temp_start)
    if sol.device.type == "cuda":
        s16 = sol.to(torch.int16).contiguous()
        cur = cost.float().contiguous().clone()
        bsol = s16.clone() if best is None else best.to(torch.int16).contiguous().clone()
        bc = cur.clone() if best_cost is None else best_cost.float().contiguous().clone()
        st = torch.zeros(4, dtype=torch.long, device=sol.device)
        _native.C().sa_assign(d.cost_table, None if d.conflict is None else d.conflict.to(torch.uint8).contiguous(),
                              bool(d.swap_moves), s16, cur, bsol, bc, int(iters), float(t0), float(cool),
                              int(interval), bool(geometric), int(max_retry), int(seed), int(offset), st,
                              int(it_begin), ts, int(chain_base))
        s = st.tolist()
        stats = {"better": s[0], "worse_accepted": s[1], "rejected": s[2]}
        if return_state:
            temp = float(np.array([s[3]], dtype=np.uint32).view(np.float32)[0]) if iters > 0 else ts
            return bsol.long(), bc, stats, s16.long(), cur, temp
        return bsol.long(), bc, stats
    out = sa_assign_reference(d.cost_table.numpy(), None if d.conflict is None else d.conflict.numpy(),
                              d.swap_moves, sol.numpy(), cost.float().numpy(), iters, t0, cool, interval,
                              geometric, max_retry, seed, offset, it_begin, ts,
                              None if best is None else best.numpy(), None if best_cost is None else best_cost.float().numpy(),
                              chain_base)
    b, c, s, cs, cc, temp = out
    if return_state:
        return (torch.from_numpy(b).long(), torch.from_numpy(c), s, torch.from_numpy(cs).long(),
                torch.from_numpy(cc), float(temp))
    return torch.from_numpy(b).long(), torch.from_numpy(c), s


def sa_assign_reference(cost, conflict, swap, sol, cur, iters, t0, cool, interval, geometric, max_retry, seed, offset,
                        it_begin=0, temp_start=None, best=None, best_cost=None, chain_base=0):
    """Host mirror of ``sa_assign_kernel`` (optim.hip), vectorised over chains.  Returns
    (best, best_cost, stats, current_sol, current_cost, temperature)."""
    cost = np.asarray(cost, np.float32)
    L, V = cost.shape
    sol = np.array(sol, dtype=np.int64)
    P = sol.shape[0]
    c = np.array(cur, dtype=np.float32)
    bc = c.copy() if best_cost is None else np.array(best_cost, dtype=np.float32)
    best = sol.copy() if best is None else np.array(best, dtype=np.int64)
    rows = np.arange(P)
    idx = np.arange(P, dtype=np.uint64) + np.uint64(chain_base)
    ar = np.arange(L)
    invL = np.float32(1.0 / L)
    temp = np.float32(t0 if temp_start is None else temp_start)
    st = [0, 0, 0]
    R = max_retry + 1
    for it in range(it_begin, it_begin + iters):
        pending = np.ones(P, bool)
        pos = np.full(P, -1)
        nv = np.zeros(P, np.int64)
        old = np.zeros(P, np.int64)
        j2 = np.full(P, -1)
        for tr in range(R):
            if not pending.any():
                break
            x, y, _, _ = philox4x32(seed, offset + it * R + tr, idx)
            cp = np.minimum((u32_to_unit(x) * np.float32(L)).astype(np.int64), L - 1)
            cv = np.minimum((u32_to_unit(y) * np.float32(V - 1)).astype(np.int64), V - 2)
            ov = sol[rows, cp]
            cv = cv + (cv >= ov)
            if swap:
                holder = (sol == cv[:, None]) & (ar[None, :] != cp[:, None])
                sw = np.where(holder.any(1), holder.argmax(1), -1)
            else:
                sw = np.full(P, -1)
            cand = sol.copy()
            cand[rows, cp] = cv
            hs = sw >= 0
            cand[rows[hs], sw[hs]] = ov[hs]
            if conflict is not None:
                bad = ((cand == cv[:, None]) & (ar[None, :] != cp[:, None]) & conflict[cp]).any(1)
                swr = np.where(hs, sw, 0)
                bad2 = ((cand == ov[:, None]) & (ar[None, :] != swr[:, None]) & conflict[swr]).any(1) & hs
                ok = ~(bad | bad2)
            else:
                ok = np.ones(P, bool)
            take = pending & ok
            sol[take] = cand[take]
            pos[take], nv[take], old[take], j2[take] = cp[take], cv[take], ov[take], sw[take]
            pending &= ~ok
        moved = pos >= 0
        pp = np.where(moved, pos, 0)
        delta = cost[pp, nv] - cost[pp, old]
        jj = np.where(j2 >= 0, j2, 0)
        delta = np.where(j2 >= 0, delta + (cost[jj, old] - cost[jj, nv]), delta).astype(np.float32)
        delta = (delta * invL).astype(np.float32)
        x2, _, _, _ = philox4x32(seed ^ 0x9E3779B97F4A7C15, offset + it, idx)
        with np.errstate(over="ignore"):
            pr = np.exp(-delta / np.maximum(temp, np.float32(1e-12))).astype(np.float32)
        acc = moved & ((delta <= 0) | (u32_to_unit(x2) < pr))
        rej = moved & ~acc
        st[0] += int((acc & (delta <= 0)).sum())
        st[1] += int((acc & (delta > 0)).sum())
        st[2] += int(rej.sum())
        r = rows[rej]
        sol[r, pos[rej]] = old[rej]
        hj = rej & (j2 >= 0)
        sol[rows[hj], j2[hj]] = nv[hj]
        c = np.where(acc, (c + delta).astype(np.float32), c)
        imp = acc & (c < bc)
        best[imp] = sol[imp]
        bc = np.where(imp, c, bc)
        if interval > 0 and (it + 1) % interval == 0:
            temp = np.float32(temp * np.float32(cool)) if geometric else np.float32(max(t0 - (it + 1) * cool, 1e-12))
    return (best, bc.astype(np.float32), {"better": st[0], "worse_accepted": st[1], "rejected": st[2]},
            sol, c.astype(np.float32), temp)


def local_focussed(d: SearchDomain, sols: torch.Tensor, costs: torch.Tensor, n_iter: int, gen=None):
    """Neighbours of each solution (reference = the start solution, not the walk), keep the best
    (SimulatedAnnealing.scala:199-234 / RandomSearch.localFocussedSearch :170-210): one batch of
    ``P * n_iter`` mutants."""
    P, L = sols.shape
    rep = sols.repeat_interleave(n_iter, 0)
    mut, _ = d.mutate(rep, 1, gen)
    mc = d.evaluate(mut).view(P, n_iter)
    j = mc.argmin(1)
    mb = mc[torch.arange(P), j]
    better = mb < costs
    out = sols.clone()
    out[better] = mut.view(P, n_iter, L)[torch.arange(P, device=sols.device)[better], j[better]]
    return out, torch.where(better, mb, costs)


def local_trajectory(d: SearchDomain, sols: torch.Tensor, costs: torch.Tensor, n_iter: int, gen=None,
                     fanout: int = 4):
    """Hill climb: each step samples ``fanout`` neighbours of the CURRENT solution and moves to the
    best if it improves (OptUtility.localTrajectorySearch, J/optimize/OptUtility.java:46-66)."""
    P, L = sols.shape
    cur, cc = sols.clone(), costs.clone()
    for _ in range(n_iter):
        nb, nc = local_focussed(d, cur, cc, fanout, gen)
        cur, cc = nb, nc
    return cur, cc


# ================================================================================================
# population optimisers
# ================================================================================================
class GeneticAlgorithm:
    """Island-model GA: ``islands`` independent pools advance together as one [I, pool, L] batch.

    Per generation and island: sort, take the ``mating`` best, make ``replacement`` children by
    single-point crossover of random mating pairs + mutation, keep valid children, purge the
    ``replacement`` worst (before or after adding, ``purge_first``).  Optional ring migration of
    island elites every ``migrate_every`` generations (the reference islands never exchange)."""

    def __init__(self, domain: SearchDomain, islands: int = 4, pool: int = 10, mating: int = 5, replacement: int = 5,
                 generations: int = 100, purge_first: bool = True, mutate_children: bool = True,
                 migrate_every: int = 0, seed: int = 0, comm: Comm | None = None,
                 recovery: RecoveryConfig | None = None, use_kernel: bool | None = None):
        self.d = domain
        self.use_kernel = use_kernel    # None: the island kernel (optimize/ga.py) whenever it applies
        self.recovery = recovery        # per-generation checkpoint / resume (utils/resilience)
        self.I, self.Pp, self.m, self.r, self.G = islands, pool, mating, replacement, generations
        self.purge_first, self.mutate_children, self.migrate_every = purge_first, mutate_children, migrate_every
        self.seed, self.comm = seed, comm

    @classmethod
    def from_properties(cls, domain, conf, islands: int = 1, **kw):
        """``opti.*`` keys of P/mlextra/optpopu.py:104-110 (a :class:`~avenir_amd.utils.config.Configuration`)."""
        return cls(domain, islands=islands, pool=conf.get_int("opti.pool.size")[0],
                   mating=conf.get_int("opti.mating.size")[0], replacement=conf.get_int("opti.replacement.size")[0],
                   generations=conf.get_int("opti.num.iter")[0], purge_first=conf.get_boolean("opti.purge.first")[0],
                   **kw)

    def run(self) -> OptResult:
        """Islands are GLOBAL: island ``g`` owns a generator seeded ``seed + 7919 g`` that draws its
        initial pool and every crossover / mutation of that island, and rank ``r`` runs islands
        ``[r * islands, (r + 1) * islands)``; migration is a ring over the global island order (one
        all-gather of the elites).  So the W-rank run equals one process running ``W * islands``
        islands, and the checkpoint — every island's pool, costs, history and generator state,
        written by rank 0 — resumes at ANY world size by re-dealing the islands by global index."""
        from ..data.table import shard_range
        comm = self.comm or get_comm()
        if self._kernel_ok():
            return self._run_islands(comm)
        d, Pp, L = self.d, self.Pp, self.d.L
        W, r = comm.world, comm.rank
        lp = IterationLoop("geneticAlgorithm", self.recovery, comm, device=d.device)
        g0, st, meta = lp.restore(d.device)
        if st is not None:
            total = int(meta["islands"])
            a, e = shard_range(total, r, W)
            pop, cost, hist = (st[k][a:e].to(d.device) for k in ("pop", "cost", "hist"))
            gens = []
            for i in range(a, e):
                gg = _gen(d.device, 0)
                gg.set_state(st["rng"][i].cpu().clone())
                gens.append(gg)
        else:
            total, a, e = self.I * W, r * self.I, (r + 1) * self.I
            gens = [_gen(d.device, self.seed + 7919 * i) for i in range(a, e)]
            pop = torch.stack([d.random(Pp, gg)[0] for gg in gens]).view(e - a, Pp, L)
            cost = d.evaluate(pop.view(-1, L)).view(e - a, Pp)
            hist = torch.empty((e - a, 0), dtype=cost.dtype, device=d.device)
        for g in range(g0, self.G):
            with lp.step(g):
                outs = [self._generation(pop[i:i + 1], cost[i:i + 1], gens[i]) for i in range(e - a)]
                if outs:
                    pop = torch.cat([o[0] for o in outs])
                    cost = torch.cat([o[1] for o in outs])
                    hist = torch.cat([hist, torch.cat([o[2] for o in outs]).view(-1, 1)], 1)
                if self.migrate_every and total > 1 and (g + 1) % self.migrate_every == 0:
                    pop, cost = self._migrate(comm, pop, cost, a, e)
            if lp.enabled:
                rng = torch.stack([gg.get_state() for gg in gens]) if gens else torch.empty((0, 1), dtype=torch.uint8)
                full = [comm.all_gather_v(x.contiguous()) for x in (pop, cost, hist, rng)]
                lp.commit(g, dict(zip(("pop", "cost", "hist", "rng"), full)), {"islands": total})
        lp.close()
        ha = comm.all_gather_v(hist.contiguous()) if comm.is_distributed else hist
        history = ha.min(0).values.tolist() if ha.shape[0] else []
        ii = torch.arange(e - a, device=d.device)
        bi = cost.argmin(1)
        bs, bc = pop[ii, bi], cost[ii, bi]
        b, c = _global_best(comm, bc, bs)
        return OptResult(b, c, bc, bs, history)

    def _kernel_ok(self) -> bool:
        """The one-launch island kernel (optimize/ga.py): assignment domains without tied groups
        or checkpointing, pools of <= 64, LDS <= 64 KiB per island; on the CPU its host twin."""
        d = self.d
        if self.use_kernel is False or not isinstance(d, AssignmentDomain) or getattr(d, "groups", None):
            return False
        if self.recovery is not None:
            return False
        P, r, m = self.Pp, self.r, self.m
        if not (2 <= P <= 64 and 1 <= r <= min(P, 32) and 1 <= m <= P and (self.purge_first or P + r <= 64)):
            return False
        lds = (2 * P + 2 * r) * d.L * 2 + (2 * P + 2 * r) * 8
        return lds <= 64 * 1024 and d.V <= 32767

    def _run_islands(self, comm) -> OptResult:
        """All of this rank's islands, G generations, in one kernel launch (per migration interval):
        islands [r * islands, (r + 1) * islands) by GLOBAL index, so the W-rank run equals one
        process running W * islands; migration (ring of elites) runs on host copies between
        launches, identically on either device."""
        from .ga import ga_assign_run, ga_init_population, ga_price
        d = self.d
        W, rk = comm.world, comm.rank
        a, e = rk * self.I, (rk + 1) * self.I
        total = self.I * W
        conf = None
        if d.conflict is not None:
            c = d.conflict.cpu().numpy()
            conf = np.triu(c, 1) | np.triu(c, 1).T
        pop = ga_init_population(e - a, self.Pp, d.L, d.V, self.seed, a, conf)
        cost = ga_price(d.cost_table.cpu().numpy().astype(np.float32), conf, d.invalid_cost, pop.astype(np.int64))
        step = self.migrate_every if (self.migrate_every and total > 1) else self.G
        hists = []
        g = 0
        while g < self.G:
            k = min(step, self.G - g)
            pop, cost, h = ga_assign_run(d, pop, cost, k, self.m, self.r, self.purge_first, self.mutate_children,
                                         self.seed, a, d.device, gen_base=g)
            hists.append(h)
            g += k
            if g < self.G and step < self.G:
                tp, tc = self._migrate(comm, torch.from_numpy(pop.astype(np.int64)), torch.from_numpy(cost), a, e)
                pop, cost = tp.numpy().astype(np.int16), tc.numpy().astype(np.float32)
        hist = torch.from_numpy(np.concatenate(hists, 1) if hists else np.zeros((e - a, 0), np.float32))
        ha = comm.all_gather_v(hist.contiguous()) if comm.is_distributed else hist
        history = ha.min(0).values.tolist() if ha.shape[0] else []
        bi = cost.argmin(1)
        ii = np.arange(e - a)
        bs = torch.from_numpy(pop[ii, bi].astype(np.int64)).to(d.device)
        bc = torch.from_numpy(cost[ii, bi]).to(d.device)
        b, c = _global_best(comm, bc, bs)
        return OptResult(b, c, bc, bs, history, {"engine": "ga_assign_kernel" if d.device.type == "cuda" else "ga_twin"})

    @staticmethod
    def _migrate(comm, pop, cost, a, e):
        """Ring migration over the global islands: island g's elite replaces the worst member of
        island g + 1 (mod the island count)."""
        ii = torch.arange(e - a, device=pop.device)
        bi = cost.argmin(1)
        elite, ec = pop[ii, bi], cost[ii, bi]
        ge, gc = comm.all_gather_v(elite.contiguous()), comm.all_gather_v(ec.contiguous())
        ge, gc = ge.roll(1, 0)[a:e], gc.roll(1, 0)[a:e]
        wi = cost.argmax(1)
        pop, cost = pop.clone(), cost.clone()
        pop[ii, wi] = ge.to(pop.device)
        cost[ii, wi] = gc.to(cost.device)
        return pop, cost

    def _generation(self, pop, cost, gen):
        """One generation of the islands in ``pop`` [I, pool, L] (all drawing from ``gen``).
        Returns (pop, cost, best cost at the generation's start per island)."""
        d, L = self.d, self.d.L
        I, Pp = pop.shape[0], pop.shape[1]
        ii = torch.arange(I, device=d.device).view(-1, 1)
        order = cost.argsort(1)
        pop, cost = pop[ii, order], cost[ii, order]
        first = cost[:, 0].clone()
        # children: 2x oversampled pairs from the mating list, first r valid per island
        npair = self.r
        a = (torch.rand((I, npair), generator=gen, device=d.device) * self.m).long().clamp_max(self.m - 1)
        b = (torch.rand((I, npair), generator=gen, device=d.device) * (self.m - 1)).long().clamp_max(max(self.m - 2, 0))
        b = b + (b >= a).long()
        pa, pb = pop[ii, a].view(-1, L), pop[ii, b.clamp_max(Pp - 1)].view(-1, L)
        c1, c2 = d.crossover(pa, pb, gen)
        kids = torch.cat([c1.view(I, npair, L), c2.view(I, npair, L)], 1).view(-1, L)
        if self.mutate_children:
            kids, _ = d.mutate(kids, 1, gen)
        kc = d.evaluate(kids).view(I, 2 * npair)
        kids = kids.view(I, 2 * npair, L)
        ko = kc.argsort(1)[:, : self.r]                              # best r children (valid first)
        kids, kc = kids[ii, ko], kc[ii, ko]
        if self.purge_first:
            pop = torch.cat([pop[:, : Pp - self.r], kids], 1)
            cost = torch.cat([cost[:, : Pp - self.r], kc], 1)
        else:
            allp, allc = torch.cat([pop, kids], 1), torch.cat([cost, kc], 1)
            o = allc.argsort(1)[:, :Pp]
            pop, cost = allp[ii, o], allc[ii, o]
        return pop, cost, first


class EvolutionaryOptimizer:
    """Mutation-only steady-state evolution (P/mlextra/optpopu.py:32-96), all islands at once:
    tournament-select the best of ``select`` random pool members, mutate a clone, purge the member
    with the worst ``w * cost + (1 - w) * age`` and insert the child."""

    def __init__(self, domain: SearchDomain, islands: int = 4, pool: int = 5, select: int = 3, iters: int = 100,
                 purge_cost_weight: float = 0.7, purge_age_scale: float = 1.0, seed: int = 0, comm: Comm | None = None):
        self.d = domain
        self.I, self.Pp, self.k, self.iters = islands, pool, select, iters
        self.w, self.age_scale, self.seed, self.comm = purge_cost_weight, purge_age_scale, seed, comm

    def run(self) -> OptResult:
        comm = self.comm or get_comm()
        d, I, Pp, L = self.d, self.I, self.Pp, self.d.L
        dev = d.device
        gen = _gen(dev, self.seed + 104729 * comm.rank)
        pop, _ = d.random(I * Pp, gen)
        cost = d.evaluate(pop).view(I, Pp)
        pop = pop.view(I, Pp, L)
        born = torch.arange(Pp, device=dev).view(1, -1).repeat(I, 1)
        ii = torch.arange(I, device=dev)
        bi0 = cost.argmin(1)
        best, bc = pop[ii, bi0].clone(), cost[ii, bi0].clone()
        history = []
        for it in range(self.iters):
            sel = torch.rand((I, Pp), generator=gen, device=dev).argsort(1)[:, : self.k]
            sc = cost.gather(1, sel)
            w = sel.gather(1, sc.argmin(1, keepdim=True)).view(-1)
            child, ok = d.mutate(pop[ii, w], 1, gen)
            cc = d.evaluate(child)
            # purge: age by insertion order (older = larger), P/mlextra/opti.py purge :630-645
            rank = born.argsort(1).argsort(1)
            age = (Pp - rank).float() * self.age_scale / Pp
            fin = torch.where(torch.isfinite(cost), cost, torch.full_like(cost, 1e30))
            aggr = self.w * fin + (1 - self.w) * age
            wi = aggr.argmax(1)
            upd = ok
            pop[ii[upd], wi[upd]] = child[upd]
            cost[ii[upd], wi[upd]] = cc[upd]
            born[ii[upd], wi[upd]] = Pp + it
            imp = upd & (cc < bc)
            best[imp], bc[imp] = child[imp], cc[imp]
            history.append(float(bc.min()))
        b, c = _global_best(comm, bc, best)
        return OptResult(b, c, bc, best, history)


class RandomSearch:
    """Random multi-start: ``n`` random solutions (sharded over ranks), global best by all-gather,
    then optional ``focussed`` or ``trajectory`` local search (S/optimize/RandomSearch.scala)."""

    def __init__(self, domain: SearchDomain, n: int = 1024, local: str | None = "focussed", local_iters: int = 50,
                 seed: int = 0, comm: Comm | None = None, top_k: int = 10):
        self.d, self.n, self.local, self.local_iters, self.seed, self.comm, self.top_k = \
            domain, n, local, local_iters, seed, comm, top_k

    def run(self) -> OptResult:
        comm = self.comm or get_comm()
        d = self.d
        gen = _gen(d.device, self.seed + 31337 * comm.rank)
        n_local = self.n // comm.world + (1 if comm.rank < self.n % comm.world else 0)
        sol, _ = d.random(max(n_local, 1), gen)
        cost = d.evaluate(sol)
        b, c = _global_best(comm, cost, sol)
        if self.local:
            bb, cc = b.view(1, -1).to(d.device), torch.tensor([c], device=d.device)
            fn = local_focussed if self.local == "focussed" else local_trajectory
            bb, cc = fn(d, bb, cc, self.local_iters, gen)
            # every rank searched its own neighbourhood: take the best again
            b, c = _global_best(comm, cc, bb)
        k = min(self.top_k, cost.numel())
        o = cost.argsort()[:k]
        return OptResult(b, c, cost[o], sol[o])


class TabuSearch:
    """Batched tabu search over an :class:`AssignmentDomain`: every iteration scores the FULL
    single-reassignment neighbourhood ``[P, L, V]`` in closed form (cost delta from the table,
    validity of every move via one ``conflict @ occupancy`` GEMM), masks tabu moves unless they
    beat the best (aspiration), and takes the best admissible move; reversing a move is tabu for
    ``tenure`` iterations (TabuSearchDomain purge, J/optimize/TabuSearchDomain.java:54-66)."""

    def __init__(self, domain: AssignmentDomain, n_chains: int = 8, iters: int = 200, tenure: int = 7, seed: int = 0,
                 comm: Comm | None = None):
        self.d, self.P, self.iters, self.tenure, self.seed, self.comm = domain, n_chains, iters, tenure, seed, comm

    def run(self) -> OptResult:
        comm = self.comm or get_comm()
        d = self.d
        dev, L, V, P = d.device, d.L, d.V, self.P
        gen = _gen(dev, self.seed + 15485863 * comm.rank)
        sol, _ = d.random(P, gen)
        cost = d.evaluate(sol)
        best, bc = sol.clone(), cost.clone()
        tabu = torch.full((P, L, V), -1, dtype=torch.long, device=dev)
        rows = torch.arange(P, device=dev)
        conf = None if d.conflict is None else d.conflict.float()
        history = []
        for it in range(self.iters):
            delta = d.neighbourhood_delta(sol)                                   # [P, L, V]
            occ = torch.nn.functional.one_hot(sol, V).float()                    # [P, L, V]
            bad = torch.zeros((P, L, V), dtype=torch.bool, device=dev)
            if conf is not None:
                bad = torch.einsum("lj,pjv->plv", conf, occ) > 0
            bad |= occ.bool()                                                    # staying put is not a move
            new_cost = cost.view(-1, 1, 1) + delta
            is_tabu = tabu > it
            admissible = ~bad & (~is_tabu | (new_cost < bc.view(-1, 1, 1)))
            score = torch.where(admissible, new_cost, torch.full_like(new_cost, float("inf"))).reshape(P, -1)
            flat = score.argmin(1)
            has = torch.isfinite(score[rows, flat])
            l, v = flat // V, flat % V
            old = sol[rows, l]
            tabu[rows[has], l[has], old[has]] = it + self.tenure
            sol[rows[has], l[has]] = v[has]
            cost = torch.where(has, score[rows, flat], cost)
            imp = cost < bc
            best[imp], bc[imp] = sol[imp], cost[imp]
            history.append(float(bc.min()))
        b, c = _global_best(comm, bc, best)
        return OptResult(b, c, bc, best, history)


# ================================================================================================
# Bayesian optimisation (continuous box) — P/mlextra/optsolo.py:91-175, finished
# ================================================================================================
class BayesianOptimizer:
    """GP (RBF kernel, Cholesky) surrogate with ``pi`` / ``ei`` / ``lcb`` acquisition maximised over
    ``acq_samples`` random candidates per step; ``cost_fn(x [n, d]) -> [n]`` is vectorised."""

    def __init__(self, cost_fn: Callable, lo: Sequence[float], hi: Sequence[float], n_init: int = 20, iters: int = 30,
                 acq: str = "ei", acq_samples: int = 2048, lcb_mult: float = 2.0, length_scale: float = 0.2,
                 noise: float = 1e-6, seed: int = 0, device="cpu"):
        self.f = cost_fn
        self.lo = torch.tensor(lo, dtype=torch.float64, device=device)
        self.hi = torch.tensor(hi, dtype=torch.float64, device=device)
        self.n_init, self.iters, self.acq, self.ns, self.kappa = n_init, iters, acq, acq_samples, lcb_mult
        self.ls, self.noise, self.seed, self.device = length_scale, noise, seed, torch.device(device)

    def _k(self, a, b):
        d2 = ((a.unsqueeze(1) - b.unsqueeze(0)) ** 2).sum(2)
        return torch.exp(-0.5 * d2 / self.ls ** 2)

    def run(self) -> OptResult:
        g = _gen(self.device, self.seed)
        D = self.lo.numel()
        span = self.hi - self.lo
        X = torch.rand((self.n_init, D), generator=g, device=self.device, dtype=torch.float64)
        y = torch.as_tensor(self.f(self.lo + X * span), device=self.device).double().view(-1)
        hist = []
        for _ in range(self.iters):
            mu_y, sd_y = y.mean(), y.std().clamp_min(1e-12)
            yn = (y - mu_y) / sd_y
            K = self._k(X, X) + self.noise * torch.eye(X.shape[0], device=self.device, dtype=torch.float64)
            Lc = torch.linalg.cholesky(K + 1e-9 * torch.eye(X.shape[0], device=self.device, dtype=torch.float64))
            alpha = torch.cholesky_solve(yn.view(-1, 1), Lc)
            C = torch.rand((self.ns, D), generator=g, device=self.device, dtype=torch.float64)
            Ks = self._k(C, X)
            mu = (Ks @ alpha).view(-1)
            v = torch.cholesky_solve(Ks.T, Lc)
            var = (1.0 - (Ks * v.T).sum(1)).clamp_min(1e-12)
            sd = var.sqrt()
            best = yn.min()
            z = (best - mu) / sd
            nrm = torch.distributions.Normal(0.0, 1.0)
            if self.acq == "pi":
                a = nrm.cdf(z)
            elif self.acq == "ei":
                a = (best - mu) * nrm.cdf(z) + sd * torch.exp(nrm.log_prob(z))
            elif self.acq == "lcb":
                a = -(mu - self.kappa * sd)
            else:
                raise ValueError(self.acq)
            xn = C[int(a.argmax())].view(1, -1)
            yv = torch.as_tensor(self.f(self.lo + xn * span), device=self.device).double().view(-1)
            X, y = torch.cat([X, xn]), torch.cat([y, yv])
            hist.append(float(y.min()))
        i = int(y.argmin())
        return OptResult((self.lo + X[i] * span), float(y[i]), y, self.lo + X * span, hist)


# ================================================================================================
# hyper-parameter search (P/supv/pasearch.py)
# ================================================================================================
def parameter_search(space: dict[str, Sequence], score_fn: Callable[[dict], float], strategy: str = "random",
                     n_iter: int = 20, seed: int = 0, t0: float = 1.0, cooling: float = 0.9,
                     comm: Comm | None = None) -> tuple[dict, float, list]:
    """Search a discrete hyper-parameter grid minimising ``score_fn(params)``.

    ``guided``: coordinate-wise sweeps (GuidedParameterSearch); ``random``: random grid points
    (RandomParameterSearch); ``sa``: simulated annealing over grid neighbours
    (SimulatedAnnealingParameterSearch).  Each evaluation trains a model, so this runs on the host
    and the models themselves use the device."""
    names = list(space)
    rng = np.random.default_rng(seed)
    cache: dict = {}

    def ev(idx):
        key = tuple(idx)
        if key not in cache:
            cache[key] = float(score_fn({n: space[n][i] for n, i in zip(names, idx)}))
        return cache[key]

    hist = []
    if strategy == "guided":
        cur = [0] * len(names)
        best = ev(cur)
        for _ in range(max(1, n_iter // max(1, sum(len(space[n]) for n in names)))):
            for k, n in enumerate(names):
                for i in range(len(space[n])):
                    cand = cur.copy()
                    cand[k] = i
                    s = ev(cand)
                    if s < best:
                        best, cur = s, cand
                    hist.append(best)
    elif strategy == "random":
        cur, best = None, float("inf")
        cands = [[int(rng.integers(len(space[n]))) for n in names] for _ in range(n_iter)]
        if comm is not None and comm.is_distributed:
            # the candidates are independent, so every rank trains its share (one
            # trial per GPU) and the scores are all-gathered; the walk below then reads the cache
            todo = sorted({tuple(c) for c in cands}, key=lambda c: cands.index(list(c)))
            mine = {c: float(score_fn({n: space[n][i] for n, i in zip(names, c)}))
                    for c in todo[comm.rank::comm.world]}
            for part in comm.all_gather_object(mine):
                cache.update(part)
        for cand in cands:
            s = ev(cand)
            if s < best:
                best, cur = s, cand
            hist.append(best)
    elif strategy == "sa":
        cur = [int(rng.integers(len(space[n]))) for n in names]
        cs = ev(cur)
        best, bcur, temp = cs, cur, t0
        for _ in range(n_iter):
            cand = cur.copy()
            k = int(rng.integers(len(names)))
            if len(space[names[k]]) > 1:
                cand[k] = (cand[k] + int(rng.choice([-1, 1]))) % len(space[names[k]])
            s = ev(cand)
            if s < cs or math.exp((cs - s) / max(temp, 1e-12)) > rng.random():
                cur, cs = cand, s
                if s < best:
                    best, bcur = s, cand
            temp *= cooling
            hist.append(best)
        cur = bcur
    else:
        raise ValueError(strategy)
    return {n: space[n][i] for n, i in zip(names, cur)}, best, hist
