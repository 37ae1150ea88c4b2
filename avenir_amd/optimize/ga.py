"""Island genetic algorithm over an assignment domain as ONE kernel launch (K22,
``csrc/kernels/optim.hip::ga_assign_kernel``) and its bit-exact host twin.

Reference: the Spark GA runs an independent GA per partition (S/optimize/GeneticAlgorithm.scala:70-163);
the Python GeneticAlgorithmOptimizer keeps a pool, crosses random pairs of its mating list and
purges (P/mlextra/optpopu.py:98-187).  Here every island is one workgroup whose pool, costs and
children stay in LDS for all G generations of a launch; its random stream is Philox keyed by the
island's GLOBAL index, so any world size and either device produce the same islands.

:func:`ga_assign_reference` replays the kernel's arithmetic in numpy — the same Philox counters,
the same fp32 cost sums in position order, the same (cost, index) orderings — so GPU output equals
it bit for bit; it is also the CPU path of :class:`~avenir_amd.optimize.search.GeneticAlgorithm`
for assignment domains.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops.random import philox4x32, u32_to_unit

_MUT_KEY = 0xD1B54A32D192ED03      # the kernel's mutation stream key (seed ^ this)
_INIT_KEY = 0x2545F4914F6CDD1D     # initial pools


_MAX_TRY = 10                      # the kernel's GA_MAX_TRY


def ga_init_population(n_islands: int, P: int, L: int, V: int, seed: int, island_base: int,
                       conflict: np.ndarray | None = None, max_try: int = 40) -> np.ndarray:
    """Initial pools [islands, P, L] int16, position by position as AssignmentDomain.random: the
    value of island gi, member p, position l, attempt a is Philox(seed ^ INIT, (p L + l) 64 + a,
    stream gi), redrawn while it clashes with an earlier conflicting position (up to ``max_try``
    attempts) — per global island, host-side."""
    gis = np.arange(island_base, island_base + n_islands, dtype=np.uint64)
    out = np.zeros((n_islands, P, L), dtype=np.int64)
    for p in range(P):
        for l in range(L):
            todo = np.arange(n_islands)
            for a in range(max_try):
                x, _, _, _ = philox4x32(seed ^ _INIT_KEY, (p * L + l) * 64 + a, gis[todo])
                out[todo, p, l] = np.minimum((u32_to_unit(x) * np.float32(V)).astype(np.int64), V - 1)
                if conflict is None or l == 0:
                    break
                clash = ((out[todo, p, :l] == out[todo, p, l][:, None]) & conflict[l, :l][None, :]).any(1)
                todo = todo[clash]
                if todo.size == 0:
                    break
    return out.astype(np.int16)


def _valid(conf: np.ndarray | None, sol: np.ndarray) -> np.ndarray:
    if conf is None:
        return np.ones(sol.shape[:-1], dtype=bool)
    same = sol[..., :, None] == sol[..., None, :]
    return ~(same & conf).any(axis=(-1, -2))


def ga_price(cost: np.ndarray, conflict: np.ndarray | None, invalid: float, sol: np.ndarray) -> np.ndarray:
    """fp32 sum of cost[l, s_l] in position order times fp32 1/L (the kernel's ``ga_price``), or
    ``invalid`` when two conflicting positions share a value.  sol [..., L] -> [...] float32."""
    L = sol.shape[-1]
    acc = np.zeros(sol.shape[:-1], dtype=np.float32)
    for l in range(L):
        acc = acc + cost[l, sol[..., l]]
    out = acc * (np.float32(1.0) / np.float32(L))
    if conflict is not None:
        same = sol[..., :, None] == sol[..., None, :]
        bad = (same & conflict).any(axis=(-1, -2))
        out = np.where(bad, np.float32(invalid), out).astype(np.float32)
    return out


def _unit_index(u: np.ndarray, n: int) -> np.ndarray:
    """min((int)(u * (float)n), n - 1) in fp32, as the kernel."""
    return np.minimum((u * np.float32(n)).astype(np.int64), n - 1)


def ga_assign_reference(cost: np.ndarray, conflict: np.ndarray | None, invalid: float, pop: np.ndarray,
                        pop_cost: np.ndarray, G: int, m: int, r: int, purge_first: bool, mutate: bool,
                        seed: int, island_base: int, gen_base: int = 0,
                        swap: bool = True) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Host twin of ``ga_assign_kernel`` (all islands at once).  Returns (pop, pop_cost, hist)."""
    cost = np.ascontiguousarray(cost, dtype=np.float32)
    conf = None
    if conflict is not None:
        conf = np.asarray(conflict, dtype=bool)
        conf = conf & ~np.eye(conf.shape[0], dtype=bool)
        conf = np.triu(conf, 1) | np.triu(conf, 1).T          # the kernel reads the upper triangle
    pop = np.array(pop, dtype=np.int64)
    pc = np.array(pop_cost, dtype=np.float32)
    I, P, L = pop.shape
    V = cost.shape[1]
    gis = np.arange(island_base, island_base + I, dtype=np.uint64)
    ii = np.arange(I)[:, None]
    hist = np.zeros((I, G), dtype=np.float32)
    for g in range(G):
        ord_ = np.argsort(pc, axis=1, kind="stable")
        hist[:, g] = pc[np.arange(I), ord_[:, 0]]
        kids = np.empty((I, 2 * r, L), dtype=np.int64)
        for k in range(r):
            ctr = 256 * (gen_base + g) + k
            x_, y_, z_, _ = philox4x32(seed, ctr, gis)
            a = _unit_index(u32_to_unit(x_), m)
            if m > 1:
                b = np.minimum((u32_to_unit(y_) * np.float32(m - 1)).astype(np.int64), m - 2)
                b = b + (b >= a)
            else:
                b = np.zeros(I, dtype=np.int64)
            if L > 1:
                x = 1 + np.minimum((u32_to_unit(z_) * np.float32(L - 1)).astype(np.int64), L - 2)
            else:
                x = np.zeros(I, dtype=np.int64)
            A = pop[np.arange(I), ord_[np.arange(I), a]]
            B = pop[np.arange(I), ord_[np.arange(I), b]]
            left = np.arange(L)[None, :] < x[:, None]
            c1, c2 = np.where(left, A, B), np.where(left, B, A)
            if mutate:
                ar = np.arange(I)
                for h, c in ((0, c1), (1, c2)):
                    done = np.zeros(I, dtype=bool)
                    for t in range(_MAX_TRY):
                        q = philox4x32(seed ^ _MUT_KEY, ctr * 16 + t, gis)
                        qp, qv = (q[0], q[1]) if h == 0 else (q[2], q[3])
                        pos = _unit_index(u32_to_unit(qp), L)
                        old = c[ar, pos]
                        v = np.minimum((u32_to_unit(qv) * np.float32(V - 1)).astype(np.int64), V - 2)
                        v = v + (v >= old)
                        cand = c.copy()
                        if swap:
                            hold = (c == v[:, None]) & (np.arange(L)[None, :] != pos[:, None])
                            has = hold.any(1)
                            first = hold.argmax(1)
                            cand[ar[has], first[has]] = old[has]
                        cand[ar, pos] = v
                        take = ~done & ((t == _MAX_TRY - 1) | _valid(conf, cand))
                        c[take] = cand[take]
                        done |= take
            kids[:, 2 * k], kids[:, 2 * k + 1] = c1, c2
        kc = ga_price(cost, conf, invalid, kids)
        kord = np.argsort(kc, axis=1, kind="stable")
        if purge_first:
            nsrc = np.concatenate([ord_[:, : P - r], P + kord[:, :r]], axis=1)
        else:
            src = np.concatenate([np.broadcast_to(np.arange(P), (I, P)), P + kord[:, :r]], axis=1)
            cc = np.concatenate([pc, kc[ii, kord[:, :r]]], axis=1)
            nsrc = np.take_along_axis(src, np.argsort(cc, axis=1, kind="stable")[:, :P], axis=1)
        allp = np.concatenate([pop, kids], axis=1)
        allc = np.concatenate([pc, kc], axis=1)
        pop = allp[ii, nsrc]
        pc = allc[ii, nsrc]
    return pop.astype(np.int16), pc, hist


def ga_assign_run(domain, pop: np.ndarray, pop_cost: np.ndarray, G: int, m: int, r: int, purge_first: bool,
                  mutate: bool, seed: int, island_base: int, device: torch.device, gen_base: int = 0):
    """Advance the islands G generations (counters from ``gen_base``) on ``device``: the kernel on the
    GPU, the twin on the host.  Returns numpy (pop, pop_cost, hist)."""
    conflict = domain.conflict
    if device.type == "cuda":
        from .. import _native
        cost = domain.cost_table.to(device).float().contiguous()
        cf = None
        if conflict is not None:
            c = conflict.to(device).bool()
            c = c & ~torch.eye(c.shape[0], dtype=torch.bool, device=device)
            cf = (c.triu(1) | c.triu(1).T).to(torch.uint8).contiguous()
        tp = torch.from_numpy(np.ascontiguousarray(pop)).to(device)
        tc = torch.from_numpy(np.ascontiguousarray(pop_cost, dtype=np.float32)).to(device)
        hist = torch.empty((pop.shape[0], G), dtype=torch.float32, device=device)
        _native.C().ga_assign(cost, cf, float(domain.invalid_cost), tp, tc, hist, G, m, r, purge_first, mutate,
                              bool(domain.swap_moves), int(seed), int(island_base), int(gen_base))
        return tp.cpu().numpy(), tc.cpu().numpy(), hist.cpu().numpy()
    cf = None if conflict is None else conflict.cpu().numpy()
    return ga_assign_reference(domain.cost_table.cpu().numpy(), cf, domain.invalid_cost, pop, pop_cost, G, m, r,
                               purge_first, mutate, seed, island_base, gen_base, bool(domain.swap_moves))
