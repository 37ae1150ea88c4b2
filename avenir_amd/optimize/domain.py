"""Population-batched search domains (K22 host side).

Reference SPI: ``BasicSearchDomain`` (J/optimize/BasicSearchDomain.java:70-394: create / mutate with
retry + validity check / component-cost cache), ``PopulationSearchDomain`` (single-point crossover
with retry, J/optimize/PopulationSearchDomain.java:53-130) and the Python ``Candidate`` /
``BaseOptimizer`` (P/mlextra/opti.py:31-538) whose domain contract is ``isValid(values)`` /
``evaluate(values)`` (P/app/fesel.py:51-63).

MI355X design: a solution is a row of an int64 tensor ``[P, L]`` (position ``l`` holds an index
into that position's value table of cardinality ``cards[l]``), and the domain maps a WHOLE
population at once — ``cost(sol) -> [P]``, ``valid(sol) -> [P] bool`` — so creation, mutation,
crossover and selection are a handful of device kernels per generation instead of one virtual
call per candidate.  Domains whose cost is a sum of per-(position, value) terms and whose
constraint is pairwise ("two positions holding the same value must not conflict") expose that
structure as ``cost_table [L, V]`` + ``conflict [L, L]`` (:class:`AssignmentDomain`) and get the
fused K22 simulated-annealing kernel and the exact O(L·V) tabu neighbourhood.
"""
from __future__ import annotations

from typing import Callable, Sequence

import torch


class SearchDomain:
    """Base: fixed-length discrete solutions.  Subclasses set ``cards`` and implement ``cost`` and
    optionally ``valid``/``decode``.  ``groups`` ties positions together (they mutate as one, the
    reference's ``opti.solution.data.groups``, P/mlextra/opti.py:95-140)."""

    cards: torch.Tensor            # [L] int64 cardinality per position
    groups: list[list[int]] | None = None
    invalid_cost: float = float("inf")
    comp_size: int = 1             # crossover points are aligned to this (opti.solution.comp.size)
    swap_moves: bool = False

    @property
    def L(self) -> int:
        return int(self.cards.numel())

    @property
    def device(self) -> torch.device:
        return self.cards.device

    def cost(self, sol: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def valid(self, sol: torch.Tensor) -> torch.Tensor:
        return torch.ones(sol.shape[0], dtype=torch.bool, device=sol.device)

    def decode(self, sol: torch.Tensor):
        return sol

    def evaluate(self, sol: torch.Tensor) -> torch.Tensor:
        """cost with invalid rows priced at ``invalid_cost`` (BasicSearchDomain.getSolutionCost:272)."""
        c = self.cost(sol).float()
        return torch.where(self.valid(sol), c, torch.full_like(c, self.invalid_cost))

    # -------------------------------------------------------------------------------------------
    # batched operators
    # -------------------------------------------------------------------------------------------
    def random(self, P: int, gen: torch.Generator | None = None, max_try: int = 10):
        """P random solutions; rows failing validity are redrawn up to ``max_try`` times
        (createCandidate, P/mlextra/opti.py:68-100).  Returns (sol [P, L], valid [P])."""
        sol = self._draw(P, gen)
        ok = self.valid(sol)
        for _ in range(max_try):
            if bool(ok.all()):
                break
            bad = (~ok).nonzero().view(-1)
            sol[bad] = self._draw(int(bad.numel()), gen)
            ok = self.valid(sol)
        return sol, ok

    def _draw(self, P: int, gen) -> torch.Tensor:
        u = torch.rand((P, self.L), generator=gen, device=self.device)
        sol = (u * self.cards.float()).long().clamp_max(self.cards - 1)
        return self._tie_groups(sol)

    def _tie_groups(self, sol: torch.Tensor) -> torch.Tensor:
        if self.groups:
            for g in self.groups:
                sol[:, g[1:]] = sol[:, g[:1]]
        return sol

    def mutate(self, sol: torch.Tensor, n_pos: int = 1, gen: torch.Generator | None = None,
               max_try: int = 10) -> tuple[torch.Tensor, torch.Tensor]:
        """Mutate ``n_pos`` positions of every row to a different value; invalid results are redrawn
        up to ``max_try`` times, rows that never validate keep their last attempt and are flagged
        (BasicSearchDomain.mutateSolution :350-394).  Returns (new_sol, valid)."""
        P = sol.shape[0]
        out = sol.clone()
        todo = torch.arange(P, device=sol.device)
        ok = torch.zeros(P, dtype=torch.bool, device=sol.device)
        for _ in range(max(1, max_try)):
            cand = sol[todo].clone()
            for _s in range(n_pos):
                cand = self._move(cand, gen)
            v = self.valid(cand)
            out[todo] = cand
            ok[todo] = v
            todo = todo[~v]
            if todo.numel() == 0:
                break
        return out, ok

    def _move(self, sol: torch.Tensor, gen) -> torch.Tensor:
        P = sol.shape[0]
        rows = torch.arange(P, device=sol.device)
        pos = (torch.rand(P, generator=gen, device=sol.device) * self.L).long().clamp_max(self.L - 1)
        card = self.cards[pos]
        old = sol[rows, pos]
        nv = (torch.rand(P, generator=gen, device=sol.device) * (card - 1).clamp_min(1).float()).long()
        nv = torch.minimum(nv, (card - 2).clamp_min(0))
        nv = nv + (nv >= old).long()
        nv = torch.where(card > 1, nv, old)
        new = sol.clone()
        if self.swap_moves:
            # the position that held the new value takes the old one (first such position)
            holder = (sol == nv.view(-1, 1)) & (torch.arange(self.L, device=sol.device).view(1, -1) != pos.view(-1, 1))
            has = holder.any(1)
            first = holder.float().argmax(1)
            new[rows[has], first[has]] = old[has]
        new[rows, pos] = nv
        if self.groups:
            for g in self.groups:
                gi = torch.tensor(g, device=sol.device)
                hit = (pos.view(-1, 1) == gi.view(1, -1)).any(1)
                if bool(hit.any()):
                    new[hit.nonzero().view(-1).view(-1, 1), gi.view(1, -1)] = nv[hit].view(-1, 1)
        return new

    def crossover(self, a: torch.Tensor, b: torch.Tensor, gen: torch.Generator | None = None):
        """Single-point crossover of row pairs (PopulationSearchDomain.crossOverForPair :53-99,
        opti.py crossOver :660-682); points aligned to ``comp_size``.  Returns two children."""
        P, L = a.shape
        lo = max(1, self.comp_size)
        pt = lo + (torch.rand(P, generator=gen, device=a.device) * max(L - lo, 1)).long()
        pt = (pt // self.comp_size) * self.comp_size
        pt = pt.clamp(1, L - 1)
        left = torch.arange(L, device=a.device).view(1, -1) < pt.view(-1, 1)
        return torch.where(left, a, b), torch.where(left, b, a)


class AssignmentDomain(SearchDomain):
    """Assignment of one of V values (e.g. employees) to each of L positions (e.g. tasks).

    cost(s) = mean_l cost_table[l, s_l]; invalid iff two positions i, j with ``conflict[i, j]`` hold
    the same value.  (TaskScheduleSearch: J/examples/TaskScheduleSearch.java:169-305.)
    """

    def __init__(self, cost_table: torch.Tensor, conflict: torch.Tensor | None = None, invalid_cost: float = 150.0,
                 swap_moves: bool = True, values: Sequence | None = None):
        self.cost_table = cost_table.float().contiguous()
        L, V = self.cost_table.shape
        self.V = V
        self.cards = torch.full((L,), V, dtype=torch.long, device=cost_table.device)
        self.conflict = None if conflict is None else conflict.to(cost_table.device).bool()
        if self.conflict is not None:
            self.conflict = self.conflict & ~torch.eye(L, dtype=torch.bool, device=cost_table.device)
        self.invalid_cost = invalid_cost
        self.swap_moves = swap_moves
        self.values = list(values) if values is not None else list(range(V))

    def to(self, device) -> "AssignmentDomain":
        return AssignmentDomain(self.cost_table.to(device), self.conflict, self.invalid_cost, self.swap_moves, self.values)

    def cost(self, sol):
        return self.cost_table.gather(1, sol.t()).t().mean(1) if sol.numel() else torch.zeros(0, device=sol.device)

    def valid(self, sol):
        if self.conflict is None:
            return torch.ones(sol.shape[0], dtype=torch.bool, device=sol.device)
        same = sol.unsqueeze(2) == sol.unsqueeze(1)          # [P, L, L]
        return ~(same & self.conflict.unsqueeze(0)).flatten(1).any(1)

    def random(self, P, gen=None, max_try=10):
        """Position-by-position construction: each new position is redrawn until it conflicts with
        no earlier position (BasicSearchDomain.createSolution :245-255), all rows at once."""
        L, dev = self.L, self.device
        sol = torch.zeros((P, L), dtype=torch.long, device=dev)
        ok = torch.ones(P, dtype=torch.bool, device=dev)
        for l in range(L):
            todo = torch.arange(P, device=dev)
            for _ in range(max(max_try, 1) * 4):
                v = (torch.rand(todo.numel(), generator=gen, device=dev) * self.V).long().clamp_max(self.V - 1)
                sol[todo, l] = v
                if self.conflict is None or l == 0:
                    todo = todo[:0]
                    break
                clash = ((sol[todo, :l] == v.view(-1, 1)) & self.conflict[l, :l].view(1, -1)).any(1)
                todo = todo[clash]
                if todo.numel() == 0:
                    break
            ok[todo] = False
        return sol, ok & self.valid(sol)

    def neighbourhood_delta(self, sol: torch.Tensor) -> torch.Tensor:
        """Exact cost change of every single-position reassignment: [P, L, V] (no swap)."""
        cur = self.cost_table.gather(1, sol.t()).t()                       # [P, L]
        return (self.cost_table.unsqueeze(0) - cur.unsqueeze(2)) / self.L


class CallbackDomain(SearchDomain):
    """Wraps a reference-style domain object with scalar ``isValid(list)`` / ``evaluate(list)``
    (P/app/fesel.py:51-63, P/app/mesched.py) over per-position value tables.  Each candidate is
    decoded and evaluated on the host: use it for costs that run external programs or models."""

    def __init__(self, obj, value_tables: Sequence[Sequence], device="cpu", invalid_cost: float = float("inf"),
                 comp_size: int = 1):
        self.obj = obj
        self.tables = [list(t) for t in value_tables]
        self.cards = torch.tensor([len(t) for t in self.tables], dtype=torch.long, device=device)
        self.invalid_cost = invalid_cost
        self.comp_size = comp_size
        self.n_eval = 0

    def decode(self, sol):
        return [[self.tables[l][i] for l, i in enumerate(row)] for row in sol.tolist()]

    def valid(self, sol):
        if not hasattr(self.obj, "isValid"):
            return super().valid(sol)
        return torch.tensor([bool(self.obj.isValid(r)) for r in self.decode(sol)], device=sol.device)

    def cost(self, sol):
        self.n_eval += sol.shape[0]
        return torch.tensor([float(self.obj.evaluate(r)) for r in self.decode(sol)], device=sol.device)


class FunctionDomain(SearchDomain):
    """Vectorised user domain: ``cost_fn(values [P, L] float) -> [P]`` and optional
    ``valid_fn``; ``value_tables[l]`` lists the admissible values of position l."""

    def __init__(self, value_tables: Sequence[Sequence[float]], cost_fn: Callable, valid_fn: Callable | None = None,
                 device="cpu", groups=None, invalid_cost: float = float("inf"), comp_size: int = 1):
        dev = torch.device(device)
        Vmax = max(len(t) for t in value_tables)
        tab = torch.zeros((len(value_tables), Vmax), dtype=torch.float32)
        for l, t in enumerate(value_tables):
            tab[l, : len(t)] = torch.tensor([float(x) for x in t])
        self.table = tab.to(dev)
        self.cards = torch.tensor([len(t) for t in value_tables], dtype=torch.long, device=dev)
        self.cost_fn, self.valid_fn = cost_fn, valid_fn
        self.groups = groups
        self.invalid_cost = invalid_cost
        self.comp_size = comp_size

    def decode(self, sol):
        return self.table.gather(1, sol.t()).t()

    def cost(self, sol):
        return torch.as_tensor(self.cost_fn(self.decode(sol)), device=sol.device).float().view(-1)

    def valid(self, sol):
        if self.valid_fn is None:
            return super().valid(sol)
        return torch.as_tensor(self.valid_fn(self.decode(sol)), device=sol.device).bool().view(-1)
