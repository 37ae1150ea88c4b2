"""More search domains: taxi fleet assignment and learning-parameter search.

* ``TaxiFleetAssignment`` (J/examples/TaxiFleetAssignment.java:145-266, R/taxiFleet.json; the
  reference is a tabu-search stub whose cost functions are unfinished): passengers -> distinct
  taxis; cost of a pair = pickup distance (haversine, miles) + ``earning_weight`` x the taxi's
  normalised earnings today (spread work across the fleet); every pair of passengers conflicts on
  the same taxi (all-different), the reference's passenger-swap move is the domain's swap move.
  Compiled into an :class:`AssignmentDomain`, so SA runs in the K22 kernel and tabu search scores
  the full neighbourhood in closed form.
* ``LearningParameterSearch`` (J/examples/LearningParameterSearch.java:60-134): hyper-parameter
  space from JSON (string values / int or float ranges); the cost of a candidate runs an external
  command with ``name=value`` arguments and extracts the metric from stdout with a regex.
  Candidates run as subprocesses (no shell), optionally several at once.
"""
from __future__ import annotations

import json
import re
import subprocess
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from typing import Sequence

import torch

from .domain import AssignmentDomain, SearchDomain
from .domains import geo_distance, read_lenient_json


class TaxiFleetAssignment(AssignmentDomain):
    def __init__(self, fleet: dict, earning_weight: float = 0.0, device="cpu"):
        self.fleet = fleet
        taxis, pax = fleet["taxis"], fleet["passengers"]
        if len(pax) > len(taxis):
            raise ValueError("more passengers than taxis")
        self.taxi_ids = [t["id"] for t in taxis]
        self.passenger_ids = [p["id"] for p in pax]
        tl = torch.tensor([t["currentLocation"] for t in taxis], dtype=torch.float64)
        pl = torch.tensor([p["currentLocation"] for p in pax], dtype=torch.float64)
        dist = geo_distance(pl[:, 0:1], pl[:, 1:2], tl[:, 0].view(1, -1), tl[:, 1].view(1, -1))    # [P, T]
        earn = torch.tensor([float(t.get("earningToday", 0.0)) for t in taxis], dtype=torch.float64)
        earn = (earn - earn.min()) / (earn.max() - earn.min()).clamp_min(1e-12)
        cost = dist + earning_weight * earn.view(1, -1)
        P = len(pax)
        conflict = ~torch.eye(P, dtype=torch.bool)
        super().__init__(cost.float().to(device), conflict.to(device), invalid_cost=1e6, swap_moves=True,
                         values=self.taxi_ids)

    @classmethod
    def from_json(cls, path, **kw):
        return cls(read_lenient_json(path), **kw)

    def assignment(self, row: Sequence[int]) -> list[tuple[str, str]]:
        return [(p, self.taxi_ids[int(t)]) for p, t in zip(self.passenger_ids, row)]


class LearningParameterSearch(SearchDomain):
    """Parameter space JSON: {"commands": [...], "execDir": "...", "outputPattern": "...",
    "parameters": [{"name", "type": "string|int|float", "values": [...]}, ...]}.  int / float
    parameters with two values are [min, max] ranges, discretised into ``grid`` steps."""

    def __init__(self, space: dict, grid: int = 10, workers: int = 1, device="cpu"):
        self.space = space
        self.cmd = list(space["commands"])
        self.exec_dir = space.get("execDir")
        self.pattern = re.compile(space["outputPattern"], re.DOTALL)
        self.names, self.tables = [], []
        for p in space["parameters"]:
            vals = p["values"]
            if p["type"] == "string":
                tab = list(vals)
            elif p["type"] == "int":
                lo, hi = int(vals[0]), int(vals[1])
                tab = [str(v) for v in range(lo, hi + 1)] if hi - lo < 1000 else \
                    [str(int(lo + (hi - lo) * i / (grid - 1))) for i in range(grid)]
            elif p["type"] == "float":
                lo, hi = float(vals[0]), float(vals[1])
                tab = [repr(lo + (hi - lo) * i / (grid - 1)) for i in range(grid)]
            else:
                raise ValueError("invalid parameter type")
            self.names.append(p["name"])
            self.tables.append(tab)
        self.cards = torch.tensor([len(t) for t in self.tables], dtype=torch.long, device=device)
        self.workers = workers
        self.history: list[tuple[dict, float]] = []

    @classmethod
    def from_json(cls, path, **kw):
        return cls(json.loads(Path(path).read_text()), **kw)

    def decode(self, sol):
        return [{n: self.tables[l][i] for l, (n, i) in enumerate(zip(self.names, row))} for row in sol.tolist()]

    def _run(self, params: dict) -> float:
        args = self.cmd + [f"{k}={v}" for k, v in params.items()]
        res = subprocess.run(args, cwd=self.exec_dir, capture_output=True, text=True, timeout=3600)
        m = self.pattern.search(res.stdout)
        if not m:
            raise RuntimeError(f"failed to extract metric from output of {args}")
        c = float(m.group(1))
        self.history.append((params, c))
        return c

    def cost(self, sol):
        cands = self.decode(sol)
        if self.workers > 1:
            with ThreadPoolExecutor(self.workers) as ex:
                costs = list(ex.map(self._run, cands))
        else:
            costs = [self._run(c) for c in cands]
        return torch.tensor(costs, dtype=torch.float32, device=sol.device)
