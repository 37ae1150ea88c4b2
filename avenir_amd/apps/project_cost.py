"""Project-cost confidence bounds by Monte-Carlo simulation (P/app/pccb.py:26-162).

The reference registers 14 samplers with ``MonteCarloSimulator`` and evaluates a Python callback
per iteration.  Here the callback is vectorised: one call prices all ``num_iter`` sampled
scenarios as tensor ops (task costs from member rates and participation shares, a Bernoulli
unexpected-work term, and per-member interruption costs over the elapsed days).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch

from ..models.montecarlo import MonteCarloSimulator


@dataclass
class ProjectCostModel:
    members: tuple = ("KD", "PL", "SP", "DJ", "DI", "PM")
    member_cost: dict = field(default_factory=lambda: {"KD": 55.0, "PL": 45.0, "SP": 35.0, "DJ": 30.0, "DI": 40.0,
                                                       "PM": 40.0})
    task_front: dict = field(default_factory=lambda: {"DJ": 60.0, "SP": 40.0})
    task_deploy: dict = field(default_factory=lambda: {"DI": 70.0, "PL": 20.0, "DJ": 10.0})
    task_mgmt: dict = field(default_factory=lambda: {"PM": 64.0, "KD": 12.0, "SP": 12.0, "DI": 12.0})
    replacement_cost: float = 40.0

    def rate(self, task: dict) -> float:
        """Cost per task hour: participation-weighted member rate (``taskCost`` / hours)."""
        return sum(self.member_cost[m] * p / 100.0 for m, p in task.items())

    def cost(self, X: torch.Tensor) -> torch.Tensor:
        """X [n, 14] columns: front, ML, ML-lead share, deploy, management hours, unexpected (0/1),
        unexpected hours, 6 per-member interruption counts (``prCost``, pccb.py:72-110)."""
        front, ml, lead, deploy, mgmt, unexp, unexp_h = (X[:, i].double() for i in range(7))
        intr = X[:, 7:13].double()
        elapsed_days = torch.floor(0.8 * (front + ml + deploy + mgmt) / 8) + 1
        ml_rate = (self.member_cost["KD"] * lead + self.member_cost["PL"] * (100.0 - lead - 10.0)
                   + self.member_cost["SP"] * 10.0) / 100.0
        c = front * self.rate(self.task_front) + ml * ml_rate + deploy * self.rate(self.task_deploy) \
            + mgmt * self.rate(self.task_mgmt) + unexp * unexp_h * self.replacement_cost
        rates = torch.tensor([self.member_cost[m] for m in self.members], dtype=torch.float64, device=X.device)
        c = c + 0.25 * elapsed_days * (intr * rates).sum(1)
        return c


def project_cost_simulation(num_iter: int, device="cpu", seed: int = 0,
                            model: ProjectCostModel | None = None) -> MonteCarloSimulator:
    """The reference's sampler set (pccb.py:121-138) on the device; returns the finished
    simulator (``getMean``, ``getStdDev``, ``getUpperTailStat``, ``getCritValue`` ...)."""
    m = model or ProjectCostModel()
    sim = MonteCarloSimulator(num_iter, lambda X, mm: mm.cost(X), device=device, seed=seed)
    sim.registerGaussianSampler(72.0, 8.0)
    sim.registerNonParametricSampler(40.0, 10.0, 20.0, 28.0, 40.0, 50.0, 60.0, 80.0, 90.0, 100.0, 80.0, 65.0, 50.0,
                                     35.0, 32.0, 40.0, 53.0, 70.0, 80.0, 85.0, 90.0, 82.0, 65.0, 45.0, 40.0, 35.0, 30.0,
                                     27.0)
    sim.registerTriangularSampler(52.0, 78.0, 60.0)
    sim.registerGaussianSampler(80.0, 12.0)
    sim.registerGaussianSampler(50.0, 5.0)
    sim.registerBernoulliTrialSampler(0.10)
    sim.registerGaussianSampler(10.0, 2.0)
    for rate in (5, 4, 2, 6, 3, 2):
        sim.registerPoissonSampler(rate)
    sim.registerExtraArgs(m)
    sim.run()
    return sim
