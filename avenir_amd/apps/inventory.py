"""Inventory planning under uncertain demand by MCMC (P/app/inv_sim.py:25-250).

Demand follows a histogram-shaped (non-parametric) density sampled with Metropolis; for each
candidate inventory level the earning of a period is
  surplus : demand x profit − (inventory − demand) x holding cost
  deficit : inventory x profit, a N(mean, sd) fraction of the shortfall is back-ordered (earns the
            profit, costs the back-order cost), the rest is lost (costs the profit).
The reference runs one chain per inventory level, one sample at a time.  Here every inventory
level gets its own chain and all chains advance together (one [levels] vector op per step, with
proposals and uniforms drawn up front), then the statistics — mean with its standard error,
upper percentile of the earning distribution, Geweke z-scores for burn-in choice — are tensor
reductions over the [steps, levels] sample matrix.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Sequence

import torch

from ..models.montecarlo import geweke_z


@dataclass
class InventorySimulation:
    demand_start: float
    demand_bin_width: float
    demand_weights: Sequence[float]
    proposal_sd: float
    profit_per_unit: float
    holding_cost_per_unit: float
    back_order_mean: float
    back_order_sd: float
    back_order_cost_per_unit: float
    device: str = "cpu"
    seed: int = 0

    @classmethod
    def from_config(cls, cfg: dict, device="cpu", seed: int = 0) -> "InventorySimulation":
        """Keys of the reference's inv_sim properties (inv_sim.py:226-237)."""
        w = [float(v) for v in str(cfg["demand.distr"]).split(",")]
        return cls(float(cfg["demand.distr.start"]), float(cfg["demand.distr.bin.width"]), w,
                   float(cfg["proposal.distr.std"]), float(cfg["profit.per.unit"]),
                   float(cfg["holding.cost.per.unit"]), float(cfg["back.order.distr.mean"]),
                   float(cfg["back.order.distr.std"]), float(cfg["back.order.cost.per.unit"]), device, seed)

    def _log_density(self, x: torch.Tensor) -> torch.Tensor:
        w = torch.tensor(self.demand_weights, dtype=torch.float64, device=x.device)
        k = torch.floor((x - self.demand_start) / self.demand_bin_width).long()
        inside = (k >= 0) & (k < len(self.demand_weights))
        return torch.where(inside, torch.log(w[k.clamp(0, len(w) - 1)]), torch.full_like(x, -torch.inf))

    def demand_chains(self, steps: int, chains: int) -> tuple[torch.Tensor, float]:
        """Metropolis samples [steps, chains] of the demand density and the acceptance rate."""
        dev = torch.device(self.device)
        g = torch.Generator(device=dev).manual_seed(self.seed)
        hi = self.demand_start + self.demand_bin_width * len(self.demand_weights)
        x = self.demand_start + (hi - self.demand_start) * torch.rand(chains, dtype=torch.float64, device=dev,
                                                                        generator=g)
        step = self.proposal_sd * torch.randn((steps, chains), dtype=torch.float64, device=dev, generator=g)
        logu = torch.log(torch.rand((steps, chains), dtype=torch.float64, device=dev, generator=g))
        out = torch.empty((steps, chains), dtype=torch.float64, device=dev)
        lp = self._log_density(x)
        acc = torch.zeros((), dtype=torch.float64, device=dev)
        for t in range(steps):
            prop = x + step[t]
            lq = self._log_density(prop)
            a = logu[t] < lq - lp
            x = torch.where(a, prop, x)
            lp = torch.where(a, lq, lp)
            acc += a.sum()
            out[t] = x
        return out, float(acc) / (steps * chains)

    def earnings(self, demand: torch.Tensor, inventory: torch.Tensor) -> torch.Tensor:
        """Per-period earning for demand [steps, L] against inventory levels [L] (``get_earning``)."""
        dem = torch.floor(demand)
        inv = inventory.to(demand).view(1, -1).expand_as(dem)
        g = torch.Generator(device=demand.device).manual_seed(self.seed + 1)
        frac = self.back_order_mean + self.back_order_sd * torch.randn(dem.shape, dtype=torch.float64,
                                                                        device=demand.device, generator=g)
        p, h, b = self.profit_per_unit, self.holding_cost_per_unit, self.back_order_cost_per_unit
        surplus = dem * p - (inv - dem) * h
        short = dem - inv
        bo = short * frac
        lost = short - bo
        deficit = inv * p + bo * p - (lost * p + bo * b)
        return torch.where(inv >= dem, surplus, deficit)

    def run(self, inventories: Sequence[int], sample_size: int, burn_in: int) -> dict:
        """Mean earning, its standard error and surplus / deficit counts per inventory level
        (``earning_mean``)."""
        inv = torch.tensor(list(inventories), dtype=torch.float64, device=torch.device(self.device))
        dem, acc = self.demand_chains(sample_size, len(inv))
        e = self.earnings(dem, inv)[burn_in:]
        n = e.shape[0]
        excess = (inv.view(1, -1) >= torch.floor(dem)).sum(0)
        return {"inventory": list(inventories), "mean": e.mean(0).tolist(),
                "stderr": (e.std(0, unbiased=False) / n ** 0.5).tolist(), "excess_count": excess.tolist(),
                "deficit_count": (sample_size - excess).tolist(), "acceptance": acc, "earnings": e}

    def percentile(self, inventories: Sequence[int], sample_size: int, burn_in: int, pct: float) -> list[float]:
        """Earning exceeded with probability ``pct`` per inventory level (``earning_percentile``)."""
        e = self.run(inventories, sample_size, burn_in)["earnings"]
        return torch.quantile(e, 1.0 - pct, dim=0).tolist()

    def geweke(self, inventory: int, sample_sizes: Sequence[int], burn_ins: Sequence[int]) -> list[tuple]:
        """(sample size, burn-in, z) per combination (``gweke_conv``): all chains at once."""
        m = max(sample_sizes)
        dem, _ = self.demand_chains(m, 1)
        e = self.earnings(dem, torch.tensor([float(inventory)]))[:, 0]
        out = []
        for s in sample_sizes:
            for b in burn_ins:
                if b < s:
                    out.append((s, b, geweke_z(e[b:s])))
        return out
