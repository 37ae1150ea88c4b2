"""Manufacturing back-order causal model (P/app/back_order.py:24-262).

``simu``: weekly demand with trend and seasonality, parts ordered from the previous week's demand
plus a safety margin, a fixed weekly production capacity with the unmet quantity deferred to the
next week, back orders from either parts shortage or capacity, and the per-unit profit after
production, parts-premium and shipping costs.  The reference evaluates one week per callback and
carries the deferred quantity in the simulator's output list; here the whole horizon is one
vectorised pass — the deferred quantity is a Lindley recursion W_t = max(0, W_{t-1} + d_t − cap),
computed in closed form as S_t − min(0, min_{k<=t} S_k) with S = cumsum(d − cap).

``infer``: causal effect of back orders on profit by intervention on a trained regressor — the
back-order feature is set to each value for every row and the mean predicted profit reported
(``back_order_intervention``).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Sequence

import torch

SEASONAL = (-580, -340, 0, 370, 1250, 3230, 3980, 3760, 2770, 980, 120, -220)
TREND = (250, 350)


def ship_cost(q: torch.Tensor) -> torch.Tensor:
    """Shipping and handling: 1.6 / 1.3 / 1.1 per unit by quantity band, + 200."""
    return torch.where(q < 1000, 1.6 * q, torch.where(q < 2000, 1.3 * q, 1.1 * q)) + 200


@dataclass
class SupplyChainSimulation:
    demand_mean: float = 7000.0
    demand_sd: float = 1000.0
    capacity: int = 140 * 70                      # machine hours x products per machine-hour
    cost_per_unit: float = 30.0
    parts_cost_per_unit: float = 12.0
    other_cost_per_unit: float = 18.0
    price_per_unit: float = 50.0
    margins: Sequence[float] = (0.0, 0.04, 0.08, 0.12, 0.16, 0.20)
    margin_weights: Sequence[float] = (25, 30, 18, 10, 5, 2)
    seasonal: Sequence[int] = field(default_factory=lambda: SEASONAL)
    device: str = "cpu"
    seed: int = 0

    def simulate(self, weeks: int) -> torch.Tensor:
        """[weeks, 6]: previous demand, demand, downtime %, parts margin %, back order, unit profit."""
        dev = torch.device(self.device)
        g = torch.Generator(device=dev).manual_seed(self.seed)
        f64 = dict(dtype=torch.float64, device=dev)
        raw = self.demand_mean + self.demand_sd * torch.randn(weeks + 1, generator=g, **f64)
        dem_raw, pdem_raw = raw[1:].floor(), raw[:-1].floor()      # previous week's demand drives parts orders
        downtime = torch.distributions.Gamma(torch.tensor(1.0, **f64), torch.tensor(1 / 0.05, **f64)).sample((weeks,))
        w = torch.tensor(self.margin_weights, **f64)
        margin = torch.tensor(self.margins, **f64)[torch.multinomial(w / w.sum(), weeks, True, generator=g)]
        it = torch.arange(weeks, device=dev) % 260
        year = it // 52
        month = ((it % 52).double() / 4.33).long().clamp_max(11)
        tadj = torch.where(year <= 2, TREND[0] * year, TREND[0] * 2 + TREND[1] * (year - 2)).double()
        sadj = torch.tensor(self.seasonal, **f64)[month]
        dem = (dem_raw + tadj + sadj).floor()
        pdem = (pdem_raw + tadj + sadj).floor()
        parts = (pdem * (1 + margin)).floor()
        bo_parts = (dem - parts).clamp_min(0)
        s = torch.cumsum(dem - self.capacity, 0)
        deferred = s - torch.cummin(s, 0).values.clamp_max(0)              # Lindley recursion
        bo = torch.maximum(bo_parts, deferred)
        ro = dem - bo
        sc = ship_cost(ro) + torch.where(bo > 0, ship_cost(bo), torch.zeros_like(bo))
        premium = (bo_parts > 0) & (torch.rand(weeks, generator=g, **f64) < 0.4)
        pc = torch.where(premium, (dem - bo_parts) * self.cost_per_unit
                         + bo_parts * (1.1 * self.parts_cost_per_unit + self.other_cost_per_unit),
                         dem * self.cost_per_unit)
        rev = torch.where(bo > 0, ro * self.price_per_unit + bo * 0.9 * self.price_per_unit, dem * self.price_per_unit)
        prof = (rev - pc - sc) / dem
        return torch.stack([pdem, dem, downtime * 100, margin * 100, bo, prof], 1)

    @staticmethod
    def lines(sim: torch.Tensor) -> list[str]:
        return [f"{int(a)},{int(b)},{c:.3f},{d:.3f},{int(e)},{f:.2f}" for a, b, c, d, e, f in sim.tolist()]


def back_order_intervention(predict, X: torch.Tensor, col: int, values: Sequence[float],
                            scale: str | None = "zscale") -> list[tuple[float, float]]:
    """do(X[:, col] = v) for each v: mean of ``predict`` over all rows (back_order.py ``infer``).
    ``scale`` standardises the features as the regressor was trained ('zscale' / 'minmax' / None)."""
    X = X.double()
    xc = X[:, col]
    if scale == "zscale":
        me, sd = xc.mean(), xc.std(unbiased=False)
        sv = [(v - me) / sd for v in values]
        Xs = (X - X.mean(0)) / X.std(0, unbiased=False).clamp_min(1e-12)
    elif scale == "minmax":
        lo, hi = xc.min(), xc.max()
        sv = [(v - lo) / (hi - lo) for v in values]
        Xs = (X - X.min(0).values) / (X.max(0).values - X.min(0).values).clamp_min(1e-12)
    else:
        sv, Xs = list(values), X.clone()
    out = []
    for v, s in zip(values, sv):
        Xi = Xs.clone()
        Xi[:, col] = float(s)
        out.append((float(v), float(torch.as_tensor(predict(Xi.float())).double().mean())))
    return out
