"""Application simulations (pccb / inv_sim / back_order): vectorised formulas vs scalar oracles
written from the reference's per-record callbacks."""
import math

import torch

from avenir_amd.apps import (InventorySimulation, ProjectCostModel, SupplyChainSimulation, back_order_intervention,
                             project_cost_simulation)


def _pr_cost_scalar(args, m: ProjectCostModel):
    front, ml, lead, deploy, mgmt, unexp, unexp_h = args[:7]
    intr = args[7:13]
    days = int(0.8 * (front + ml + deploy + mgmt) / 8) + 1

    def task(t, h):
        return sum(m.member_cost[k] * h * v / 100.0 for k, v in t.items())
    c = task(m.task_front, front)
    c += task({"KD": lead, "PL": 100.0 - lead - 10.0, "SP": 10.0}, ml)
    c += task(m.task_deploy, deploy) + task(m.task_mgmt, mgmt)
    if unexp:
        c += unexp_h * m.replacement_cost
    c += sum(0.25 * days * intr[i] * m.member_cost[m.members[i]] for i in range(6))
    return c


def test_project_cost_matches_scalar_callback():
    sim = project_cost_simulation(2000, seed=1)
    m = ProjectCostModel()
    X = sim._draw(16, 0)
    vec = m.cost(X)
    for i in range(16):
        assert math.isclose(float(vec[i]), _pr_cost_scalar([float(v) for v in X[i]], m), rel_tol=1e-9)
    assert 10000 < sim.getMean() < 40000 and sim.getStdDev() > 0


def _inv_sim():
    return InventorySimulation(demand_start=0, demand_bin_width=10,
                               demand_weights=[7, 12, 22, 16, 13, 10, 8, 12, 19, 23, 27, 34, 25, 18, 12, 5, 2],
                               proposal_sd=15, profit_per_unit=10, holding_cost_per_unit=2, back_order_mean=0.4,
                               back_order_sd=0.05, back_order_cost_per_unit=3, seed=3)


def test_inventory_chain_matches_target_density():
    s = _inv_sim()
    d, acc = s.demand_chains(6000, 64)
    d = d[500:].reshape(-1)
    w = torch.tensor(s.demand_weights, dtype=torch.float64)
    hist = torch.histc(d, bins=len(w), min=0, max=10 * len(w))
    emp = hist / hist.sum()
    assert (emp - w / w.sum()).abs().max() < 0.02
    assert 0.1 < acc < 0.95


def test_inventory_earnings_formula():
    s = _inv_sim()
    dem = torch.tensor([[50.0], [120.0]], dtype=torch.float64)
    e = s.earnings(dem, torch.tensor([100.0]))
    assert math.isclose(float(e[0, 0]), 50 * 10 - 50 * 2)
    # deficit: 100 sold; 20 short, back-ordered fraction f ~ N(0.4, 0.05)
    f = (float(e[1, 0]) - (100 * 10 - 20 * 10)) / (20 * (10 + 10 - 3))
    assert 0.2 < f < 0.6
    r = s.run([60, 100, 140], 3000, 300)
    assert len(r["mean"]) == 3 and all(v > 0 for v in r["stderr"])
    p = s.percentile([60, 100, 140], 3000, 300, 0.9)
    assert all(pv <= mv for pv, mv in zip(p, r["mean"]))   # 10th percentile below the mean
    z = s.geweke(100, [2000, 4000], [100, 500])
    assert len(z) == 4 and all(math.isfinite(v[2]) for v in z)


def test_supply_lindley_deferred_quantity_matches_loop():
    sim = SupplyChainSimulation(seed=5).simulate(520)
    pdem, dem, _, _, bo, prof = sim.T
    cap = 140 * 70
    deferred, prev = [], 0.0
    for d in dem.tolist():
        r = d + prev
        prev = r - cap if r > cap else 0.0
        deferred.append(prev)
    deferred = torch.tensor(deferred, dtype=torch.float64)
    assert torch.all(bo >= deferred - 1e-9)
    assert torch.isfinite(prof).all() and (bo >= 0).all()
    assert len(SupplyChainSimulation.lines(sim[:3])) == 3


def test_back_order_intervention_monotone_on_linear_model():
    X = torch.randn(500, 5, dtype=torch.float64)
    out = back_order_intervention(lambda Z: -2.0 * Z[:, 4], X, 4, [0.0, 1.0, 2.0], scale=None)
    assert [round(v, 6) for _, v in out] == [0.0, -2.0, -4.0]
