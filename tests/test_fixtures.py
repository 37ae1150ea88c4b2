"""Tutorial fixture generators (P/app/*.py): field layout, seed determinism, label rates."""
import numpy as np
import pytest

from avenir_amd.data import fixtures as F

CASES = {
    "advt": ((20, 10, 15, 30, 1), 7),
    "atm_xaction": ((5, 14, 10), 3),
    "cs_escalate": ((400, 0.05), 9),
    "cust_seg": ((300, 10), 6),
    "cust_value": ((300,), 5),
    "elearn": ((300,), 11),
    "exp_prod_price": ((10,), 2),
    "freq_items": ((100, 10, 200), None),
    "heart_disease": ((500, 0.05), 11),
    "lead_time": ((300,), 5),
    "loan_approve": ((200,), 13),
    "machine_op": ((300,), 9),
    "pat": ((300,), 5),
    "power": ((3,), 2),
    "prot_seq": ((50, 20, 40, 10), 2),
    "prsale": ((5,), 5),
    "ranproj": ((16, 20), 16),
    "retarget": ((300,), 4),
    "sales_lead": ((400,), 12),
    "supplier": ((6, 4), 3),
    "telecom_churn": ((400, 30, 5), 7),
    "visit_history": ((100, 30), None),
    "lat_long": ((50, 37.0, -122.0, 38.0, -121.0), 2),
    "hosp_readmit": ((400,), 12),
    "disease": ((400,), 8),
    "event_seq": ((100,), None),
    "buy_xaction": ((50, 20, 0.3), 4),
    "id_gen": ((20, 12), 1),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_fixture_layout_and_determinism(name):
    args, nfields = CASES[name]
    a = F.FIXTURES[name](*args, seed=3)
    b = F.FIXTURES[name](*args, seed=3)
    assert a == b and len(a) > 0
    if nfields is not None:
        assert all(len(r.split(",")) == nfields for r in a), a[:3]
    c = F.FIXTURES[name](*args, seed=4)
    assert c != a


def test_heart_disease_class_rate_and_conditionals():
    rows = [r.split(",") for r in F.heart_disease(20000, 0.0, seed=1)]
    y = np.array([r[-1] for r in rows])
    assert abs((y == "1").mean() - 0.25) < 0.02
    chol = np.array([float(r[2]) for r in rows])
    assert chol[y == "1"].mean() > chol[y == "0"].mean() + 25      # N(190, 8) vs N(150, 15)


def test_sales_lead_and_telecom_rates():
    y = np.array([r.split(",")[-1] for r in F.sales_lead(20000, seed=2)])
    rate = (y == "1").mean()
    assert 0.05 < rate < 0.95
    rows = [r.split(",") for r in F.telecom_churn(20000, 30, 0, seed=2)]
    churn = np.array([int(r[-1]) for r in rows])
    assert abs(churn.mean() - 0.29) < 0.03        # randint(1,100) < 30 -> 29 %


def test_truncated_normal_bounds():
    rng = np.random.default_rng(0)
    x = F._tnorm(rng, 10.0, 2.0, 100000)
    assert x.min() >= 4.0 and x.max() <= 16.0 and abs(x.mean() - 10) < 0.05


def test_dummy_vars_expand_columns():
    rows = F.pat(50, seed=1)
    d = F.dummy_vars(rows, F.PAT_DUMMY)
    assert all(len(r.split(",")) == 2 + 3 + 3 + 4 for r in d)
    for r0, r1 in zip(rows, d):
        a, b = r0.split(","), r1.split(",")
        assert b[2 + ["Y", "M", "O"].index(a[2])] == "1" and sum(v == "1" for v in b[2:5]) == 1


def test_exp_prod_price_pipeline():
    disc = F.exp_prod_price_discounts(4, seed=1)
    model = F.exp_prod_price_model(disc, seed=1)
    assert len(model) == len(disc) == 16
    rew = F.exp_prod_price_reward(model, disc[:5], seed=1)
    assert len(rew) == 5 and all(len(r.split(",")) == 3 for r in rew)


def test_price_opt_revenue_peaks():
    prices, stats = F.price_opt(6, seed=1)
    assert len(prices) == len(stats) > 0
    by = {}
    for s in stats:
        p, pr, rev = s.split(",")
        by.setdefault(p, []).append(int(rev))
    for revs in by.values():
        k = int(np.argmax(revs))
        assert all(revs[i] <= revs[i + 1] + 40 for i in range(k))   # rises to the peak (up to jitter)


def test_ruby_generators_rates_and_pipeline():
    rows = [r.split(",") for r in F.hosp_readmit(20000, seed=1)]
    low = np.mean([r[11] == "Y" for r in rows if r[8] == "low"])
    high = np.mean([r[11] == "Y" for r in rows if r[8] == "high"])
    assert 0.05 < high < low < 0.9                      # low follow-up adds 8 points of risk
    d = [r.split(",") for r in F.disease(20000, seed=2)]
    young = np.mean([r[7] == "Yes" for r in d if int(r[1]) < 40])
    old = np.mean([r[7] == "Yes" for r in d if int(r[1]) >= 70])
    assert young < old
    ev = F.event_seq(200, seed=3)
    assert all(len(e.split(",")) >= 6 and set(e.split(",")[1:]) <= set(F.EVENT_STATES) for e in ev)
    xs = F.buy_xaction(40, 120, 0.5, seed=4)
    by = {}
    for ln in xs:
        c, _, date, amt = ln.split(",")
        by.setdefault(c, []).append((np.datetime64(date), int(amt)))
    for h in by.values():                               # the script's amount rules
        assert 40 <= h[0][1] <= 219
        for (d0, a0), (d1, a1) in zip(h, h[1:]):
            gap = int((d1 - d0).astype(int))
            if gap < 30:
                assert (40 <= a1 <= 59) if a0 < 40 else (25 <= a1 <= 34)
    seqs = F.xaction_seq(xs)
    assert seqs and all(set(s.split(",")[1:]) <= set(F.MARK_STATES) for s in seqs)
    hist = [c + "," + ",".join(f"{d},{a}" for d, a in h) for c, h in by.items()]
    st = F.xaction_state(hist)
    assert len(st) == sum(len(h) >= 2 for h in by.values())
    model = np.eye(9, dtype=int) * 5 + 1
    plan = F.mark_plan(xs, model)
    assert len(plan) == sum(len(h) >= 2 for h in by.values())
    c, date = plan[0].split(", ")
    last = by[c][-1][0]
    assert int((np.datetime64(date) - last).astype(int)) in (15, 45, 90)


def test_elearn_int_fields_for_entity_schema():
    rows = [r.split(",") for r in F.elearn(50, seed=3, as_int=True)]
    assert all(len(r) == 11 and all(v.lstrip("-").isdigit() for v in r[1:10]) and r[10] in "PF" for r in rows)
