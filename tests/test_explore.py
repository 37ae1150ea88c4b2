"""Exploratory analytics, encodings and re-sampling tests (CPU oracles; gpu parity)."""
import math

import numpy as np
import pytest
import torch

from avenir_amd.data import synth
from avenir_amd.data.table import load_csv
from avenir_amd.models import explore as E
from avenir_amd.models.sampling import AdaBoost, bagging_indices, relief, smote, undersample
from avenir_amd.utils.schema import FeatureSchema

from _dist import run_world


def _churn(tmp_path, n=3000, seed=0):
    p = tmp_path / "c.csv"
    synth.write_churn(p, n, seed=seed)
    return p, load_csv(p, FeatureSchema.from_json(synth.CHURN_SCHEMA))


def test_mutual_information_vs_sklearn(tmp_path):
    from sklearn.metrics import mutual_info_score
    _, t = _churn(tmp_path)
    mi = E.MutualInformation()
    r = mi.fit(t)
    y = t.labels[: t.n].numpy()
    for j, f in enumerate(t.binned_fields):
        ref = mutual_info_score(t.codes[j, : t.n].numpy(), y)
        assert r.feature_class[f.ordinal] == pytest.approx(ref, rel=1e-9, abs=1e-12)
    a, b = t.binned_fields[0].ordinal, t.binned_fields[1].ordinal
    ref = mutual_info_score(t.codes[0, : t.n].numpy(), t.codes[1, : t.n].numpy())
    assert r.feature_pair[(a, b)] == pytest.approx(ref, rel=1e-9, abs=1e-12)
    joint = t.codes[0, : t.n].long() * 10 + t.codes[1, : t.n].long()
    assert r.pair_class[(a, b)] == pytest.approx(mutual_info_score(joint.numpy(), y), rel=1e-9)
    for ranking in (mi.mim(), mi.mifs(), mi.jmi(), mi.disr(), mi.mrmr()):
        assert sorted(f for f, _ in ranking) == sorted(r.feature_class)
    # MIM ranks the strongest churn driver (minUsed / dataUsed multipliers) near the top
    assert mi.mim()[0][0] in (1, 2, 3)


def test_contingency_stats():
    tab = torch.tensor([[10.0, 20.0], [30.0, 40.0]])
    cs = E.ContingencyStats(tab)
    # phi^2 for a 2x2 table
    n = 100.0
    chi2 = cs.chi_square()[0]
    assert cs.cramer_index() == pytest.approx(chi2 / n, rel=1e-9)
    assert 0 <= cs.concentration_coeff() <= 1
    assert not math.isnan(cs.uncertainty_coeff())


def test_categorical_correlation_and_affinity(tmp_path):
    _, t = _churn(tmp_path)
    cc = E.categorical_correlation(t)
    assert len(cc) == 10 and all(v >= -1e-9 for v in cc.values())
    aff = E.class_affinity(t, "distrDiff", pos_class=1)
    assert set(aff) == {1, 2, 3, 4, 5}
    # overage raises churn in the generator: highest affinity for "closed" within minUsed
    assert aff[1][0][0] == "overage"


def test_supervised_encodings(tmp_path):
    p, t = _churn(tmp_path, 2000)
    enc = E.supervised_encoding(t, "supervisedRatio", scale=1000)
    lines = [ln.split(",") for ln in p.read_text().splitlines()]
    v = "high"
    pos = sum(1 for it in lines if it[2] == v and it[6] == "closed")
    tot = sum(1 for it in lines if it[2] == v)
    assert enc[2][v] == (pos * 1000) // tot
    woe = E.supervised_encoding(t, "weightOfEvidence", scale=100)
    assert all(isinstance(x, float) for x in woe[1].values())
    M = E.apply_encoding(t, enc)
    assert M.shape == (2000, 5)
    loo = E.leave_one_out_encoding(t, t.labels.float())
    assert loo.shape == (2000, 5)
    dummy, names = E.binary_dummy(t)
    assert dummy.shape[1] == 18 and int(dummy.sum()) == 2000 * 5
    fh = E.feature_hashing([["a", "b"], ["a", "c"]], 16)
    assert fh.shape == (2, 16) and float(fh.abs().sum()) == 4
    # Table / device variant == the string API over the same categorical values
    cats = [f for f in t.binned_fields if f.is_categorical]
    strs = [[f.bin_label(int(t.codes[j, i])) for j, f in enumerate(t.binned_fields) if f.is_categorical]
            for i in range(t.n)]
    assert torch.equal(E.feature_hashing_table(t, 32), E.feature_hashing(strs, 32))
    assert len(cats) == len(strs[0])


def test_numerical_correlation():
    g = torch.Generator().manual_seed(0)
    X = torch.randn(5000, 4, generator=g)
    X[:, 1] = X[:, 0] * 0.8 + 0.2 * X[:, 1]
    r = E.numerical_correlation(X)
    ref = torch.tensor(np.corrcoef(X.numpy().T))
    assert torch.allclose(r, ref, atol=1e-9)


def _rank_corr(rank, world, X):
    from avenir_amd.parallel.comm import get_comm
    n = X.shape[0]
    return E.numerical_correlation(X[rank * n // world:(rank + 1) * n // world], get_comm())


def test_numerical_correlation_distributed():
    X = torch.randn(1001, 3, generator=torch.Generator().manual_seed(2))
    ref = E.numerical_correlation(X)
    for r in run_world(_rank_corr, 2, X):
        assert torch.allclose(r, ref, atol=1e-10)


def test_rules_ks_eventtime(tmp_path):
    _, t = _churn(tmp_path, 1000)
    ev = E.RuleEvaluator({"r1": (lambda tt: tt.codes[0, : tt.n] == 3, 1)})
    res = ev.evaluate(t)["r1"]
    assert 0 < res["support"] < 1 and 0 <= res["confidence"] <= 1
    ks, crit, drift = E.kolmogorov_smirnov_drift(torch.tensor([10, 20, 30.0]), torch.tensor([30, 20, 10.0]))
    assert ks == pytest.approx(1 / 3) and drift is False or drift is True
    h = E.event_time_distribution(torch.tensor([0, 3600, 7200, 86400]), "hourOfDay")
    assert h[0] == 2 and h[1] == 1


def test_sampling_and_boosting():
    x, y = synth.supervised(600, 3, 2, seed=4)
    y[:500] = 0
    y[500:] = 1
    nx, _ = smote(x, y, 1, 200, k=3)
    assert nx.shape == (200, 3)
    keep = undersample(y)
    kept = y[keep]
    assert abs(int((kept == 0).sum()) - int((kept == 1).sum())) < 60
    bi = bagging_indices(100, 25)
    assert bi.shape == (100,) and int(bi[:25].max()) < 25
    ab = AdaBoost()
    w = torch.full((600,), 1 / 600)
    pred = y.clone()
    pred[:60] = 1 - pred[:60]
    e = ab.error(pred, y, w)
    assert e == pytest.approx(0.1)
    w2 = ab.update(pred, y, w, e)
    assert float(w2[:60].mean()) > float(w2[60:].mean())
    r = relief(x, y, k=2)
    assert r.shape == (3,)
