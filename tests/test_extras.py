"""Split statistics, cost arbitration, one-class SVM, model predictor, extra optimiser domains,
forecaster, semantic search, misc helpers."""
import json
import math
import sys

import numpy as np
import pytest
import torch

from avenir_amd.analytics.forecast import AdditiveForecaster
from avenir_amd.data import synth
from avenir_amd.data.table import load_csv
from avenir_amd.models import splitstat as SS
from avenir_amd.models.cost import CostBasedArbitrator, CostSchema
from avenir_amd.models.svm import OneClassSVM
from avenir_amd.optimize import SimulatedAnnealing, TabuSearch
from avenir_amd.optimize.apps import LearningParameterSearch, TaxiFleetAssignment
from avenir_amd.text.semsearch import ALGOS, SemanticSearch, hashing_embedder
from avenir_amd.utils import misc as M
from avenir_amd.utils.schema import FeatureSchema


def test_split_stat_algorithms():
    # 2 splits x 2 segments x 2 classes
    c = torch.tensor([[[40, 10], [10, 40]], [[25, 25], [25, 25]]], dtype=torch.float64)
    ent = SS.split_stat(c, "entropy")
    assert ent[0] < ent[1] and float(ent[1]) == pytest.approx(1.0)
    gini = SS.split_stat(c, "giniIndex")
    assert float(gini[1]) == pytest.approx(0.5)
    h = SS.split_stat(c, "hellingerDistance")
    p0, p1 = np.array([0.8, 0.2]), np.array([0.2, 0.8])
    assert float(h[0]) == pytest.approx(math.sqrt(((np.sqrt(p0) - np.sqrt(p1)) ** 2).sum()))
    assert float(h[1]) == pytest.approx(0.0)
    ccr = SS.split_stat(c, "classConfidenceRatio")
    assert float(ccr[1]) == pytest.approx(1.0) and ccr[0] < 1.0
    assert float(SS.split_info(c)[0]) == pytest.approx(1.0)
    with pytest.raises(ValueError):
        SS.split_stat(torch.ones(1, 2, 3), "hellingerDistance")


def test_class_partition_stats(tmp_path):
    p = tmp_path / "h.csv"
    p.write_text("\n".join(synth.call_hangup_lines(2000, seed=1)) + "\n")
    t = load_csv(p, FeatureSchema.from_json(synth.CALL_HANGUP_SCHEMA), raw_numeric=True)
    stats = SS.class_partition_stats(t, "entropy")
    assert len(stats) > 5
    for s in stats[:20]:
        assert s["counts"].sum() == 2000
        assert s["gain"] >= -1e-9
    best = max(stats, key=lambda s: s["gain"])
    assert best["gain"] > 0.01
    lines = SS.partition_lines(stats)
    assert lines[0].count(",") >= 2
    num = [s for s in stats if ":" in s["key"] or s["key"].replace(".", "").isdigit()]
    assert num


def test_cost_arbitrator_and_schema(ref_resource):
    a = CostBasedArbitrator("N", "Y", false_neg_cost=5, false_pos_cost=3)
    assert a.arbitrate(40, 60) == "Y"            # pos cost 3*60+40=220 < neg cost 5*40+60=260
    assert a.arbitrate(5, 95) == "N"             # pos cost 290 > neg cost 120
    assert a.classify(40) == "Y" and a.classify(30) == "N"      # threshold 300 // 8 = 37
    assert a.classify(torch.tensor([30, 40])).tolist() == [False, True]
    cs = CostSchema.from_json(ref_resource("churnPreventCost.json"))
    assert cs.findCost(4, 2.0) == -200.0
    assert cs.findCost(1, "a", "b") == 0.0
    assert torch.allclose(cs.batch_cost([4, 6], torch.tensor([[1.0, 1.0]])), torch.tensor([900.0]))


def test_one_class_svm():
    g = torch.Generator().manual_seed(0)
    X = torch.randn((300, 2), generator=g)
    oc = OneClassSVM(nu=0.1, gamma=0.5).fit(X)
    pred = oc.predict(X)
    frac_out = float((pred == -1).float().mean())
    assert 0.03 < frac_out < 0.2
    far = torch.tensor([[6.0, 6.0], [-5.0, 4.0]])
    assert (oc.predict(far) == -1).all()
    assert int(oc.predict(torch.zeros(1, 2))) == 1


def test_model_predictor_and_deterministic(tmp_path):
    from avenir_amd.models.supervised import (DeterministicPredictiveModel, LogisticRegressionClassifier,
                                              ModelPredictor)
    from avenir_amd.models.tree import RandomForest, TreeParams
    p = tmp_path / "h.csv"
    p.write_text("\n".join(synth.call_hangup_lines(1500, seed=3)) + "\n")
    schema = FeatureSchema.from_json(synth.CALL_HANGUP_SCHEMA)
    t = load_csv(p, schema, raw_numeric=True, keep_lines=True)
    rf = RandomForest(schema, 3, TreeParams(binary=True, stopping="maxDepth", max_depth=3,
                                            sub_sampling="withReplace", attr_selection="randomAll")).fit(t)
    files = []
    for i, tr in enumerate(rf.trees):
        f = tmp_path / f"t{i}.json"
        f.write_text(json.dumps(tr.state()))
        files.append(f)
    mp = ModelPredictor.from_state_files(files, schema, output_mode="withActualClassAttr")
    lines = mp.predict_lines(t)
    assert len(lines) == 1500 and lines[0].count(",") == 2
    assert mp.error_rate() < 0.5
    X = np.random.default_rng(0).normal(size=(200, 2)).astype(np.float32)
    y = (X[:, 0] > 0).astype(int)
    dm = DeterministicPredictiveModel(LogisticRegressionClassifier(device="cpu").fit(X, y)).enableErrorCounting()
    dm.predict(X, y)
    assert dm.getError() < 0.1


def test_taxi_fleet(ref_resource):
    d = TaxiFleetAssignment.from_json(ref_resource("taxiFleet.json"))
    assert d.L == len(d.passenger_ids) and d.V == len(d.taxi_ids)
    r = TabuSearch(d, n_chains=8, iters=100).run()
    row = r.best.tolist()
    assert len(set(row)) == len(row)                     # distinct taxis
    greedy_lb = float(d.cost_table.min(1).values.mean())
    assert r.best_cost >= greedy_lb - 1e-6
    sa = SimulatedAnnealing(d, n_chains=32, iters=2000, t0=0.5, cooling=0.995, interval=5).run()
    assert sa.best_cost <= r.best_cost * 1.2 and len(set(sa.best.tolist())) == len(row)
    assert d.assignment(row)[0][0] == d.passenger_ids[0]


def test_learning_parameter_search(tmp_path):
    script = tmp_path / "model.py"
    script.write_text("import sys\nkv = dict(a.split('=') for a in sys.argv[1:])\n"
                      "err = (int(kv['depth']) - 5) ** 2 * 0.01 + abs(float(kv['lr']) - 0.3)\n"
                      "print(f'validation error: {err:.4f}')\n")
    space = {"commands": [sys.executable, str(script)], "outputPattern": r"validation error: ([0-9.]+)",
             "parameters": [{"name": "depth", "type": "int", "values": ["2", "8"]},
                            {"name": "lr", "type": "float", "values": ["0.1", "0.5"]}]}
    d = LearningParameterSearch(space, grid=5, workers=4)
    from avenir_amd.optimize import RandomSearch
    r = RandomSearch(d, n=12, local="focussed", local_iters=6).run()
    best = d.decode(r.best.view(1, -1))[0]
    assert r.best_cost < 0.2 and len(d.history) >= 12
    assert set(best) == {"depth", "lr"}


def test_forecaster(tmp_path):
    day = 86400.0
    t = torch.arange(0, 400, dtype=torch.float64) * day
    y = 10 + 0.02 * (t / day) + 3 * torch.sin(2 * math.pi * t / (7 * day))
    y[200:] += 0.05 * (t[200:] / day - 200)                # changepoint
    y = y + 0.1 * torch.randn(400, generator=torch.Generator().manual_seed(0), dtype=torch.float64)
    f = AdditiveForecaster(n_changepoints=20, yearly=0, weekly=3).fit(t[:350], y[:350])
    v = f.validate(t[350:], y[350:])
    assert v["rmse"] < 1.0
    p = tmp_path / "fc.ckpt"
    f.save(p)
    g = AdditiveForecaster.load(p)
    assert torch.allclose(g.predict(t[350:])["yhat"], f.predict(t[350:])["yhat"])
    assert f.future_times(7).shape == (7,)


def test_semantic_search():
    docs = ["The GPU kernel streams tiles through local memory. Matrix cores multiply tiles quickly.",
            "Bananas and apples are sold at the fruit market. Oranges are juicy fruit.",
            "Storms bring rain and wind. The weather forecast says cloudy skies."]
    ss = SemanticSearch(hashing_embedder(128))
    for d in docs:
        ss.add(d)
    for algo in ALGOS:
        top = ss.search("fruit market apples", algo, top=3)
        assert len(top) == 3
        if algo not in ("tokenMed",):         # median of near-orthogonal random vectors is noise
            assert top[0][0] == 1, algo


def test_misc_helpers():
    ids = M.gen_ids(50, 8, seed=1)
    assert len(set(ids)) == 50 and all(len(i) == 8 for i in ids)
    loc = M.rand_location(37.7, -122.4, 5.0, n=100)
    assert loc.shape == (100, 2) and float((loc[:, 0] - 37.7).abs().max()) < 0.1
    sf = M.StepFunction((0, 10, 1.0), (10, 20, 2.0))
    assert sf.find(5) == 1.0 and sf.find(15) == 2.0 and sf.find(-3) == 1.0 and sf.find(30) == 2.0
    dv = M.DummyVarGenerator(3, {1: ["a", "b", "c"]})
    assert dv.processRow("x,b,3") == "x,0,1,0,3"
    lines = [f"r{i},{w}" for i, w in enumerate([0.0, 1.0, 0.0, 3.0])]
    s = M.weighted_record_sample(lines, 1, 400)
    assert all(l.startswith(("r1", "r3")) for l in s)
    assert M.pac_num_samples(1000, 0.1, 0.05) == int(math.log(1000 / 0.05) / 0.1)
    assert M.terms_hyp_space([2, 3], 2) == 3 * 4 * 2
    assert M.disjunctive_hyp_space([2, 2, 2], 2, 3, 1) == 8 * 2
    assert M.conjunctive_hyp_space_ln([2, 2], 2, 2) == pytest.approx(4 * math.log(2) + math.log(2))


def test_score_model_generator(tmp_path):
    from avenir_amd.data.generators import class_conditional, loan_approval
    from avenir_amd.models.bayes import NaiveBayes
    m = loan_approval()
    cols, label, score = m.generate(20000, seed=1)
    assert 0.2 < float(label.float().mean()) < 0.8
    assert float(cols["income"].min()) >= 50 and float(cols["income"].max()) <= 160
    lines = m.lines(500, seed=2)
    assert len(lines) == 500 and lines[0].count(",") == 12
    # the generated data is learnable: NB over the schema beats the majority rate
    f = tmp_path / "loan.csv"
    f.write_text("\n".join(m.lines(5000, seed=3)) + "\n")
    sch = m.schema("approved")
    for fd in sch["fields"]:
        if fd.get("dataType") == "int":
            fd["bucketWidth"] = max(1, int((fd["max"] or 100) - (fd["min"] or 0)) // 10) if fd["max"] else 5
            fd["min"] = fd["min"] or 0
            fd["max"] = fd["max"] or 60
    t = load_csv(f, FeatureSchema.from_json(sch))
    nb = NaiveBayes(t.schema).fit(t)
    r = nb.predict(t)
    acc = float((r.pred.long() == t.labels[: t.n].long()).float().mean())
    maj = max(float(t.labels[: t.n].float().mean()), 1 - float(t.labels[: t.n].float().mean()))
    assert acc > maj + 0.05
    cols2, y = class_conditional([60, 40], {"status": [("cat", ["m", "s"], [100, 20]), ("cat", ["m", "s"], [20, 100])],
                                            "income": [("num", 120, 10), ("num", 80, 10)]}, 4000)
    assert float(cols2["income"][y == 0].mean()) > float(cols2["income"][y == 1].mean()) + 30


def test_corpus_embedder_retrieval():
    """Corpus-trained embedder (parity unpinned vs ssearch.py's BERT): queries made of topic words
    retrieve documents of that topic."""
    import random as _r
    from avenir_amd.text.semsearch import search_corpus
    rng = _r.Random(4)
    topics = [[f"{p}{i}" for i in range(12)] for p in ("gpu", "fruit", "storm")]
    docs, lab = [], []
    for k in range(45):
        t = k % 3
        sents = [" ".join(rng.choice(topics[t]) for _ in range(8)) + "." for _ in range(4)]
        docs.append(" ".join(sents))
        lab.append(t)
    ss = search_corpus(docs, dim=32, epochs=15, seed=1)
    for t in range(3):
        q = " ".join(topics[t][:3])
        for algo in ("tokenAvMax", "docAv", "sentAv"):
            top = ss.search(q, algo, top=5)
            prec = sum(lab[i] == t for i, _ in top) / 5
            assert prec >= 0.8, (t, algo, prec)
