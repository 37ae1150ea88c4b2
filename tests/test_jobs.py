"""Every registered CLI job on small seeded data (CPU), each checked against a plain
Python / torch oracle of the reference behaviour it re-implements."""
import json
import math
import random
from collections import Counter, defaultdict
from pathlib import Path

import numpy as np
import pytest
import torch

from avenir_amd.cli import JOBS, main

FIX = Path(__file__).parent / "fixtures"


def run(*args):
    assert main([str(a) for a in args] + ["--device", "cpu"]) == 0


def lines(p):
    p = Path(p)
    if p.is_dir():
        return [l for f in sorted(p.iterdir()) if f.is_file() for l in f.read_text().splitlines() if l.strip()]
    return [l for l in p.read_text().splitlines() if l.strip()]


def props(tmp, name, text):
    p = tmp / name
    p.write_text(text)
    return p


def test_job_count():
    # every reference MR (42) / Spark (27) job plus the external pipeline stages and drivers
    assert len(JOBS) >= 75


# ---------------------------------------------------------------------------------------------
# explore
# ---------------------------------------------------------------------------------------------
@pytest.fixture
def cat_data(tmp_path):
    rng = np.random.default_rng(3)
    rows = []
    for i in range(600):
        a = rng.choice(["x", "y", "z"])
        b = a if rng.random() < 0.7 else rng.choice(["x", "y", "z"])
        c = rng.choice(["p", "q"])
        cls = "T" if (a == "x" and rng.random() < 0.8) or rng.random() < 0.2 else "F"
        rows.append(f"r{i},{a},{b},{c},{cls}")
    data = tmp_path / "cat.csv"
    data.write_text("\n".join(rows) + "\n")
    schema = tmp_path / "cat.json"
    schema.write_text(json.dumps({"fields": [
        {"name": "id", "ordinal": 0, "id": True, "dataType": "string"},
        {"name": "a", "ordinal": 1, "dataType": "categorical", "feature": True, "cardinality": ["x", "y", "z"]},
        {"name": "b", "ordinal": 2, "dataType": "categorical", "feature": True, "cardinality": ["x", "y", "z"]},
        {"name": "c", "ordinal": 3, "dataType": "categorical", "feature": True, "cardinality": ["p", "q"]},
        {"name": "cls", "ordinal": 4, "dataType": "categorical", "cardinality": ["F", "T"]}]}))
    return data, schema, [r.split(",") for r in rows]


def _cramer(rows, i, j):
    t = Counter((r[i], r[j]) for r in rows)
    ri, cj = sorted({r[i] for r in rows}), sorted({r[j] for r in rows})
    M = np.array([[t[(a, b)] for b in cj] for a in ri], dtype=float)
    rs, cs = M.sum(1), M.sum(0)
    return ((M * M / np.outer(rs, cs)).sum() - 1.0) / (min(M.shape) - 1)


def test_cramer_and_heterogeneity(tmp_path, cat_data):
    data, schema, rows = cat_data
    cfg = props(tmp_path, "crc.properties", f"crc.feature.schema.file.path={schema}\ncrc.source.attributes=1\n"
                f"crc.dest.attributes=2,3\ncac.feature.schema.file.path={schema}\ncac.first.set.attributes=1\n"
                "cac.second.set..attributes=2\nhrc.heterogeneity.algorithm=gini\n")
    out = tmp_path / "crc.txt"
    run("cramerCorrelation", "-i", data, "-o", out, "-c", cfg)
    got = {tuple(l.split(",")[:2]): float(l.split(",")[2]) for l in lines(out)}
    assert got[("a", "b")] == pytest.approx(_cramer(rows, 1, 2), rel=1e-9)
    assert got[("a", "c")] == pytest.approx(_cramer(rows, 1, 3), rel=1e-9)
    out2 = tmp_path / "hrc.txt"
    run("heterogeneityReductionCorrelation", "-i", data, "-o", out2, "-c", cfg)
    (l,) = lines(out2)
    assert l.startswith("a,b,") and 0 < float(l.split(",")[2]) < 1


def test_numerical_correlation(tmp_path):
    rng = np.random.default_rng(0)
    X = rng.normal(size=(500, 3))
    X[:, 1] = X[:, 0] * 2 + rng.normal(scale=0.3, size=500)
    data = tmp_path / "num.csv"
    data.write_text("\n".join(",".join(f"{v:.6f}" for v in r) for r in X))
    cfg = props(tmp_path, "nuc.properties", "nuc.attr.pairs=0:1,0:2\n")
    out = tmp_path / "nuc.txt"
    run("numericalCorrelation", "-i", data, "-o", out, "-c", cfg)
    got = [float(l.split(",")[2]) for l in lines(out)]
    Xr = np.round(X, 6)
    assert got[0] == pytest.approx(np.corrcoef(Xr[:, 0], Xr[:, 1])[0, 1], rel=1e-6)
    assert got[1] == pytest.approx(np.corrcoef(Xr[:, 0], Xr[:, 2])[0, 1], rel=1e-6)


def test_rule_evaluator(tmp_path, cat_data):
    data, schema, rows = cat_data
    cfg = props(tmp_path, "rue.properties", "rue.rule.names=r1,r2\nrue.rule.r1=1 eq x > T\n"
                "rue.rule.r2=1 in y:z and 3 eq p > F\nrue.class.attr.ord=4\nrue.class.values=F,T\n"
                "rue.conf.strategy=confAccuracy\n")
    out = tmp_path / "rue.txt"
    run("ruleEvaluator", "-i", data, "-o", out, "-c", cfg)
    got = {l.split(",")[0]: (float(l.split(",")[1]), float(l.split(",")[2])) for l in lines(out)}
    cov1 = [r for r in rows if r[1] == "x"]
    cov2 = [r for r in rows if r[1] in ("y", "z") and r[3] == "p"]
    assert got["r1"][0] == pytest.approx(round(sum(r[4] == "T" for r in cov1) / len(cov1), 3), abs=1e-3)
    assert got["r1"][1] == pytest.approx(round(len(cov1) / len(rows), 3), abs=1e-3)
    assert got["r2"][0] == pytest.approx(round(sum(r[4] == "F" for r in cov2) / len(cov2), 3), abs=1e-3)


def test_rule_expression_parser():
    from avenir_amd.utils.rules import RuleExpression
    r = RuleExpression.create_rule("1 gt int:10 and 2 notIn a:b > yes")
    rows = [["0", "11", "c"], ["0", "11", "a"], ["0", "5", "c"], ["0", "12.5", "d"]]
    assert r.consequent == "yes"
    assert r.evaluate_rows(rows).tolist() == [True, False, False, True]


def test_samplers_and_adaboost(tmp_path, cat_data):
    data, schema, rows = cat_data
    cfg = props(tmp_path, "s.properties", "usb.class.attr.ord=4\nbas.batch.size=100\nabe.pred.class.attr.ord=1\n"
                "abe.actual.class.attr.ord=2\nabe.boost.attr.ord=5\nabu.pred.class.attr.ord=1\n"
                "abu.actual.class.attr.ord=2\nabu.boost.attr.ord=5\nabu.intial.weight=1.0\n")
    out = tmp_path / "usb"
    run("underSamplingBalancer", "-i", data, "-o", out, "-c", cfg)
    cnt = Counter(l.split(",")[4] for l in lines(out))
    assert abs(cnt["T"] - cnt["F"]) < 0.3 * max(cnt.values())
    out = tmp_path / "bag"
    run("baggingSampler", "-i", data, "-o", out, "-c", cfg)
    assert len(lines(out)) == len(rows) and set(lines(out)) <= set(l for l in data.read_text().splitlines())
    wdata = tmp_path / "w.csv"
    wdata.write_text("\n".join(",".join(r[:5]) + ",0.5" for r in rows))
    out = tmp_path / "err.txt"
    run("adaBoostError", "-i", wdata, "-o", out, "-c", cfg)
    err = float(lines(out)[0].split("=")[1])
    exp = sum(0.5 * (r[1] != r[2]) for r in rows) / len(rows)
    assert err == pytest.approx(exp, abs=1e-6)
    cfg2 = props(tmp_path, "u.properties", cfg.read_text() + f"abu.error.file.path={out}\n")
    out2 = tmp_path / "upd"
    run("adaBoostUpdate", "-i", wdata, "-o", out2, "-c", cfg2)
    alpha = 0.5 * math.log((1 - err) / err)
    got = [float(l.split(",")[5]) for l in lines(out2)]
    expw = [0.5 * math.exp(alpha if r[1] != r[2] else -alpha) for r in rows]
    assert np.allclose(got, expw, atol=1e-6)


def test_top_matches_and_smote_pipeline_pieces(tmp_path):
    # pair file: srcId,trgId,srcRec(3),trgRec(3),rank with class at record ordinal 2
    recs = {f"e{i}": [f"e{i}", str(i), "A" if i < 6 else "B"] for i in range(10)}
    pairs = []
    for i in range(10):
        for j in range(i + 1, 10):
            pairs.append(",".join([f"e{i}", f"e{j}"] + recs[f"e{i}"] + recs[f"e{j}"] + [str(abs(i - j) * 10)]))
    inp = tmp_path / "pairs.txt"
    inp.write_text("\n".join(pairs))
    cfg = props(tmp_path, "tmc.properties", "tmc.class.attr.ord=2\ntmc.top.match.count=2\ntmc.compact.output=true\n"
                "tmc.include.class.in.output=false\n")
    out = tmp_path / "tmc.txt"
    run("topMatchesByClass", "-i", inp, "-o", out, "-c", cfg)
    got = {l.split(",")[0]: l.split(",") for l in lines(out)}
    # e0's two nearest same-class records are e1 and e2
    assert got["e0"][3::3][:2] == ["e1", "e2"]
    assert "e6" not in got["e5"]


def test_class_partition_and_data_partitioner(tmp_path):
    from avenir_amd.data import synth
    data, schema = tmp_path / "h.csv", tmp_path / "h.json"
    data.write_text("\n".join(synth.call_hangup_lines(800, seed=2)) + "\n")
    schema.write_text(json.dumps(synth.CALL_HANGUP_SCHEMA))
    cfg = props(tmp_path, "cpg.properties", "cpg.split.algorithm=giniIndex\n")
    out = tmp_path / "splits.txt"
    run("classPartitionGenerator", "-i", data, "-o", out, "-c", cfg, "--schema", schema)
    ls = lines(out)
    assert len(ls) > 3
    cfg2 = props(tmp_path, "dap.properties", f"dap.split.path={out}\n")
    pout = tmp_path / "parts"
    run("dataPartitioner", "-i", data, "-o", pout, "-c", cfg2, "--schema", schema)
    segs = list(pout.glob("split=*/segment=*/part-*"))
    assert len(segs) >= 2
    assert sum(len(lines(s)) for s in segs) == 800


def test_encodings_and_mappers(tmp_path, cat_data):
    data, schema, rows = cat_data
    conf = tmp_path / "enc.conf"
    stat = tmp_path / "stat.txt"
    conf.write_text(f"""
categoricalFeatureHashingEncoding {{
  cat.fieldOrdinals = [1,2]
  encoding.size = 8
  row.size = 5
}}
categoricalLeaveOneOutEncoding {{
  cat.field.ordinals = [1,2]
  class.field.ordinal = 4
  class.pos.val = "T"
  regularization.factor = 10
  rand.std.dev = 0.0
  train.data.set = true
  target.stat.file.path = "{stat}"
}}
binaryDummyVariableGenerator {{
  cat.field.ordinals = [1,3]
  true.value = "1"
  false.value = "0"
}}
linearMapper {{
  id.field.ordinals = [0]
  quant.field.ordinals = [0,1]
  retained.field.ordinals = [2]
  trans.matrix.path = "{tmp_path / 'M.txt'}"
}}
""")
    out = tmp_path / "fh"
    run("categoricalFeatureHashingEncoding", "-i", data, "-o", out, "-c", conf)
    ls = lines(out)
    assert len(ls[0].split(",")) == 3 + 8
    assert all(sum(abs(int(v)) for v in l.split(",")[3:11]) in (0, 2) for l in ls)
    out = tmp_path / "loo"
    run("categoricalLeaveOneOutEncoding", "-i", data, "-o", out, "-c", conf)
    st = {tuple(l.split(",")[:2]): (int(l.split(",")[2]), int(l.split(",")[3])) for l in lines(stat)}
    r0 = lines(out)[0].split(",")
    y0 = 1 if rows[0][4] == "T" else -1
    c, s = st[("1", rows[0][1])]
    assert float(r0[1]) == pytest.approx((s - y0) / (c - 1 + 10), abs=1e-3)
    out = tmp_path / "dv"
    run("binaryDummyVariableGenerator", "-i", data, "-o", out, "-c", conf)
    r = lines(out)[0].split(",")
    assert len(r) == 5 - 2 + 3 + 2 and r[1:4].count("1") == 1
    num = tmp_path / "num.csv"
    num.write_text("1,2,a\n3,4,b\n")
    (tmp_path / "M.txt").write_text("1,1\n1,-1\n")
    out = tmp_path / "lm"
    run("linearMapper", "-i", num, "-o", out, "-c", conf)
    assert lines(out) == ["1,3.000,-1.000,a", "3,7.000,-1.000,b"]


def test_relief_and_fisher_svm(tmp_path):
    from avenir_amd.data import synth
    data, schema = tmp_path / "h.csv", tmp_path / "h.json"
    data.write_text("\n".join(synth.call_hangup_lines(500, seed=5)) + "\n")
    schema.write_text(json.dumps(synth.CALL_HANGUP_SCHEMA))
    out = tmp_path / "relief.txt"
    run("reliefFeatureRelevance", "-i", data, "-o", out, "--schema", schema)
    assert len(lines(out)) >= 3
    out = tmp_path / "fisher.txt"
    run("fisherDiscriminant", "-i", data, "-o", out, "--schema", schema)
    assert len(lines(out)) >= 3 and all(len(l.split(",")) == 4 for l in lines(out))
    cfg = props(tmp_path, "svm.properties", "svm.kernel.type=rbf\nsvm.kernel.param=0.5\n")
    out = tmp_path / "svm.txt"
    run("supportVectorMachine", "-i", data, "-o", out, "-c", cfg, "--schema", schema)
    ls = lines(out)
    assert ls[-1].startswith("bias,") and len(ls) > 2


def test_incremental_pca(tmp_path):
    rng = np.random.default_rng(1)
    rows = []
    for k in ("a", "b"):
        for t in range(200):
            z = rng.normal()
            rows.append(f"{k},{z:.5f},{2 * z + 0.01 * rng.normal():.5f}")
    data = tmp_path / "p.csv"
    data.write_text("\n".join(rows))
    st = tmp_path / "state.txt"
    conf = tmp_path / "p.conf"
    conf.write_text(f'incrementalPrincipalComponent {{\n id.field.ordinals = [0]\n quant.field.ordinals = [1,2]\n'
                    f' state.filePath = "{st}"\n}}\n')
    out = tmp_path / "pca"
    run("incrementalPrincipalComponent", "-i", data, "-o", out, "-c", conf)
    ls = lines(st)
    assert ls[0].startswith("a,2,")
    w = [float(v) for v in ls[3].split(",")]
    assert abs(abs(w[1] / w[0]) - 2.0) < 0.3          # first component ~ (1, 2) / sqrt(5)
    run("incrementalPrincipalComponent", "-i", data, "-o", tmp_path / "pca2", "-c", conf)
    assert int(lines(st)[0].split(",")[3]) == 400       # state resumed and extended


# ---------------------------------------------------------------------------------------------
# markov / sequence
# ---------------------------------------------------------------------------------------------
def test_hmm_builder_fully_tagged_and_viterbi(tmp_path):
    rng = random.Random(0)
    rows = []
    for i in range(200):
        st = "H"
        toks = []
        for _ in range(10):
            st = st if rng.random() < 0.8 else ("L" if st == "H" else "H")
            ob = ("a" if rng.random() < 0.8 else "b") if st == "H" else ("b" if rng.random() < 0.8 else "a")
            toks.append(f"{ob}:{st}")
        rows.append(f"s{i}," + ",".join(toks))
    data = tmp_path / "tagged.txt"
    data.write_text("\n".join(rows))
    cfg = props(tmp_path, "hmm.properties", "hmmb.skip.field.count=1\nhmmb.model.states=H,L\n"
                "hmmb.model.observations=a,b\nhmmb.trans.prob.scale=1000\n")
    model = tmp_path / "hmm.txt"
    run("hiddenMarkovModelBuilder", "-i", data, "-o", model, "-c", cfg)
    ml = lines(model)
    assert ml[:2] == ["H,L", "a,b"] and len(ml) == 7
    # transition counts oracle (StateTransitionProbability integer rows)
    tr = Counter()
    for r in rows:
        s = [t.split(":")[1] for t in r.split(",")[1:]]
        tr.update(zip(s[:-1], s[1:]))
    hh = tr[("H", "H")] * 1000 // (tr[("H", "H")] + tr[("H", "L")])
    assert int(ml[2].split(",")[0]) == hh
    obs = tmp_path / "obs.txt"
    obs.write_text("u1,a,a,a,b,b,b,b\n")
    out = tmp_path / "vit.txt"
    cfg2 = props(tmp_path, "vsp.properties", "vsp.output.state.only=false\nvsp.sub.field.delim=:\n")
    run("viterbiStatePredictor", "-i", obs, "-o", out, "--model", model, "-c", cfg2)
    assert lines(out)[0].startswith("u1,a:H,a:H,a:H,")


def test_hmm_partially_tagged_reference_windows(tmp_path):
    from avenir_amd.models.markov import HiddenMarkovModelBuilder
    b = HiddenMarkovModelBuilder(["S1", "S2"], ["o1", "o2", "o3"])
    row = ["o1", "S1", "o2", "o3", "o1", "S2", "o2"]
    tr, em, ini = b.partially_tagged_counts([row], [3, 2, 1])
    # reference arithmetic: state S1 at 1: right window = 5 - 1/2 = 5 -> right bound 6; left bound = 1-5 -> 0
    # S1 left: j=0 (o1, w=3); right: j=2..6 (o2 w3, o3 w2, o1 w1, S2 skipped, o2 w1)
    assert em[0].tolist() == [3 + 1, 3 + 1, 2]
    assert tr.tolist() == [[0, 1], [0, 0]] and ini.tolist() == [1, 0]


def test_markov_classifier_and_pst(tmp_path):
    rng = np.random.default_rng(2)
    rows = []
    for i in range(300):
        cls = "T" if i % 2 else "F"
        p = 0.8 if cls == "T" else 0.3
        s, seq = "A", []
        for _ in range(12):
            s = s if rng.random() < p else ("B" if s == "A" else "A")
            seq.append(s)
        rows.append(f"u{i},{cls}," + ",".join(seq))
    data = tmp_path / "seq.txt"
    data.write_text("\n".join(rows))
    cfg = props(tmp_path, "conv.properties", "mst.skip.field.count=1\nmst.model.states=A,B\n"
                "mst.class.label.field.ord=1\nmst.class.labels=T,F\nmmc.id.field.ord=0\nmmc.class.labels=T,F\n"
                "mmc.log.odds.threshold=0\nmmc.skip.field.count=2\nmmc.validation.mode=true\n"
                "mmc.class.label.field.ord=1\n")
    model = tmp_path / "mm.txt"
    run("markovStateTransitionModel", "-i", data, "-o", model, "-c", cfg)
    out = tmp_path / "pred"
    run("markovModelClassifier", "-i", data, "-o", out, "--model", model, "-c", cfg)
    res = [l.split(",") for l in lines(out)]
    acc = sum(r[1] == r[2] for r in res) / len(res)
    assert acc > 0.8
    cfg2 = props(tmp_path, "pst.properties", "pstg.skip.field.count=1\npstg.max.seq.length=3\n"
                 "pstg.class.label.field.ord=1\n")
    out2 = tmp_path / "pst.txt"
    run("probabilisticSuffixTreeGenerator", "-i", data, "-o", out2, "-c", cfg2)
    got = {tuple(l.split(",")[:-1]): int(l.split(",")[-1]) for l in lines(out2)}
    exp = Counter()
    for r in rows:
        p = r.split(",")
        s = p[2:]
        for w in (2, 3):
            for a in range(len(s) - w + 1):
                exp[(p[1],) + tuple(s[a:a + w])] += 1
                exp[(p[1], "$")] += 1
    assert got == dict(exp)


def test_gsp_candidates(tmp_path):
    from avenir_amd.ops import sequence_ops as SO
    seqs = ["a,b", "b,c", "c,d", "b,b", "c,a"]
    data = tmp_path / "k2.txt"
    data.write_text("\n".join(seqs))
    cfg = props(tmp_path, "cgs.properties", "cgs.item.set.length=2\n")
    out = tmp_path / "cand.txt"
    run("candidateGenerationWithSelfJoin", "-i", data, "-o", out, "-c", cfg)
    S = [tuple(s.split(",")) for s in seqs]
    exp = sorted({a + (b[-1],) for a in S for b in S if a[1:] == b[:-1]})
    assert lines(out) == [",".join(c) for c in exp]
    X = torch.randint(0, 4, (200, 3))
    C = SO.gsp_join(X)
    U = torch.unique(X, dim=0).tolist()
    ref = [a + [b[-1]] for a in U for b in U if a[1:] == b[:-1]]
    assert C.tolist() == ref


def test_ctmc_jobs(tmp_path):
    rng = np.random.default_rng(4)
    rows = []
    for k in ("k1", "k2"):
        t = 0
        s = "F"
        for _ in range(300):
            rows.append(f"{k},{t},{s}")
            t += int(rng.exponential(3600_000 * (2 if s == "F" else 1)))
            s = rng.choice([x for x in ("F", "P", "L") if x != s])
    data = tmp_path / "st.txt"
    data.write_text("\n".join(rows))
    conf = tmp_path / "sup.conf"
    tra = tmp_path / "tra"
    conf.write_text(f"""stateTransitionRate {{
  key.field.ordinals = [0]
  time.field.ordinal = 1
  state.field.ordinal = 2
  state.values = ["F", "P", "L"]
  rate.time.unit = "hour"
  input.time.unit = "ms"
  trans.rate.output.precision = 9
}}
contTimeStateTransitionStats {{
  key.field.len = 1
  state.values = ["F", "P", "L"]
  time.horizon = 4
  state.trans.file.path = "{tra}"
  state.trans.stat = "futureStateProb"
}}
""")
    run("stateTransitionRate", "-i", data, "-o", tra, "-c", conf)
    ls = lines(tra)
    assert len(ls) == 2 and ls[0].startswith("(k1,")
    q = [float(v) for v in ls[0][1:-1].split(",")[1:]]
    assert abs(sum(q[0:3])) < 1e-6 and q[0] < 0
    inp = tmp_path / "init.txt"
    inp.write_text("k1,F,F\nk1,F,L\nk2,P,P\n")
    out = tmp_path / "ras"
    run("contTimeStateTransitionStats", "-i", inp, "-o", out, "-c", conf)
    v = [float(l[1:-1].split(",")[1]) for l in lines(out)]
    assert 0 < v[0] < 1 and 0 < v[1] < 1
    Q = torch.tensor(q, dtype=torch.float64).view(3, 3)
    P = torch.matrix_exp(Q * 4)
    assert v[0] == pytest.approx(float(P[0, 0]), abs=1e-6)
    assert v[1] == pytest.approx(float(P[0, 2]), abs=1e-6)


def test_sequence_analytics_jobs(tmp_path):
    data = tmp_path / "ev.txt"
    day = 86400_000
    data.write_text("\n".join(f"u{i % 3},{i * 3600_000 + 5 * day},{'abc'[i % 3]}" for i in range(48)))
    conf = tmp_path / "seq.conf"
    conf.write_text("""eventTimeDistribution {
  id.field.ordinals = [0]
  time.field.ordinal = 1
}
sequenceGenerator {
  id.field.ordinals = [0]
  val.field.ordinals = [2]
  seq.field = 1
}
markovChainPredictor {
  id.fieldOrdinals = [0]
  attr.ordinal = 2
  seq.fieldOrd = 1
  window.size = 2
}
dotMatrixMatching {
  window.size = 2
}
""")
    out = tmp_path / "etd"
    run("eventTimeDistribution", "-i", data, "-o", out, "-c", conf)
    ls = lines(out)
    assert len(ls) == 3 and sum(int(x.split(":")[1]) for x in ls[0].split(",")[1:]) == 16
    out = tmp_path / "sg"
    run("sequenceGenerator", "-i", data, "-o", out, "-c", conf)
    assert lines(out)[0] == "u0," + ",".join(["a"] * 16)
    out = tmp_path / "tde"
    run("timeDelayEmbeddingModel", "-i", data, "-o", out, "-c", conf)
    assert lines(out)[0] == "u0,a:a,15"
    seqs = tmp_path / "s.txt"
    seqs.write_text("x,a,b,c,d\ny,a,b,c,e\nz,q,r,s,t\n")
    out = tmp_path / "dm"
    run("dotMatrixMatching", "-i", seqs, "-o", out, "-c", conf)
    got = {tuple(l.split(",")[:2]): float(l.split(",")[2]) for l in lines(out)}
    assert got[("x", "y")] > 0 and got[("x", "z")] == 0


# ---------------------------------------------------------------------------------------------
# association / clustering / bandits / similarity / optimisers
# ---------------------------------------------------------------------------------------------
def test_rule_miner_and_marker(tmp_path):
    fi = tmp_path / "fi.txt"
    fi.write_text("a,0.6\nb,0.5\nc,0.2\na,b,0.4\n")
    cfg = props(tmp_path, "arm.properties", "arm.conf.threshold=0.7\narm.max.ante.size=1\n"
                f"iim.item.set.file.path={fi}\niim.skip.field.count=1\n")
    out = tmp_path / "rules.txt"
    run("associationRuleMiner", "-i", fi, "-o", out, "-c", cfg)
    assert lines(out) == ["b -> a"]      # 0.4 / 0.5 = 0.8 > 0.7; a -> b is 0.67
    tx = tmp_path / "tx.txt"
    tx.write_text("t1,a,z,b\n")
    fi1 = tmp_path / "fi1.txt"
    fi1.write_text("a,0.6\nb,0.5\n")
    cfg2 = props(tmp_path, "iim.properties", f"iim.item.set.file.path={fi1}\n")
    out2 = tmp_path / "marked.txt"
    run("infrequentItemMarker", "-i", tx, "-o", out2, "-c", cfg2)
    assert lines(out2) == ["t1,a,*,b"]


def test_distance_store_and_agglomerative(tmp_path):
    pairs = tmp_path / "pairs.txt"
    pairs.write_text("a,b,0.9\na,c,0.85\nb,c,0.9\nd,e,0.95\na,d,0.1\nc,e,0.05\n")
    cfg = props(tmp_path, "agg.properties", "eds.pair.input=true\nagg.min.av.edge.weight.threshold=0.5\n")
    store = tmp_path / "store"
    run("entityDistanceStore", "-i", pairs, "-o", store, "-c", cfg)
    from avenir_amd.utils.distance_store import EntityDistanceStore
    s = EntityDistanceStore(store)
    assert s.read("a") == {"b": 0.9, "c": 0.85, "d": 0.1}
    ents = tmp_path / "ents.txt"
    ents.write_text("a\nb\nc\nd\ne\n")
    out = tmp_path / "cl.txt"
    run("agglomerativeGraphical", "-i", ents, "-o", out, "-c", cfg, "--model", store)
    cl = [l.split(",")[1:-1] for l in lines(out)]
    assert cl == [["a", "b", "c"], ["d", "e"]]


def test_kmeanspp_and_similarity(tmp_path):
    rng = np.random.default_rng(0)
    rows = []
    for g in ("g1", "g2"):
        for c in ((0, 0), (4, 4), (0, 4)):
            for _ in range(40):
                rows.append(f"{g},{c[0] + rng.normal(0, .2):.4f},{c[1] + rng.normal(0, .2):.4f}")
    data = tmp_path / "pts.csv"
    data.write_text("\n".join(rows))
    conf = tmp_path / "km.conf"
    conf.write_text(f"""kMeansPlusPlusCluster {{
  id.fieldOrdinals = [0]
  num.clusters = [2,3,4,5]
  num.iter = 20
  cluster.outputPath = "{tmp_path / 'cent'}"
}}
recordSimilarity {{
  attr.ordinals = [1,2]
  id.ordinal = 0
  distance.scale = 1000
}}
nearestRecords {{
  neighbor.count = 2
}}
groupedRecordSimilarity {{
  group.field.ordinals = [0]
  attr.ordinals = [1,2]
  id.ordinal = 0
}}
""")
    out = tmp_path / "km"
    run("kMeansPlusPlusCluster", "-i", data, "-o", out, "-c", conf)
    kn = [l for l in lines(out) if "knuckle" in l]
    assert kn == ["g1,knuckle,3", "g2,knuckle,3"]
    small = tmp_path / "small.csv"
    small.write_text("p,0,0\nq,1,0\nr,10,10\n")
    out = tmp_path / "rs"
    run("recordSimilarity", "-i", small, "-o", out, "-c", conf)
    got = {tuple(l.split(",")[:2]): int(l.split(",")[-1]) for l in lines(out)}
    assert got[("p", "q")] < got[("p", "r")] and len(got) == 3
    out2 = tmp_path / "nr"
    run("nearestRecords", "-i", out, "-o", out2, "-c", conf)
    assert lines(out2)[0] == "p,q,r"


def test_batch_bandits(tmp_path):
    rows = []
    for g in ("g1", "g2"):
        for j, m in enumerate([1.0, 5.0, 2.0, 0.5]):
            rows.append(f"{g},item{j},10,{m}")
    data = tmp_path / "state.txt"
    data.write_text("\n".join(rows))
    cfg = props(tmp_path, "b.properties", "global.batch.size=1\ncurrent.round.num=50\ncount.ordinal=2\n"
                "reward.ordinal=3\nexploration.count.factor=1\nrandom.selection.prob=0.0\n")
    for j in ("greedyRandomBandit", "auerDeterministic", "softMaxBandit", "randomFirstGreedyBandit"):
        out = tmp_path / j
        run(j, "-i", data, "-o", out, "-c", cfg)
        ls = lines(out)
        assert len(ls) == 2 and all(l.split(",")[0] in ("g1", "g2") for l in ls)
        if j in ("auerDeterministic", "randomFirstGreedyBandit", "greedyRandomBandit"):
            assert all(l.endswith("item1") for l in ls), (j, ls)


def test_population_optimisers(tmp_path):
    conf = tmp_path / "opt.conf"
    conf.write_text(f"""geneticAlgorithm {{
  num.generations = 20
  population.size = 8
  num.optimizers = 2
  domain.callback.config.file = "{FIX / 'taskSched.json'}"
}}
randomSearch {{
  max.num.iterations = 20
  num.optimizers = 2
  locally.optimize = true
  domain.callback.config.file = "{FIX / 'taskSched.json'}"
}}
""")
    for j in ("geneticAlgorithm", "randomSearch"):
        out = tmp_path / j
        run(j, "-o", out, "-c", conf)
        ls = lines(out)
        assert ls and ":" in ls[0]


def test_nb_text_mode(tmp_path):
    docs = ["the cheap pills offer now,spam", "meeting agenda for monday,ham", "cheap offer click now,spam",
            "project meeting notes,ham", "win cheap prize now,spam", "monday project review,ham"]
    data = tmp_path / "docs.txt"
    data.write_text("\n".join(docs))
    cfg = props(tmp_path, "t.properties", "bad.tabular.input=false\nbap.tabular.input=false\n")
    model = tmp_path / "nbt.txt"
    run("bayesianDistribution", "-i", data, "-o", model, "-c", cfg)
    ml = lines(model)
    assert "spam,1,cheap,3" in ml and "ham,,,3" in ml and ",1,meeting,2" in ml
    test = tmp_path / "q.txt"
    test.write_text("cheap prize offer,?\nmonday meeting,?\n")
    out = tmp_path / "p.txt"
    run("bayesianPredictor", "-i", test, "-o", out, "-c", cfg, "--model", model)
    assert [l.split(",")[2] for l in lines(out)] == ["spam", "ham"]
