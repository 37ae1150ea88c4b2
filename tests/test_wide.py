"""High-cardinality categoricals (> 255 values: uint16 codes + the K2w kernel) and the reference's
``field.delim.regex`` delimiters (multi-character literals, regexes).

Reference: J/explore/CategoricalContinuousEncoding.java:116-137 keys (attribute, raw value) with no
limit on the number of values; S/explore/CategoricalLeaveOneOutEncoding.scala:80 likewise."""
import collections
import json
import math

import numpy as np
import pytest
import torch

from avenir_amd.data.table import load_csv
from avenir_amd.models.explore import (apply_encoding, class_affinity, leave_one_out_encoding,
                                       supervised_encoding)
from avenir_amd.ops import histogram as H
from avenir_amd.utils.schema import FeatureSchema

NV = 10_000


def _write(tmp_path, n=40_000, nv=NV, seed=0, delim=","):
    rng = np.random.default_rng(seed)
    sup = rng.integers(0, nv, n)
    reg = rng.integers(0, 4, n)
    # the class depends on the supplier id so the encodings carry signal
    p = 0.2 + 0.6 * (sup % 7 == 0)
    y = (rng.random(n) < p).astype(int)
    lines = [delim.join([f"r{i}", f"S{sup[i]:05d}", f"R{reg[i]}", "T" if y[i] else "F"]) for i in range(n)]
    data = tmp_path / "hica.csv"
    data.write_text("\n".join(lines) + "\n")
    schema = {"fields": [
        {"name": "id", "ordinal": 0, "id": True, "dataType": "string"},
        {"name": "supplier", "ordinal": 1, "feature": True, "dataType": "categorical"},      # no cardinality
        {"name": "region", "ordinal": 2, "feature": True, "dataType": "categorical",
         "cardinality": ["R0", "R1", "R2", "R3"]},
        {"name": "late", "ordinal": 3, "classAttribute": True, "dataType": "categorical", "cardinality": ["F", "T"]}]}
    sp = tmp_path / "hica.json"
    sp.write_text(json.dumps(schema))
    return data, sp, lines


def _oracle_counts(lines, delim=","):
    cnt = collections.defaultdict(lambda: [0, 0])
    for ln in lines:
        r = ln.split(delim)
        cnt[r[1]][1 if r[3] == "T" else 0] += 1
    return cnt


def test_wide_table_and_supervised_encoding(tmp_path):
    data, sp, lines = _write(tmp_path)
    t = load_csv(data, FeatureSchema.from_json(sp), ",")
    assert t.codes.dtype == torch.uint16 and t.wide and t.missing == 65535
    sup_f = t.binned_fields[0]
    assert sup_f.num_bins > 255
    enc = supervised_encoding(t, "supervisedRatio", 1000, pos_class=1)
    cnt = _oracle_counts(lines)
    for v, (neg, pos) in cnt.items():
        assert enc[1][v] == math.trunc(pos * 1000 / (pos + neg))
    woe = supervised_encoding(t, "weightOfEvidence", 100, pos_class=1, integer=False)
    all_pos = sum(c[1] for c in cnt.values())
    all_neg = sum(c[0] for c in cnt.values())
    v0 = sorted(cnt)[3]
    neg, pos = cnt[v0]
    assert abs(woe[1][v0] - math.log((pos / all_pos) / (max(neg, 1) / all_neg)) * 100) < 1e-6
    X = apply_encoding(t, enc)
    assert X.shape == (t.n, 2)
    r0 = lines[0].split(",")
    assert float(X[0, 0]) == enc[1][r0[1]]


def test_wide_leave_one_out_and_affinity(tmp_path):
    data, sp, lines = _write(tmp_path, n=20_000, seed=1)
    t = load_csv(data, FeatureSchema.from_json(sp), ",")
    y = (t.labels[: t.n] == 1).double()
    loo = leave_one_out_encoding(t, y)
    sums = collections.defaultdict(float)
    cnts = collections.defaultdict(int)
    for ln in lines:
        r = ln.split(",")
        sums[r[1]] += r[3] == "T"
        cnts[r[1]] += 1
    for i in (0, 17, 1234):
        r = lines[i].split(",")
        yi = float(r[3] == "T")
        exp = (sums[r[1]] - yi) / max(cnts[r[1]] - 1, 1e-12)
        assert abs(float(loo[i, 0]) - exp) < 1e-5
    aff = class_affinity(t, "distrDiff", pos_class=1)
    cnt = _oracle_counts(lines)
    tp = sum(c[1] for c in cnt.values())
    tn = sum(c[0] for c in cnt.values())
    d = dict(aff[1])
    for v in list(cnt)[:20]:
        neg, pos = cnt[v]
        assert abs(d[v] - (pos / tp - neg / tn)) < 1e-9


def test_multichar_and_regex_delimiters(tmp_path):
    data, sp, lines = _write(tmp_path, n=2000, nv=300, delim=",,")
    t = load_csv(data, FeatureSchema.from_json(sp), ",,")             # native multi-char literal
    t2 = load_csv(data, FeatureSchema.from_json(sp), ",+")            # a real regex: Python splitter
    assert t.n == t2.n == 2000
    assert torch.equal(t.codes[:, : t.n], t2.codes[:, : t2.n])
    assert torch.equal(t.labels[: t.n], t2.labels[: t2.n])
    assert t.ids[:3] == ["r0", "r1", "r2"]


@pytest.mark.gpu
@pytest.mark.parametrize("nv,mode", [(NV, 0), (NV, 2), (40_000, 0)])
def test_wide_histogram_kernel_matches_cpu(cuda, nv, mode):
    g = torch.Generator().manual_seed(nv)
    n = 300_000
    codes = torch.randint(0, nv, (2, n + 16), generator=g).to(torch.int32)
    codes[:, ::97] = 65535                                        # missing
    codes = codes.to(torch.uint16)
    labels = torch.randint(0, 3, (n + 16,), generator=g).to(torch.uint8)
    bins = [nv, 17]
    codes[1] = (codes[1].to(torch.int32) % 17).to(torch.uint16)
    ref = H.class_histogram(codes, n, bins, labels, 3, count_labels=True)
    got = H.class_histogram(codes.to(cuda), n, bins, labels.to(cuda), 3, count_labels=True, mode=mode)
    assert torch.equal(got.cpu(), ref)


@pytest.mark.gpu
def test_wide_encoding_gpu_matches_cpu(cuda, tmp_path):
    data, sp, _ = _write(tmp_path)
    t = load_csv(data, FeatureSchema.from_json(sp), ",")
    tg = load_csv(data, FeatureSchema.from_json(sp), ",", device=cuda)
    assert tg.codes.dtype == torch.uint16
    for strat in ("supervisedRatio", "weightOfEvidence"):
        assert supervised_encoding(tg, strat) == supervised_encoding(t, strat)
    y = (t.labels[: t.n] == 1).double()
    assert torch.allclose(leave_one_out_encoding(tg, y.to(cuda)).cpu(), leave_one_out_encoding(t, y))
    a, b = class_affinity(tg, "oddsRatio"), class_affinity(t, "oddsRatio")
    assert a.keys() == b.keys()
    for k in a:
        da, db = dict(a[k]), dict(b[k])
        # odds ratios are +inf where a value never occurs with the negative class: compare with
        # equality first (inf == inf), then relatively, then NaN-to-NaN
        assert all(da[v] == db[v] or math.isclose(da[v], db[v], rel_tol=1e-12)
                   or (math.isnan(da[v]) and math.isnan(db[v])) for v in db)
    cg = H.class_histogram(tg.codes, tg.n, tg.bins, tg.labels, tg.n_classes)
    assert torch.equal(cg.cpu(), H.class_histogram(t.codes, t.n, t.bins, t.labels, t.n_classes))


# ---------------------------------------------------------------------------------------------
# > 65,534 values: int32 codes (INT32_MAX = missing), same kernels (int32 instantiations)
# ---------------------------------------------------------------------------------------------
HUGE = 100_000


def test_huge_categorical_table_and_encodings(tmp_path):
    data, sp, lines = _write(tmp_path, n=150_000, nv=HUGE, seed=2)
    t = load_csv(data, FeatureSchema.from_json(sp), ",")
    assert t.codes.dtype == torch.int32 and t.wide and t.missing == 2**31 - 1
    sup_f = t.binned_fields[0]
    assert sup_f.num_bins > 65535
    # codes round-trip to the raw strings (first-seen dictionary order)
    for i in (0, 5, 149_999):
        assert sup_f.cardinality[int(t.codes[0, i])] == lines[i].split(",")[1]
    enc = supervised_encoding(t, "supervisedRatio", 1000, pos_class=1)
    cnt = _oracle_counts(lines)
    for v in list(cnt)[:200]:
        neg, pos = cnt[v]
        assert enc[1][v] == math.trunc(pos * 1000 / (pos + neg))
    X = apply_encoding(t, enc)
    assert float(X[7, 0]) == enc[1][lines[7].split(",")[1]]
    y = (t.labels[: t.n] == 1).double()
    loo = leave_one_out_encoding(t, y)
    sums = collections.defaultdict(float)
    cnts = collections.defaultdict(int)
    for ln in lines:
        r = ln.split(",")
        sums[r[1]] += r[3] == "T"
        cnts[r[1]] += 1
    for i in (0, 17, 123_456):
        r = lines[i].split(",")
        exp = (sums[r[1]] - float(r[3] == "T")) / max(cnts[r[1]] - 1, 1e-12)
        assert abs(float(loo[i, 0]) - exp) < 1e-5
    # the pure-Python parser (regex delimiter) gives the same int32 table
    t2 = load_csv(data, FeatureSchema.from_json(sp), ",+")
    assert t2.codes.dtype == torch.int32 and torch.equal(t2.codes[:, : t2.n], t.codes[:, : t.n])


def test_huge_categorical_naive_bayes_cpu(tmp_path):
    from avenir_amd.models.bayes import NaiveBayes
    data, sp, _ = _write(tmp_path, n=150_000, nv=HUGE, seed=3)
    t = load_csv(data, FeatureSchema.from_json(sp), ",")
    assert t.codes.dtype == torch.int32
    nb = NaiveBayes().fit(t)
    p = nb.predict(t)
    assert p.pred.shape[0] == t.n and float(p.prob.sum(1).mean()) == pytest.approx(1.0, rel=1e-4)


@pytest.mark.gpu
def test_huge_categorical_gpu_matches_cpu(cuda, tmp_path):
    from avenir_amd.models.bayes import NaiveBayes
    data, sp, _ = _write(tmp_path, n=400_000, nv=HUGE, seed=4)
    t = load_csv(data, FeatureSchema.from_json(sp), ",")
    tg = load_csv(data, FeatureSchema.from_json(sp), ",", device=cuda)
    assert tg.codes.dtype == torch.int32 and torch.equal(tg.codes.cpu(), t.codes)
    for mode in (0, 2):
        assert torch.equal(H.class_histogram(tg.codes, tg.n, tg.bins, tg.labels, 2, mode=mode).cpu(),
                           H.class_histogram(t.codes, t.n, t.bins, t.labels, 2))
    assert supervised_encoding(tg, "supervisedRatio") == supervised_encoding(t, "supervisedRatio")
    y = (t.labels[: t.n] == 1).double()
    assert torch.allclose(leave_one_out_encoding(tg, y.to(cuda)).cpu(), leave_one_out_encoding(t, y))
    pc = NaiveBayes().fit(t).predict(t)
    pg = NaiveBayes().fit(tg).predict(tg)                  # nb_predict_wide, int32 instantiation
    assert torch.equal(pg.pred.cpu(), pc.pred)
    assert torch.allclose(pg.prob.cpu(), pc.prob, atol=1e-5)
    assert torch.equal(pg.confusion.cpu(), pc.confusion)


@pytest.mark.gpu
def test_wide_naive_bayes_predict_kernel(cuda, tmp_path):
    """uint16-code tables take the wide NB kernel on the GPU (previously a torch fallback)."""
    from avenir_amd.models.bayes import NaiveBayes
    data, sp, _ = _write(tmp_path)
    t = load_csv(data, FeatureSchema.from_json(sp), ",")
    tg = t.to(cuda)
    pc = NaiveBayes().fit(t).predict(t)
    pg = NaiveBayes().fit(tg).predict(tg)
    assert torch.equal(pg.pred.cpu(), pc.pred)
    assert torch.allclose(pg.prob.cpu(), pc.prob, atol=1e-5)
