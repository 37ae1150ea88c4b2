"""Naive Bayes slice: counts vs an independent oracle, prediction, model I/O, world-size equivalence,
and HIP-kernel numerics (gpu)."""
import math

import pytest
import torch

from avenir_amd.data import synth
from avenir_amd.data.table import Table, load_csv, pad16
from avenir_amd.models.bayes import NaiveBayes
from avenir_amd.ops import histogram as H
from avenir_amd.utils.schema import FeatureSchema

from _dist import run_world


def _churn_table(tmp_path, n=2000, seed=0):
    p = tmp_path / "churn.csv"
    synth.write_churn(p, n, seed=seed)
    return p, load_csv(p, FeatureSchema.from_json(synth.CHURN_SCHEMA))


def test_histogram_oracle(tmp_path):
    p, t = _churn_table(tmp_path)
    counts = H.class_histogram(t.codes, t.n, t.bins, t.labels, 2)
    # oracle: python dict counting straight from the CSV text
    lines = p.read_text().splitlines()
    schema = FeatureSchema.from_json(synth.CHURN_SCHEMA)
    cls = schema.find_class_attr_field()
    o = 0
    for f in t.binned_fields:
        for c, cv in enumerate(cls.cardinality):
            for b, bv in enumerate(f.cardinality):
                exp = sum(1 for ln in lines if ln.split(",")[f.ordinal] == bv and ln.split(",")[6] == cv)
                assert int(counts[c, o + b]) == exp
        o += f.num_bins


def test_nb_fit_predict_cpu(tmp_path):
    _, t = _churn_table(tmp_path, 4000)
    nb = NaiveBayes(t.schema).fit(t)
    pr = nb.predict(t)
    acc = float((pr.pred.long() == t.labels[: t.n].long()).float().mean())
    assert acc > 0.55
    assert int(pr.confusion.sum()) == t.n
    assert torch.allclose(pr.prob.sum(1), torch.ones(t.n), atol=1e-5)
    # brute-force posterior for one record
    r = 11
    lp = nb.tables()["logp"].double()
    s = nb.tables()["logprior"].double().clone()
    o = 0
    for f, b in enumerate(nb.bins):
        s += lp[:, o + int(t.codes[f, r])]
        o += b
    ref = torch.softmax(s, 0)
    assert torch.allclose(pr.prob[r].double(), ref, atol=1e-5)


def test_nb_model_roundtrip(tmp_path):
    _, t = _churn_table(tmp_path, 1500)
    nb = NaiveBayes(t.schema).fit(t)
    mp = tmp_path / "model.txt"
    nb.save_model(mp)
    txt = mp.read_text().splitlines()
    assert any(line.startswith("closed,1,overage,") for line in txt)
    assert any(line.startswith(",5,") for line in txt)
    nb2 = NaiveBayes.load_model(mp, t.schema)
    assert torch.equal(nb2.counts, nb.counts)
    assert torch.equal(nb.predict(t).pred, nb2.predict(t).pred)


def test_nb_continuous_features():
    schema = FeatureSchema.from_json({"fields": [
        {"name": "x", "ordinal": 0, "dataType": "double", "feature": True},
        {"name": "k", "ordinal": 1, "dataType": "categorical", "cardinality": ["a", "b"], "feature": True},
        {"name": "y", "ordinal": 2, "dataType": "categorical", "cardinality": ["n", "p"]}]})
    g = torch.Generator().manual_seed(0)
    n = 3000
    y = torch.randint(0, 2, (n,), generator=g)
    x = torch.randn(n, generator=g) + 2.0 * y
    k = torch.where(torch.rand(n, generator=g) < 0.5 + 0.3 * (y * 2 - 1), 1, 0)
    from avenir_amd.data.table import from_arrays
    t = from_arrays(schema, {0: x.tolist(), 1: ["ab"[i] for i in k.tolist()], 2: ["np"[i] for i in y.tolist()]})
    nb = NaiveBayes(schema).fit(t)
    assert float(nb.moments[1, 0, 1] / nb.moments[1, 0, 0]) == pytest.approx(float(x[y == 1].mean()), rel=1e-6)
    pr = nb.predict(t)
    assert float((pr.pred.long() == y).float().mean()) > 0.8


def _rank_fit(rank, world, path):
    from avenir_amd.parallel.comm import get_comm
    t = load_csv(path, FeatureSchema.from_json(synth.CHURN_SCHEMA), rank=rank, world=world)
    nb = NaiveBayes(t.schema, comm=get_comm()).fit(t)
    pr = nb.predict(t)
    cnt = nb.validation_counters(pr.confusion)
    return nb.counts.tolist(), nb.class_n.tolist(), cnt.as_dict()


def test_nb_world_size_equivalence(tmp_path):
    p, t = _churn_table(tmp_path, 3001, seed=5)
    nb1 = NaiveBayes(t.schema).fit(t)
    res = run_world(_rank_fit, 2, str(p))
    for counts, cls_n, _ in res:
        assert counts == nb1.counts.tolist()
        assert cls_n == nb1.class_n.tolist()
    v = res[0][2]["Validation"]
    assert v["Correct"] + v["Incorrect"] == 3001


# ---------------------------------------------------------------------------------------------
# GPU numerics: HIP kernels vs the PyTorch CPU reference of the same op
# ---------------------------------------------------------------------------------------------
def _random_codes(n, bins, C, seed=0, missing_frac=0.01):
    g = torch.Generator().manual_seed(seed)
    ld = pad16(n)
    codes = torch.full((len(bins), ld), 255, dtype=torch.uint8)
    for f, b in enumerate(bins):
        v = torch.randint(0, b, (n,), generator=g)
        v[torch.rand(n, generator=g) < missing_frac] = 255
        codes[f, :n] = v.to(torch.uint8)
    lab = torch.full((ld,), 255, dtype=torch.uint8)
    lab[:n] = torch.randint(0, C, (n,), generator=g).to(torch.uint8)
    return codes, lab


@pytest.mark.gpu
@pytest.mark.parametrize("n,bins,C,mode", [
    (100_003, [4, 3, 3, 3, 5], 2, 0),          # class-split fast path, ragged tail
    (100_003, [4, 3, 3, 3, 5], 2, 3),          # packed-idx path
    (33_333, [7, 1, 2], 4, 0),                 # class-split C=4
    (33_335, [7, 6, 2, 5, 3, 3, 1, 2, 4, 7], 1, 0),  # class-split C=1, two groups
    (1 << 20, [2, 8, 4, 2, 3, 5, 7, 1, 2], 2, 0),  # > 8 features -> two feature groups
    (50_000, [17, 30, 9], 3, 0),               # LDS path (C*B > 16)
    (50_000, [4, 3], 2, 1),                    # forced LDS path
    (20_000, [200, 250], 5, 2),                # global atomics path
])
def test_class_histogram_gpu(cuda, n, bins, C, mode):
    codes, lab = _random_codes(n, bins, C, seed=n)
    ref = H.class_histogram(codes, n, bins, lab, C, count_labels=True)
    got = H.class_histogram(codes.to(cuda), n, bins, lab.to(cuda), C, mode=mode, count_labels=True)
    assert torch.equal(got.cpu(), ref)


@pytest.mark.gpu
def test_class_histogram_gpu_skewed_long_run(cuda):
    """Every row in ONE bin and class over 2^28 rows: each lane's 16-bit counters grow past what a
    64-lane sum of 16-bit fields can hold, so the kernel must widen before the cross-lane sum."""
    n = 1 << 28
    codes = torch.ones((2, n), dtype=torch.uint8, device=cuda)
    codes[1] = 2
    lab = torch.zeros(n, dtype=torch.uint8, device=cuda)
    got = H.class_histogram(codes, n, [4, 3], lab, 2, count_labels=True).cpu()
    assert int(got[0, 1]) == n and int(got[0, 4 + 2]) == n and int(got[0, -1]) == n
    assert int(got.sum()) == 3 * n


@pytest.mark.gpu
def test_pair_bigram_moments_gpu(cuda):
    n, bins, C = 70_001, [4, 6, 3], 3
    codes, lab = _random_codes(n, bins, C, seed=1)
    pairs = [(0, 1), (1, 2), (0, 2)]
    ref = H.pair_histogram(codes, n, bins, pairs, lab, C)
    got = H.pair_histogram(codes.to(cuda), n, bins, pairs, lab.to(cuda), C)
    for a, b in zip(ref, got):
        assert torch.equal(a, b.cpu())
    st, sl, _ = synth.markov_sequences(5000, 7, 12, 3, seed=2)
    st[::13, 9:] = -1
    r = H.bigram_histogram(st, 7, sl, 3)
    g = H.bigram_histogram(st.to(cuda), 7, sl.to(cuda), 3)
    assert torch.equal(r, g.cpu())
    x = torch.randn(4, pad16(n))
    rm = H.class_moments(x, n, lab, C)
    gm = H.class_moments(x.to(cuda), n, lab.to(cuda), C)
    assert torch.allclose(rm, gm.cpu(), rtol=1e-9, atol=1e-6)


@pytest.mark.gpu
def test_nb_predict_gpu_matches_cpu(cuda, tmp_path):
    _, t = _churn_table(tmp_path, 20_000, seed=9)
    nb = NaiveBayes(t.schema).fit(t)
    cpu = nb.predict(t)
    tg = t.to(cuda)
    nbg = NaiveBayes(t.schema).fit(tg)
    assert torch.equal(nbg.counts.cpu(), nb.counts)
    gpu = nbg.predict(tg)
    assert torch.equal(gpu.pred.cpu(), cpu.pred)
    assert torch.allclose(gpu.prob.cpu(), cpu.prob, atol=1e-5)
    assert torch.equal(gpu.confusion.cpu(), cpu.confusion)
    ref_c = nb.predict(t, ref_scale=True)
    ref_g = nbg.predict(tg, ref_scale=True)
    assert torch.allclose(ref_g.prob.cpu(), ref_c.prob, rtol=1e-4)


@pytest.mark.gpu
def test_nb_finalize_kernel_matches_cpu(cuda, tmp_path):
    _, t = _churn_table(tmp_path, 5000, seed=4)
    for laplace in (0.0, 1.0):
        nbc = NaiveBayes(t.schema, laplace=laplace).fit(t)
        nbg = NaiveBayes(t.schema, laplace=laplace).fit(t.to(cuda))
        tc, tg = nbc.tables(), nbg.tables()
        for k in ("logp", "logfp", "logprior"):
            assert torch.allclose(tg[k].cpu(), tc[k].float(), atol=1e-5), (k, laplace)


class _DoublingComm:
    """Stand-in for a 2-rank RCCL communicator on one GPU: all_reduce doubles in place on the
    CURRENT stream (like RCCL, which orders itself after the caller's stream), so the side-stream
    reduce / finalize ordering of NaiveBayes.fit is exercised without a second GPU."""
    is_distributed = True
    backend = "nccl"
    rank, world = 0, 2

    def all_reduce(self, t, op="sum", checked=True):
        torch.cuda._sleep(2_000_000)          # a slow collective: exposes missing waits
        t.add_(t.clone())
        return t

    def check(self, block=True):              # Comm's p2p status gate: nothing can fail here
        pass


@pytest.mark.gpu
def test_nb_side_stream_reduce_ordering(cuda):
    from avenir_amd.data.synth import CHURN_SCHEMA, churn_device
    from avenir_amd.data.table import Table
    from avenir_amd.utils.schema import FeatureSchema
    schema = FeatureSchema.from_json(CHURN_SCHEMA)
    n = 1 << 20
    codes, labels = churn_device(n, seed=3, device=cuda)
    t = Table(schema, n, codes, schema.feature_fields, torch.zeros((0, codes.shape[1]), device=cuda), [],
              labels, schema.find_class_attr_field())
    t.pack_rows()
    single = NaiveBayes(schema).fit(t)
    ref_counts = single.counts.clone() * 2
    ref_tables = {k: v.clone() for k, v in single.tables().items()}
    nb = NaiveBayes(schema, comm=_DoublingComm())
    for _ in range(3):                         # back-to-back fits, reads only at the end
        nb.fit(t)
    assert torch.equal(nb.counts, ref_counts)  # property read waits for the side stream
    tb = nb.tables()
    for k in ("logp", "logfp", "logprior"):
        assert torch.allclose(tb[k], ref_tables[k], atol=1e-6), k
    nb.fit(t)
    pr = nb.predict(t)                         # predict on the main stream waits too
    sp = single.predict(t)
    assert torch.equal(pr.pred, sp.pred)
    assert int(nb.class_n.sum()) == 2 * n
