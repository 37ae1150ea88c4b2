"""Prediction and sequence jobs on native input and output.

``viterbiStatePredictor``, ``markovModelClassifier``, ``probabilisticSuffixTreeGenerator`` (K5),
``bayesianPredictor``, ``decisionTree`` (level mode), ``modelPredictor`` and ``knnClassifier`` read
their input through the native record / CSV parsers and write through the native formatter with
the input lines kept as byte spans (data/lines.py).  Each job runs twice on the same data: the
native path (one-character delimiter) and the split-row path (the same delimiter as the regex
``[,]``) — outputs must be identical.  World 3 (gloo ranks, byte-range shards) must equal world 1.
GPU: the device tokenizer / device CSV parser + kernels against the CPU run."""
from __future__ import annotations

import json
import random
from pathlib import Path

import pytest

from avenir_amd.cli import main
from avenir_amd.data import records as R
from avenir_amd.data import synth
from avenir_amd.data import synth_text as S
from avenir_amd.data import table as TB

from _dist import run_world


def _lines(p):
    p = Path(p)
    if p.is_dir():
        return [l for f in sorted(p.iterdir()) if f.is_file() for l in f.read_text().splitlines() if l.strip()]
    return [l for l in p.read_text().splitlines() if l.strip()]


def _run(args):
    assert main([str(a) for a in args]) == 0


def _obs_file(path, tagged, n_unknown=25):
    """``id,o,o,...`` observation rows from the tagged sequences, some with an unknown token."""
    rnd = random.Random(5)
    out = []
    for i, ln in enumerate(tagged.read_text().splitlines()):
        f = ln.split(",")
        obs = [t.split(":")[0] for t in f[1:]]
        if i < n_unknown:
            obs[rnd.randrange(len(obs))] = "zz"
        out.append(",".join([f[0]] + obs[: rnd.randint(1, len(obs))]))
    path.write_text("\n".join(out) + "\n")


def _setup(tmp: Path, name: str):
    """(job argv without the config, config text) for case ``name``; models are built here."""
    if name.startswith("vit"):
        tagged = tmp / "tagged.txt"
        S.tagged_sequences(tagged, 2000, seed=3)
        hcfg = tmp / "hmm.properties"
        hcfg.write_text("hmmb.model.states=S,T,U\nhmmb.model.observations=a,b,c,d\nhmmb.skip.field.count=1\n"
                        "hmmb.trans.prob.scale=1000\n")
        model = tmp / "hmm.txt"
        _run(["hiddenMarkovModelBuilder", "-i", tagged, "-o", model, "-c", hcfg, "--device", "cpu"])
        data = tmp / "obs.txt"
        _obs_file(data, tagged)
        extra = "vsp.output.state.only=false\nvsp.sub.field.delim=:\n" if name == "vit_pairs" else ""
        return ["viterbiStatePredictor", "-i", data, "--model", model], "vsp.skip.field.count=1\n" + extra
    if name == "mmc":
        data = tmp / "seq.txt"
        S.state_sequences(data, 3000, seed=4)
        mcfg = tmp / "mst.properties"
        mcfg.write_text("mst.model.states=" + ",".join(S.STATES) + "\nmst.skip.field.count=2\n"
                        "mst.class.label.field.ord=1\nmst.class.labels=T,F\n")
        model = tmp / "mm.txt"
        _run(["markovStateTransitionModel", "-i", data, "-o", model, "-c", mcfg, "--device", "cpu"])
        return (["markovModelClassifier", "-i", data, "--model", model],
                "mmc.class.labels=T,F\nmmc.skip.field.count=2\nmmc.validation.mode=true\n"
                "mmc.class.label.field.ord=1\nmmc.log.odds.threshold=0.1\n")
    if name.startswith("pst"):
        if name == "pst_stream":
            data = tmp / "ev.txt"
            S.events(data, 4000, n_keys=30, seed=6)
            return (["probabilisticSuffixTreeGenerator", "-i", data],
                    "pstg.input.format.sequential=false\npstg.data.field.ordinal=2\npstg.id.field.ordinals=0\n"
                    "pstg.max.seq.length=3\n")
        data = tmp / "seq.txt"
        S.state_sequences(data, 3000, seq_len=7, seed=7)
        extra = "pstg.id.field.ordinals=0\n" if name == "pst_id" else ""
        return (["probabilisticSuffixTreeGenerator", "-i", data],
                "pstg.skip.field.count=1\npstg.class.label.field.ord=1\npstg.max.seq.length=4\n" + extra)
    if name.startswith("nbp"):
        data, schema = tmp / "churn.csv", tmp / "churn.json"
        synth.write_churn(data, 3000, seed=1, schema_path=schema)
        model = tmp / "nb.txt"
        _run(["bayesianDistribution", "-i", data, "-o", model, "--schema", schema, "--device", "cpu"])
        extra = "bap.output.feature.prob.only=true\n" if name == "nbp_fp" else ""
        return ["bayesianPredictor", "-i", data, "--schema", schema, "--model", model], extra
    data, schema = tmp / "hangup.csv", tmp / "hangup.json"
    data.write_text("\n".join(synth.call_hangup_lines(2500, seed=2)) + "\n")
    schema.write_text(json.dumps(synth.CALL_HANGUP_SCHEMA))
    if name == "detr":
        return (["decisionTree", "-i", data, "--schema", schema],
                "dtb.split.algorithm=giniIndex\ndtb.path.stopping.strategy=maxDepth\ndtb.max.depth.limit=3\n"
                f"dtb.decision.file.path.out={tmp / 'dp_out.json'}\n")
    if name == "knn":
        return ["knnClassifier", "-i", data, "--train", data, "--schema", schema], "nen.top.match.count=5\n"
    # modelPredictor over a small forest
    cls_ord = [f["ordinal"] for f in synth.CALL_HANGUP_SCHEMA["fields"] if not f.get("feature") and not f.get("id")][0]
    forest = tmp / "forest"
    fcfg = tmp / "rafo.properties"
    fcfg.write_text(f"dtb.feature.schema.file.path={schema}\ndtb.split.algorithm=giniIndex\n"
                    "dtb.path.stopping.strategy=maxDepth\ndtb.max.depth.limit=3\ndtb.num.trees=3\n")
    _run(["randomForest", "-i", data, "-o", forest, "-c", fcfg, "--device", "cpu"])
    mode = "withRecord" if name == "mop" else "withActualClassAttr"
    return (["modelPredictor", "-i", data],
            f"mop.model.dir.path={forest}\nmop.output.mode={mode}\nmop.rec.id.ordinal=0\n"
            f"mop.rec.class.attr.ordinal={cls_ord}\n")


CASES = ["vit", "vit_pairs", "mmc", "pst", "pst_id", "pst_stream", "nbp", "nbp_fp", "detr", "knn", "mop", "mop_cls"]


def _cfg(tmp, text, regex=False, tag=""):
    p = tmp / f"job{tag}{'_re' if regex else ''}.properties"
    p.write_text(text + ("field.delim.regex=[,]\n" if regex else "field.delim.regex=,\n"))
    return p


@pytest.mark.parametrize("name", CASES)
def test_native_output_equals_row_path(tmp_path, name):
    argv, text = _setup(tmp_path, name)
    _run(argv + ["-o", tmp_path / "native.txt", "-c", _cfg(tmp_path, text), "--device", "cpu"])
    _run(argv + ["-o", tmp_path / "rows.txt", "-c", _cfg(tmp_path, text, regex=True), "--device", "cpu"])
    got, ref = _lines(tmp_path / "native.txt"), _lines(tmp_path / "rows.txt")
    assert got and got == ref


def _world(rank, world, argv, out, cfg):
    assert main([str(a) for a in argv] + ["-o", out, "-c", cfg, "--device", "cpu"]) == 0
    return True


@pytest.mark.parametrize("name", ["vit", "mmc", "pst", "pst_stream", "mop", "nbp"])
def test_native_predictors_world_invariant(tmp_path, name):
    argv, text = _setup(tmp_path, name)
    cfg = _cfg(tmp_path, text)
    _run(argv + ["-o", tmp_path / "w1.txt", "-c", cfg, "--device", "cpu"])
    run_world(_world, 3, [str(a) for a in argv], str(tmp_path / "w3.txt"), str(cfg), timeout=300)
    assert _lines(tmp_path / "w3.txt") == _lines(tmp_path / "w1.txt")


def test_pst_matches_reference_semantics(tmp_path):
    """The class field counts into the skip (ProbabilisticSuffixTreeGenerator.java:118-122) and the
    root line carries the configured root symbol."""
    data = tmp_path / "s.txt"
    data.write_text("u1,T,A,B,A\nu2,F,B,B\nu3,T,A\n")
    cfg = _cfg(tmp_path, "pstg.skip.field.count=1\npstg.class.label.field.ord=1\npstg.max.seq.length=3\n"
                         "pstg.tree.root.symbol=#\n")
    _run(["probabilisticSuffixTreeGenerator", "-i", data, "-o", tmp_path / "o.txt", "-c", cfg, "--device", "cpu"])
    assert _lines(tmp_path / "o.txt") == ["F,#,1", "F,B,B,1", "T,#,3", "T,A,B,1", "T,A,B,A,1", "T,B,A,1"]


def _close(a: list[str], b: list[str], rel=1e-4, abs_=2e-3):
    """Line-by-line equality with numeric fields compared approximately (GPU float math)."""
    assert len(a) == len(b)
    for x, y in zip(a, b):
        if x == y:
            continue
        fx, fy = x.split(","), y.split(",")
        assert len(fx) == len(fy), (x, y)
        for u, v in zip(fx, fy):
            if u == v:
                continue
            fu, fv = float(u), float(v)
            assert abs(fu - fv) <= abs_ + rel * abs(fv), (x, y)


def _knn_tie_rows(data, schema_path, k: int, rel: float = 2e-5) -> set[int]:
    """Rows whose k-th and (k+1)-th nearest training records are equidistant up to fp32 rounding
    under the knnClassifier distance (min-max scaled numeric terms + a weight-2 category mismatch,
    1 against a missing value), computed in fp64 on the host: the only rows where two correct
    implementations (fp32 MFMA vs fp64, or mixed vs one-hot) may pick different neighbour sets."""
    import torch
    from avenir_amd.data import table as TBm
    from avenir_amd.jobs.core import _category_codes, _numeric_block
    from avenir_amd.utils.schema import FeatureSchema
    schema = FeatureSchema.from_json(Path(schema_path))
    t = TBm.load_csv(str(data), schema, raw_numeric=True)
    X = _numeric_block(t).double()
    lo, hi = X.min(0).values, X.max(0).values
    X = (X - lo) / (hi - lo).clamp_min(1e-12)
    C = _category_codes(t).long()
    d2 = torch.cdist(X, X) ** 2
    for f in range(C.shape[1]):
        a, b = C[:, f].view(-1, 1), C[:, f].view(1, -1)
        d2 += torch.where((a < 0) & (b < 0), 0.0, torch.where((a < 0) | (b < 0), 1.0, torch.where(a != b, 2.0, 0.0)))
    srt = d2.clamp_min(0).sqrt().sort(1).values
    dk, dk1 = srt[:, k - 1], srt[:, k]
    return set(torch.nonzero((dk1 - dk).abs() <= rel * (1 + dk)).view(-1).tolist())


def _assert_knn_equal_except_ties(a: list[str], b: list[str], tmp_path, k: int):
    """Every differing prediction must sit on a row where the k-th neighbour is tied."""
    assert len(a) == len(b)
    assert [x.rsplit(",", 1)[0] for x in a] == [y.rsplit(",", 1)[0] for y in b]
    diff = [i for i, (x, y) in enumerate(zip(a, b)) if x != y]
    if diff:
        ties = _knn_tie_rows(tmp_path / "hangup.csv", tmp_path / "hangup.json", k)
        assert set(diff) <= ties, f"non-tie rows differ: {sorted(set(diff) - ties)[:10]}"


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_native_predictors_gpu_equal_cpu(tmp_path, name, monkeypatch):
    monkeypatch.setattr(R, "DEVICE_MIN_BYTES", 0)        # device tokenizer on small files too
    monkeypatch.setattr(R, "DEVICE_FORMAT_MIN_ROWS", 0)  # device output formatter too
    monkeypatch.setattr(TB, "_GPU_CSV_MIN_BYTES", 0)     # device CSV parser too
    argv, text = _setup(tmp_path, name)
    cfg = _cfg(tmp_path, text)
    _run(argv + ["-o", tmp_path / "gpu.txt", "-c", cfg, "--device", "cuda"])
    _run(argv + ["-o", tmp_path / "cpu.txt", "-c", cfg, "--device", "cpu"])
    g, c = _lines(tmp_path / "gpu.txt"), _lines(tmp_path / "cpu.txt")
    if name in ("mmc", "nbp", "nbp_fp"):
        _close(g, c)
    elif name == "knn":      # equidistant neighbours: MFMA fp32 vs fp64 distances may break ties apart
        _assert_knn_equal_except_ties(g, c, tmp_path, 5)
    else:
        assert g == c


def _knn_oracle_pair(device):
    """Mixed-type kNN (numeric block + category codes) and the one-hot oracle on the same records."""
    import torch
    from avenir_amd.models.knn import NearestNeighbor
    g = torch.Generator().manual_seed(4)
    n, q = 1500, 400
    Xn = torch.rand((n + q, 5), generator=g)
    Xc = torch.randint(0, 4, (n + q, 3), generator=g).int()
    Xc[::37, 1] = -1                                        # missing categories
    oh = torch.cat([torch.nn.functional.one_hot(Xc[:, j].long().clamp_min(0), 4).float()
                    * (Xc[:, j:j + 1] >= 0) for j in range(3)], 1)
    y = (Xn[:, 0] + (Xc[:, 0] == 2).float() > 0.9).long()
    wc = torch.full((3,), 2.0)
    dev = torch.device(device)
    m = NearestNeighbor(k=7).fit_mixed(Xn[:n].to(dev), Xc[:n].to(dev), wc.to(dev), y[:n].to(dev), 2)
    o = NearestNeighbor(k=7).fit(torch.cat([Xn, oh], 1)[:n].to(dev), y[:n].to(dev), 2)
    dm, _ = m.kneighbors(Xn[n:].to(dev), Qc=Xc[n:].to(dev))
    do, _ = o.kneighbors(torch.cat([Xn, oh], 1)[n:].to(dev))
    return dm.cpu(), do.cpu()


def test_mixed_knn_equals_one_hot_oracle_cpu():
    dm, do = _knn_oracle_pair("cpu")
    assert (dm - do).abs().max() < 1e-4


@pytest.mark.gpu
def test_mixed_knn_equals_one_hot_oracle_gpu(cuda):
    dm, do = _knn_oracle_pair(cuda)
    assert (dm - do).abs().max() < 1e-3


def test_knn_job_mixed_path_matches_one_hot_fallback(tmp_path, monkeypatch):
    """knnClassifier with categorical attributes runs mixed_knn (no one-hot matrix); forcing the
    one-hot fallback (column limit 0) gives the same predictions up to equidistant-neighbour ties."""
    from avenir_amd.ops import distance as D
    argv, text = _setup(tmp_path, "knn")
    cfg = _cfg(tmp_path, text)
    calls = []
    real = D.distributed_knn_mixed
    monkeypatch.setattr(D, "distributed_knn_mixed", lambda *a, **k: calls.append(1) or real(*a, **k))
    _run(argv + ["-o", tmp_path / "mixed.txt", "-c", cfg, "--device", "cpu"])
    assert calls, "the mixed-type path did not run"
    monkeypatch.setattr(D, "mixed_knn_max_dims", lambda: 0)
    _run(argv + ["-o", tmp_path / "onehot.txt", "-c", cfg, "--device", "cpu"])
    a, b = _lines(tmp_path / "mixed.txt"), _lines(tmp_path / "onehot.txt")
    _assert_knn_equal_except_ties(a, b, tmp_path, 5)
