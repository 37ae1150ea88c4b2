"""Record-wise exploration / encoding jobs on native input and output (no
per-row Python in the jobs' main paths).

Each job runs twice on the same data: the native path (one-character delimiter: the K1 token
table, device columns, the native formatter writing raw line bytes) and the split-row path (the
same delimiter as the regex ``[,]``) — outputs must be identical.  The keyed / data-parallel ones
also run at world 2 (gloo ranks, byte-range shards) and must equal world 1."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

from avenir_amd.cli import main

from _dist import run_world


def _lines(p):
    p = Path(p)
    if p.is_dir():
        return [l for f in sorted(p.iterdir()) if f.is_file() for l in f.read_text().splitlines() if l.strip()]
    return [l for l in p.read_text().splitlines() if l.strip()]


def _cat_rows(n=700, seed=3):
    rng = np.random.default_rng(seed)
    rows = []
    for i in range(n):
        a = rng.choice(["x", "y", "z", "Y"])
        b = a if rng.random() < 0.7 else rng.choice(["x", "y", "z"])
        c = rng.choice(["p", "q"])
        cls = "T" if (a == "x" and rng.random() < 0.8) or rng.random() < 0.2 else "F"
        rows.append(f"r{i},{a},{b},{c},{cls},{rng.random():.4f},{rng.normal():.5f}")
    return rows


def _setup(tmp: Path, name: str, regex: bool):
    """(argv, config path) of case ``name`` with the literal or the regex delimiter."""
    data = tmp / "d.csv"
    data.write_text("\n".join(_cat_rows()) + "\n")
    dl = "[,]" if regex else ","
    tag = "re" if regex else "lit"
    if name in ("hash", "loo", "loo_test", "dummy", "dummy_ci", "lmap", "ipca"):
        num = tmp / "num.csv"
        if not num.exists():
            rng = np.random.default_rng(8)
            num.write_text("\n".join(f"k{int(rng.integers(0, 9))},{rng.normal():.5f},{rng.normal():.5f},w{i}"
                                     for i in range(900)) + "\n")
        (tmp / "M.txt").write_text("1,1\n1,-1\n0.5,2\n")
        stat = tmp / f"stat_{tag}.txt"
        if name == "loo_test":
            stat.write_text("1,x,100,20\n1,y,50,-10\n1,z,40,2\n1,Y,12,5\n2,x,70,7\n2,y,30,3\n2,z,10,-1\n2,Y,9,1\n")
        block = {
            "hash": ("categoricalFeatureHashingEncoding", "cat.fieldOrdinals = [1,3]\n encoding.size = 6\n"),
            "loo": ("categoricalLeaveOneOutEncoding", f"cat.field.ordinals = [2,1]\n class.field.ordinal = 4\n"
                    f' class.pos.val = "T"\n rand.std.dev = 0.2\n train.data.set = true\n'
                    f' target.stat.file.path = "{stat}"\n'),
            "loo_test": ("categoricalLeaveOneOutEncoding", f"cat.field.ordinals = [1,2]\n class.field.ordinal = 4\n"
                         f' class.pos.val = "T"\n train.data.set = false\n target.stat.file.path = "{stat}"\n'),
            "dummy": ("binaryDummyVariableGenerator", 'cat.field.ordinals = [1,3]\n true.value = "T"\n'),
            "dummy_ci": ("binaryDummyVariableGenerator", "cat.field.ordinals = [1]\n case.insensitive = true\n"
                         ' fieldUniqueValues.1 = ["x", "y"]\n'),
            "lmap": ("linearMapper", f'id.field.ordinals = [3]\n quant.field.ordinals = [1,2]\n'
                     f' retained.field.ordinals = [0]\n trans.matrix.path = "{tmp / "M.txt"}"\n output.precision = 4\n'),
            "ipca": ("incrementalPrincipalComponent", "id.field.ordinals = [0]\n quant.field.ordinals = [1,2]\n"),
        }[name]
        conf = tmp / f"{name}_{tag}.conf"
        conf.write_text(f'{block[0]} {{\n field.delim.in = "{dl}"\n {block[1]}}}\n')
        inp = num if name in ("lmap", "ipca") else data
        return [block[0], "-i", inp], conf
    if name in ("ctime", "etd"):
        rng = np.random.default_rng(12)
        ev = tmp / "ev.txt"
        ev.write_text("\n".join(f"u{int(rng.integers(0, 7))},{int(rng.integers(0, 40 * 86400_000))},"
                                f"{rng.choice(['F', 'P', 'L'])},{rng.choice(['F', 'P', 'L'])}" for _ in range(800)) + "\n")
        rates = tmp / "rates.txt"
        rates.write_text("\n".join("(" + ",".join([f"u{k}"] + [f"{v:.6f}" for v in
                                                              (np.eye(3) * -3 + 1 + 0.1 * k).reshape(-1)]) + ")"
                                   for k in range(7)) + "\n")
        if name == "ctime":
            block = ("contTimeStateTransitionStats", f'key.field.len = 1\n state.values = ["F", "P", "L"]\n'
                     f' time.horizon = 2\n state.trans.file.path = "{rates}"\n state.trans.stat = "StateTransitionCount"\n'
                     f' target.states = ["P", "L"]\n')
            inp = tmp / "ct.txt"
            inp.write_text("\n".join(",".join([l.split(",")[0]] + l.split(",")[2:]) for l in ev.read_text().split()))
        else:
            block = ("eventTimeDistribution", "id.field.ordinals = [0]\n time.field.ordinal = 1\n"
                     ' time.resolution = "dayOfWeek"\n')
            inp = ev
        conf = tmp / f"{name}_{tag}.conf"
        conf.write_text(f'{block[0]} {{\n field.delim.in = "{dl}"\n {block[1]}}}\n')
        return [block[0], "-i", inp], conf
    if name in ("smote", "smote_exp"):
        import json
        rng = np.random.default_rng(21)
        recs = [[f"id{i:04d}", f"{rng.random():.4f}", str(int(rng.integers(0, 50))), str(rng.choice(["u", "v", "w"])), "1"]
                for i in range(300)]
        lines = []
        for i in range(300):
            nbrs = rng.choice(300, int(rng.integers(1, 5)), replace=False)
            lines.append(",".join(recs[i] + [x for j in nbrs for x in recs[j]]))
        lines.append("short,1,2")                      # fewer than two records: skipped
        inp = tmp / "nb.txt"
        inp.write_text("\n".join(lines) + "\n")
        sch = tmp / "sm.json"
        sch.write_text(json.dumps({"fields": [
            {"name": "id", "ordinal": 0, "id": True, "dataType": "string"},
            {"name": "x", "ordinal": 1, "dataType": "double", "feature": True},
            {"name": "k", "ordinal": 2, "dataType": "int", "feature": True},
            {"name": "c", "ordinal": 3, "dataType": "categorical", "feature": True, "cardinality": ["u", "v", "w"]},
            {"name": "cls", "ordinal": 4, "dataType": "categorical", "cardinality": ["0", "1"]}]}))
        cfg = tmp / f"{name}_{tag}.properties"
        cfg.write_text(f"cbos.rec.len=5\ncbos.over.sampling.multiplier=3\ncbos.feature.schema.file.path={sch}\n"
                       f"cbos.neighbor.sampling.distr={'exponential' if name == 'smote_exp' else 'uniform'}\n"
                       f"cbos.random.seed=7\nfield.delim.regex={dl}\n")
        return ["classBasedOverSampler", "-i", inp], cfg
    if name == "relief":
        import json
        rng = np.random.default_rng(31)
        recs = tmp / "recs.txt"
        recs.write_text("\n".join(f"e{i},{rng.choice(['a', 'b'])},{rng.random():.3f},{rng.choice(['u', 'v'])}"
                                   for i in range(200)) + "\n")
        nbh = tmp / "nbh.txt"
        nbh.write_text("\n".join(",".join([f"e{i}", str(rng.choice(['a', 'b'])), str(rng.choice(['a', 'b']))]
                                          + [f"e{int(j)}" for j in rng.choice(210, 4)]) for i in range(200)) + "\n")
        sch = tmp / "rl.json"
        sch.write_text(json.dumps({"fields": [
            {"name": "id", "ordinal": 0, "id": True, "dataType": "string"},
            {"name": "c", "ordinal": 1, "dataType": "categorical", "feature": True, "cardinality": ["a", "b"]},
            {"name": "x", "ordinal": 2, "dataType": "double", "feature": True, "min": 0, "max": 1},
            {"name": "k", "ordinal": 3, "dataType": "categorical", "feature": True, "cardinality": ["u", "v"]}]}))
        cfg = tmp / f"relief_{tag}.properties"
        cfg.write_text(f"ffr.neighborhood.file.path={nbh}\nffr.id.ord=0\nffr.attr.ordinals=1,2,3\n"
                       f"ffr.attr.schema.file.path={sch}\nfield.delim.regex={dl}\n")
        return ["reliefFeatureRelevance", "-i", recs], cfg
    if name == "bag":
        cfg = tmp / f"bag_{tag}.properties"
        cfg.write_text(f"bas.batch.size=64\nbas.random.seed=4\nfield.delim.regex={dl}\n")
        return ["baggingSampler", "-i", data], cfg
    if name in ("nor", "pro", "tef", "tra"):
        if name == "tef":
            rng = np.random.default_rng(13)
            ev = tmp / "tev.txt"
            ev.write_text("\n".join(f"u{int(rng.integers(0, 7))},{int(rng.integers(0, 4000_000))},x" for _ in range(900))
                          + "\n")
            cfg = tmp / f"tef_{tag}.properties"
            cfg.write_text(f"tef.time.stamp.field.ordinal=1\ntef.time.range=100:2000\ntef.time.stamp.in.mili=true\n"
                           f"field.delim.regex={dl}\n")
            return ["temporalFilter", "-i", ev], cfg
        if name == "tra":
            import json
            enc = tmp / "enc.txt"
            enc.write_text("1,x,10\n1,y,20\n3,p,P!\n")
            sch = tmp / "tra.json"
            sch.write_text(json.dumps({"fields": [
                {"name": "a", "ordinal": 1, "transformers": ["keyValueTrans"], "targetFieldOrdinals": [1, 7]},
                {"name": "c", "ordinal": 3, "transformers": ["keyValueTrans"]}]}))
            tconf = tmp / "trans.conf"
            tconf.write_text(f'transformers {{\n keyValueTrans {{\n  hdfsDataPath = "{enc}"\n  fieldDelim = ","\n }}\n}}\n')
            cfg = tmp / f"tra_{tag}.properties"
            cfg.write_text(f"tra.transformer.schema.file.path={sch}\ntra.transformer.config.file.path={tconf}\n"
                           f"field.delim.regex={dl}\n")
            return ["transformer", "-i", data], cfg
        text = {"nor": "nor.num.attribute.ordinals=5,6\nnor.normalizing.strategy=zscore\nnor.force.unit.range=true\n"
                       "nor.floating.precision=4\n",
                "pro": "pro.projection.field=0,5,1\npro.select.filter=5 gt 0.5 and 1 in x:y\n"}[name]
        cfg = tmp / f"{name}_{tag}.properties"
        cfg.write_text(text + f"field.delim.regex={dl}\n")
        return [{"nor": "normalizer", "pro": "projection"}[name], "-i", data], cfg
    if name in ("uvc", "tig", "tig_rep", "nads"):
        rng = np.random.default_rng(14)
        ev = tmp / "tev2.txt"
        ev.write_text("\n".join(f"u{int(rng.integers(0, 9))},{int(rng.integers(0, 400))},{rng.choice(['a', 'B', 'b'])}"
                                f",{rng.random():.3f}" for _ in range(900)) + "\n")
        block = {"uvc": ("uniqueValueCounter", "cat.field.ordinals = [1,3]\n count.values = true\n", data),
                 "tig": ("timeIntervalGenerator", "id.fieldOrdinals = [0]\n time.fieldOrdinal = 1\n", ev),
                 "tig_rep": ("timeIntervalGenerator", "id.fieldOrdinals = [0]\n time.fieldOrdinal = 1\n"
                             " time.keepField = false\n", ev),
                 "nads": ("numericalAttrDistrStats", "id.fieldOrdinals = [1]\n attr.ordinals = [5,6]\n"
                          " attrBinWidth.5 = 0.1\n bin.width = 0.5\n", data)}[name]
        conf = tmp / f"{name}_{tag}.conf"
        conf.write_text(f'{block[0]} {{\n field.delim.in = "{dl}"\n {block[1]}}}\n')
        return [block[0], "-i", block[2]], conf
    if name == "iim":
        items = tmp / "items.txt"
        rng = np.random.default_rng(2)
        items.write_text("\n".join(f"t{i}," + ",".join(rng.choice(list("abcdefgh"), int(rng.integers(1, 6))))
                                   for i in range(500)) + "\n")
        fi = tmp / "fi.txt"
        fi.write_text("a,0.4\nc,0.3\ne,0.2\n")
        cfg = tmp / f"iim_{tag}.properties"
        cfg.write_text(f"iim.item.set.file.path={fi}\niim.skip.field.count=1\nfield.delim.regex={dl}\n")
        return ["infrequentItemMarker", "-i", items], cfg
    props = {
        "spc": ("sequencePositionalCluster", "quant.field.ordinal=6\nseq.num.field.ordinal=5\nwindow.time.span=0.05\n"
                "score.threshold=0.55\ncond.expression=$0 gt 0\n"),
        "kmc": ("kmeansCluster", "kmc.attr.ordinals=5,6\nkmc.num.clusters=2,3\nkmc.max.iterations=20\n"),
        "nuc": ("numericalCorrelation", "nuc.attr.pairs=5:6,6:5\n"),
        "rue": ("ruleEvaluator", "rue.rule.names=r1,r2,r3\nrue.rule.r1=1 eq x > T\n"
                "rue.rule.r2=1 in y:z and 3 eq p > F\nrue.rule.r3=5 gt 0.5 and 6 le 0 > T\nrue.class.attr.ord=4\n"),
        "usb": ("underSamplingBalancer", "usb.class.attr.ord=4\n"),
        "abe": ("adaBoostError", "abe.pred.class.attr.ord=1\nabe.actual.class.attr.ord=2\nabe.boost.attr.ord=5\n"),
    }
    if name == "abu":
        err = tmp / "err.txt"
        err.write_text("error=0.3\n")
        job, text = "adaBoostUpdate", (f"abu.pred.class.attr.ord=1\nabu.actual.class.attr.ord=2\nabu.boost.attr.ord=5\n"
                                       f"abu.error.file.path={err}\nabe.output.precision=5\n")
    else:
        job, text = props[name]
    cfg = tmp / f"{name}_{tag}.properties"
    cfg.write_text(text + f"field.delim.regex={dl}\n")
    return [job, "-i", data], cfg


CASES = ["nuc", "rue", "usb", "abe", "abu", "hash", "loo", "loo_test", "dummy", "dummy_ci", "lmap", "ipca", "spc",
         "kmc", "ctime", "etd", "iim", "smote", "smote_exp", "relief", "bag", "nor", "pro", "tef", "tra", "uvc", "tig", "tig_rep", "nads"]


@pytest.mark.parametrize("name", CASES)
def test_native_equals_row_path(tmp_path, name):
    argv, cfg = _setup(tmp_path, name, False)
    assert main([str(a) for a in argv] + ["-o", str(tmp_path / "native"), "-c", str(cfg), "--device", "cpu"]) == 0
    argv, cfg2 = _setup(tmp_path, name, True)
    assert main([str(a) for a in argv] + ["-o", str(tmp_path / "rows"), "-c", str(cfg2), "--device", "cpu"]) == 0
    got, ref = _lines(tmp_path / "native"), _lines(tmp_path / "rows")
    assert got and got == ref
    if name == "loo":
        assert _lines(tmp_path / "stat_lit.txt") == _lines(tmp_path / "stat_re.txt")


def _world(rank, world, argv, out, cfg):
    assert main([str(a) for a in argv] + ["-o", out, "-c", cfg, "--device", "cpu"]) == 0
    return True


@pytest.mark.parametrize("name", ["rue", "usb", "abe", "hash", "dummy", "lmap", "ipca", "spc", "ctime", "etd", "iim", "smote", "relief", "bag", "nor", "pro", "tef", "tra", "uvc", "tig", "tig_rep", "nads", "loo"])
def test_world2_equals_world1(tmp_path, name):
    argv, cfg = _setup(tmp_path, name, False)
    assert main([str(a) for a in argv] + ["-o", str(tmp_path / "w1"), "-c", str(cfg), "--device", "cpu"]) == 0
    run_world(_world, 2, [str(a) for a in argv], str(tmp_path / "w2"), str(cfg), timeout=300)
    assert _lines(tmp_path / "w2") == _lines(tmp_path / "w1")


def test_word_count_native_equals_counter(tmp_path):
    from collections import Counter
    rng = np.random.default_rng(5)
    words = ["alpha", "beta", "gamma", "delta", "Zeta", "éta"]
    text = "\n".join(" ".join(rng.choice(words, int(rng.integers(0, 9)))) + ("\t  x" if i % 7 == 0 else "")
                     for i in range(2000)) + "\n"
    inp = tmp_path / "t.txt"
    inp.write_text(text)
    ref = [f"{w},{n}" for w, n in sorted(Counter(w for l in text.splitlines() for w in l.split()).items())]
    assert main(["wordCount", "-i", str(inp), "-o", str(tmp_path / "w1"), "--device", "cpu"]) == 0
    assert _lines(tmp_path / "w1") == ref
    run_world(_world_wc, 2, str(inp), str(tmp_path / "w2"), timeout=300)
    assert _lines(tmp_path / "w2") == ref


def _world_wc(rank, world, inp, out):
    assert main(["wordCount", "-i", inp, "-o", out, "--device", "cpu"]) == 0
    return True


def _docs(tmp, n=800, seed=9):
    rng = np.random.default_rng(seed)
    words = ["Cheap", "pills", "offer", "NOW", "meeting", "agenda", "Monday", "the", "a", "prize!", "win",
             "project", "notes", "x2", "co-op", "É", "review."]
    rows = []
    for _ in range(n):
        spam = rng.random() < 0.4
        ws = rng.choice(words[:5] + words[8:11] if spam else words[4:], int(rng.integers(1, 9)))
        rows.append(" ".join(ws) + ("," + ("spam" if spam else "ham-ok")))
    p = tmp / "docs.txt"
    p.write_text("\n".join(rows) + "\n")
    q = tmp / "q.txt"
    q.write_text("\n".join(" ".join(rng.choice(words, 4)) + ",?" for _ in range(300)) + "\n")
    return p, q


@pytest.mark.parametrize("world", [1, 2])
def test_text_nb_native_equals_row_path(tmp_path, world):
    data, q = _docs(tmp_path)
    outs = {}
    for regex in (False, True):
        dl = "[,]" if regex else ","
        cfg = tmp_path / f"t{int(regex)}.properties"
        cfg.write_text(f"bad.tabular.input=false\nbap.tabular.input=false\nfield.delim.regex={dl}\n")
        model, out = tmp_path / f"m{int(regex)}.txt", tmp_path / f"p{int(regex)}"
        if world == 1 or regex:
            assert main(["bayesianDistribution", "-i", str(data), "-o", str(model), "-c", str(cfg), "--device", "cpu"]) == 0
            assert main(["bayesianPredictor", "-i", str(q), "-o", str(out), "-c", str(cfg), "--model", str(model),
                         "--device", "cpu"]) == 0
        else:
            run_world(_world_nb, 2, str(data), str(q), str(cfg), str(model), str(out), timeout=300)
        outs[regex] = (_lines(model), _lines(out))
    assert outs[False][0] and outs[False] == outs[True]


def _world_nb(rank, world, data, q, cfg, model, out):
    assert main(["bayesianDistribution", "-i", data, "-o", model, "-c", cfg, "--device", "cpu"]) == 0
    from avenir_amd.parallel.comm import get_comm
    get_comm().barrier()
    assert main(["bayesianPredictor", "-i", q, "-o", out, "-c", cfg, "--model", model, "--device", "cpu"]) == 0
    return True


def _sts_world(rank, world, argv, out):
    assert main(argv + ["-o", out, "--device", "cpu"]) == 0
    return True


@pytest.mark.parametrize("topk", [0, 5])
def test_same_type_similarity_world_invariant(tmp_path, topk):
    """sameTypeSimilarity with both sets row-sharded (training shards on the ring for top-k, one
    all-gather for all pairs): world 2 writes exactly the world-1 output."""
    from avenir_amd.data.fixtures import FIXTURES
    fix = Path(__file__).parent / "fixtures"
    data = FIXTURES["elearn"](300, seed=7, as_int=True)
    tr, te = tmp_path / "train.txt", tmp_path / "test.txt"
    tr.write_text("\n".join(data[:200]) + "\n")
    te.write_text("\n".join(data[200:]) + "\n")
    props = tmp_path / "sts.properties"
    props.write_text(f"sts.same.schema.file.path={fix / 'elearnActivity.json'}\nsts.distance.scale=1000\n"
                     f"sts.top.match.count={topk}\n")
    argv = ["sameTypeSimilarity", "-i", str(te), "--train", str(tr), "-c", str(props)]
    assert main(argv + ["-o", str(tmp_path / "w1"), "--device", "cpu"]) == 0
    w1 = _lines(tmp_path / "w1")
    assert len(w1) == 100 * (topk or 200)
    run_world(_sts_world, 2, argv, str(tmp_path / "w2"), timeout=300)
    assert _lines(tmp_path / "w2") == w1


def _close_lines(a: list[str], b: list[str], rel=1e-4, abs_=2e-3):
    """Line-by-line equality with numeric fields compared approximately (GPU float math)."""
    assert len(a) == len(b)
    for x, y in zip(a, b):
        if x == y:
            continue
        fx, fy = x.strip("()").split(","), y.strip("()").split(",")
        assert len(fx) == len(fy), (x, y)
        for u, v in zip(fx, fy):
            if u != v:
                assert abs(float(u) - float(v)) <= abs_ + rel * abs(float(v)), (x, y)


GPU_CASES = ["rue", "usb", "abe", "abu", "hash", "loo_test", "dummy", "lmap", "spc", "ctime", "etd", "iim", "smote",
             "relief", "bag", "nor", "pro", "tef", "tra", "uvc", "tig", "nads"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", GPU_CASES)
def test_native_jobs_gpu_equal_cpu(tmp_path, name, monkeypatch):
    """The device tokenizer (forced on small files) + device kernels against the CPU run."""
    from avenir_amd.data import records as R
    monkeypatch.setattr(R, "DEVICE_MIN_BYTES", 0)
    monkeypatch.setattr(R, "DEVICE_FORMAT_MIN_ROWS", 0)
    argv, cfg = _setup(tmp_path, name, False)
    assert main([str(a) for a in argv] + ["-o", str(tmp_path / "gpu"), "-c", str(cfg), "--device", "cuda"]) == 0
    assert main([str(a) for a in argv] + ["-o", str(tmp_path / "cpu"), "-c", str(cfg), "--device", "cpu"]) == 0
    g, c = _lines(tmp_path / "gpu"), _lines(tmp_path / "cpu")
    assert c
    _close_lines(g, c)


def test_distance_store_native_equals_python(tmp_path):
    """entityDistanceStore from pair lines: the code-based CSR build equals write_pairs."""
    import numpy as np
    from avenir_amd.utils.distance_store import EntityDistanceStore
    rng = np.random.default_rng(2)
    pairs = [(f"e{int(rng.integers(0, 60))}", f"e{int(rng.integers(0, 60))}", float(rng.integers(1, 999)))
             for _ in range(700)]
    inp = tmp_path / "pairs.txt"
    inp.write_text("\n".join(f"{a},{b},{int(d)}" for a, b, d in pairs) + "\n")
    cfg = tmp_path / "eds.properties"
    cfg.write_text("eds.pair.input=true\n")
    assert main(["entityDistanceStore", "-i", str(inp), "-o", str(tmp_path / "native"), "-c", str(cfg),
                 "--device", "cpu"]) == 0
    EntityDistanceStore.write_pairs([a for a, _, _ in pairs], [b for _, b, _ in pairs], [d for _, _, d in pairs],
                                    tmp_path / "py")
    for f in ("indptr.npy", "cols.npy", "vals.npy"):
        assert np.array_equal(np.load(tmp_path / "native" / f), np.load(tmp_path / "py" / f)), f
    assert (tmp_path / "native" / "entities.json").read_text() == (tmp_path / "py" / "entities.json").read_text()


@pytest.mark.parametrize("name", ["spc", "rue", "pro"])
def test_jobs_with_no_output_rows(tmp_path, name):
    """A job whose selection keeps no line writes an empty output (the native formatter got null
    span pointers for an empty selection and raised)."""
    argv, cfg = _setup(tmp_path, name, False)
    text = cfg.read_text()
    text = {"spc": lambda t: t.replace("score.threshold=0.55", "score.threshold=1.5"),
            "rue": lambda t: t,
            "pro": lambda t: t.replace("5 gt 0.5", "5 gt 5.0")}[name](text)
    cfg.write_text(text)
    assert main([str(a) for a in argv] + ["-o", str(tmp_path / "out"), "-c", str(cfg), "--device", "cpu"]) == 0
    if name != "rue":
        assert _lines(tmp_path / "out") == []


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["spc", "pro", "usb"])
def test_jobs_with_no_output_rows_gpu(tmp_path, name):
    """The same on the device paths (device tokenizer, device formatter)."""
    argv, cfg = _setup(tmp_path, name, False)
    text = cfg.read_text()
    text = {"spc": lambda t: t.replace("score.threshold=0.55", "score.threshold=1.5"),
            "pro": lambda t: t.replace("5 gt 0.5", "5 gt 5.0"),
            "usb": lambda t: t}[name](text)
    cfg.write_text(text)
    assert main([str(a) for a in argv] + ["-o", str(tmp_path / "out"), "-c", str(cfg), "--device", "cuda"]) == 0
    if name != "usb":
        assert _lines(tmp_path / "out") == []


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["loo", "loo_test", "nuc", "hash", "dummy", "rue", "nads", "spc", "bag"])
def test_gpu_equals_cpu(tmp_path, name):
    """The device paths of the record-wise jobs (device tokenizer, LDS-privatised statistics,
    device formatter) write what the host paths write."""
    argv, cfg = _setup(tmp_path, name, False)
    outs = {}
    for dev in ("cpu", "cuda"):
        assert main([str(a) for a in argv] + ["-o", str(tmp_path / dev), "-c", str(cfg), "--device", dev]) == 0
        outs[dev] = _lines(tmp_path / dev)
        if name == "loo":
            outs[dev + "_stat"] = _lines(tmp_path / "stat_lit.txt")
    if name == "nuc":       # fp64 sums in another order: equal to the last couple of digits
        a = [float(l.split(",")[-1]) for l in outs["cpu"]]
        b = [float(l.split(",")[-1]) for l in outs["cuda"]]
        assert a and np.allclose(a, b, rtol=1e-12, atol=1e-15)
        return
    assert outs["cpu"] and outs["cpu"] == outs["cuda"]
    if name == "loo":
        assert outs["cpu_stat"] == outs["cuda_stat"]
