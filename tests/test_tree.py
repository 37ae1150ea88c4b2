"""Decision tree / random forest / GBT tests: split enumeration, reference-semantics oracle, JSON
model, world-size equivalence, sklearn-parity accuracy, GPU numerics."""
import itertools
import json

import pytest
import torch

from avenir_amd.data import synth
from avenir_amd.data.table import from_arrays, load_csv
from avenir_amd.models.tree import (DecisionTree, DecisionTreeBuilder, GBTParams, GradientBoostedTrees,
                                    RandomForest, TreeEnsemble, TreeParams, build_split_space,
                                    categorical_splits, encode_for_tree, impurity)
from avenir_amd.utils.schema import FeatureField, FeatureSchema

from _dist import run_world


def _hangup(tmp_path, n=3000, seed=0):
    p = tmp_path / "hang.csv"
    p.write_text("\n".join(synth.call_hangup_lines(n, seed=seed)) + "\n")
    schema = FeatureSchema.from_json(synth.CALL_HANGUP_SCHEMA)
    return p, schema, load_csv(p, schema, raw_numeric=True)


def test_categorical_partitions():
    f = FeatureField("x", 1, "categorical", feature=True, cardinality=list("abcd"), max_split=2)
    assert len(categorical_splits(f)) == 7           # Stirling S(4,2)
    f.max_split = 3
    assert len(categorical_splits(f)) == 7 + 6       # + S(4,3)
    for sp in categorical_splits(f):
        assert sorted(set(sp.segmap)) == list(range(sp.n_seg))


def test_numeric_split_space(tmp_path):
    _, schema, t = _hangup(tmp_path, 200)
    space = build_split_space(schema, t)
    hold = [fs for fs in space if fs.field.name == "hold time"][0]
    assert hold.points[:3] == [60, 120, 180] and hold.points[-1] == 540
    assert len(hold.splits) == 9  # maxSplit default 2 -> one point per split
    sp = hold.splits[0]
    assert sp.predicates == ["5 le 60", "5 gt 60"]
    codes = encode_for_tree(space, t)
    x = t.numeric[0, : t.n]
    j = space.index(hold)
    assert torch.equal(codes[j, : t.n].long(), torch.bucketize(x, torch.tensor(hold.points), right=False))


def _oracle_root_split(lines, schema, algorithm="giniIndex"):
    """Brute force over the reference's candidate splits straight from the CSV text."""
    cls = schema.find_class_attr_field()
    best = None
    for fs in build_split_space(schema, None if False else _table_from_lines(lines, schema)):
        for sp in fs.splits:
            seg_counts = [dict() for _ in range(sp.n_seg)]
            for ln in lines:
                it = ln.split(",")
                if fs.kind == "cat":
                    b = fs.field.cardinality.index(it[fs.field.ordinal])
                else:
                    v = float(it[fs.field.ordinal])
                    b = sum(1 for p in fs.points if p < v)
                g = sp.segmap[b]
                seg_counts[g][it[cls.ordinal]] = seg_counts[g].get(it[cls.ordinal], 0) + 1
            tot = sum(sum(d.values()) for d in seg_counts)
            w = 0.0
            nonempty = 0
            for d in seg_counts:
                n = sum(d.values())
                if n == 0:
                    continue
                nonempty += 1
                cnt = torch.tensor([d.get(c, 0) for c in cls.cardinality]).unsqueeze(0)
                w += float(impurity(cnt, algorithm)[0]) * n
            if nonempty < 2:
                continue
            w /= tot
            if best is None or w < best[0] - 1e-12:
                best = (w, sp.predicates)
    return best


def _table_from_lines(lines, schema):
    cols = {}
    for f in schema.fields:
        cols[f.ordinal] = [ln.split(",")[f.ordinal] for ln in lines]
    import copy
    s2 = copy.deepcopy(schema)
    for f in s2.fields:
        if f.is_numeric:
            f.bucket_width = None
            cols[f.ordinal] = [float(v) for v in cols[f.ordinal]]
    return from_arrays(s2, cols)


@pytest.mark.parametrize("algo", ["giniIndex", "entropy"])
def test_root_split_matches_oracle(tmp_path, algo):
    p, schema, t = _hangup(tmp_path, 1500, seed=3)
    lines = p.read_text().splitlines()
    oracle = _oracle_root_split(lines, schema, algo)
    tree = DecisionTreeBuilder(schema, TreeParams(algorithm=algo, max_depth=2)).fit(t)
    root = tree.nodes[0]
    kids = [tree.nodes[c] for c in root.children if c >= 0]
    assert sorted(k.predicates[0] for k in kids) == sorted(
        pp for pp, k in zip(oracle[1], range(len(oracle[1]))))
    assert sum(k.population for k in kids) == 1500


def test_tree_predict_first_matching_path(tmp_path):
    p, schema, t = _hangup(tmp_path, 2000, seed=4)
    tree = DecisionTreeBuilder(schema, TreeParams(max_depth=3, attr_selection="all")).fit(t)
    ens = TreeEnsemble([tree])
    prob = ens.predict_proba(t)
    # python re-implementation of DecisionTreeModel: first path whose predicates all match
    lines = p.read_text().splitlines()

    def match(pred, it):
        a = pred.split()
        v = it[int(a[0])]
        if a[1] == "in":
            return v in a[2].split(":")
        x = float(v)
        if a[1] == "le":
            return x <= float(a[2]) and (len(a) < 4 or x > float(a[3]))
        return x > float(a[2]) and (len(a) < 4 or x <= float(a[3]))
    paths = tree.to_decision_paths()["decisionPaths"]
    for r in range(0, 2000, 97):
        it = lines[r].split(",")
        for dp in paths:
            if all(match(pr["predicateStr"], it) for pr in dp["predicates"][1:]):
                exp = [dp["classValPr"][c] for c in tree.class_values]
                assert torch.allclose(prob[r], torch.tensor(exp, dtype=torch.float32), atol=1e-6)
                break
        else:
            raise AssertionError("no path matched")


def test_decision_path_json(tmp_path):
    _, schema, t = _hangup(tmp_path, 800)
    tree = DecisionTreeBuilder(schema, TreeParams(max_depth=2)).fit(t)
    out = tmp_path / "tree.json"
    tree.save_json(out, total_population=800)
    d = json.loads(out.read_text())
    dp = d["decisionPaths"][0]
    assert dp["predicates"][0]["predicateStr"] == "$root"
    assert set(dp["classValPr"]) == {"T", "F"}
    assert sum(x["population"] for x in d["decisionPaths"]) == 800
    st = tree.state()
    t2 = DecisionTree.from_state(json.loads(json.dumps(st)), schema)
    assert torch.equal(TreeEnsemble([t2]).predict(t), TreeEnsemble([tree]).predict(t))


def test_stopping_strategies(tmp_path):
    _, schema, t = _hangup(tmp_path, 1000)
    tr = DecisionTreeBuilder(schema, TreeParams(stopping="minPopulation", min_population=300,
                                                attr_selection="all")).fit(t)
    for nd in tr.nodes:
        if not nd.is_leaf:
            assert nd.population >= 300
    tr2 = DecisionTreeBuilder(schema, TreeParams(stopping="minInfoGain", min_info_gain=0.5)).fit(t)
    assert all(nd.is_leaf for nd in tr2.nodes[1:])


def _rank_tree(rank, world, path):
    from avenir_amd.parallel.comm import get_comm
    schema = FeatureSchema.from_json(synth.CALL_HANGUP_SCHEMA)
    t = load_csv(path, schema, rank=rank, world=world, raw_numeric=True)
    tr = DecisionTreeBuilder(schema, TreeParams(max_depth=3, split_selection="randomAmongTop"),
                             comm=get_comm()).fit(t)
    return tr.state()


def test_tree_world_size_equivalence(tmp_path):
    p, schema, t = _hangup(tmp_path, 2001, seed=8)
    ref = DecisionTreeBuilder(schema, TreeParams(max_depth=3, split_selection="randomAmongTop")).fit(t).state()
    res = run_world(_rank_tree, 2, str(p))
    for st in res:
        assert [n["predicates"] for n in st["nodes"]] == [n["predicates"] for n in ref["nodes"]]
        assert [n["population"] for n in st["nodes"]] == [n["population"] for n in ref["nodes"]]


def _blobs(n=4000, d=6, seed=0):
    x, y = synth.supervised(n, d, 2, seed=seed, sep=0.5)
    fields = [{"name": f"x{i}", "ordinal": i, "dataType": "double", "feature": True} for i in range(d)]
    fields.append({"name": "y", "ordinal": d, "dataType": "categorical", "cardinality": ["0", "1"]})
    schema = FeatureSchema.from_json({"fields": fields})
    cols = {i: x[:, i].tolist() for i in range(d)}
    cols[d] = [str(v) for v in y.tolist()]
    return schema, from_arrays(schema, cols), x, y


def test_random_forest_accuracy():
    schema, t, x, y = _blobs()
    rf = RandomForest(schema, n_trees=8, params=TreeParams(binary=True, max_depth=6, sub_sampling="withReplace",
                                                           attr_selection="randomAll")).fit(t)
    acc = float((rf.predict(t).cpu() == y).float().mean())
    from sklearn.ensemble import RandomForestClassifier
    sk = RandomForestClassifier(n_estimators=8, max_depth=6, random_state=0).fit(x.numpy(), y.numpy())
    sk_acc = float((torch.tensor(sk.predict(x.numpy())) == y).float().mean())
    assert acc > sk_acc - 0.05, (acc, sk_acc)


def test_gbt_accuracy():
    schema, t, x, y = _blobs(3000, 5, seed=2)
    gb = GradientBoostedTrees(schema, GBTParams(n_estimators=30, max_depth=3, learning_rate=0.12)).fit(t)
    assert gb.train_loss[-1] < gb.train_loss[0]
    acc = float((gb.predict(t).cpu() == y).float().mean())
    from sklearn.ensemble import GradientBoostingClassifier
    sk = GradientBoostingClassifier(n_estimators=30, max_depth=3, learning_rate=0.12).fit(x.numpy(), y.numpy())
    sk_acc = float((torch.tensor(sk.predict(x.numpy())) == y).float().mean())
    assert acc > sk_acc - 0.04, (acc, sk_acc)


def test_gbt_multiclass():
    x, y = synth.supervised(1500, 4, 3, seed=5)
    fields = [{"name": f"x{i}", "ordinal": i, "dataType": "double", "feature": True} for i in range(4)]
    fields.append({"name": "y", "ordinal": 4, "dataType": "categorical", "cardinality": ["0", "1", "2"]})
    schema = FeatureSchema.from_json({"fields": fields})
    cols = {i: x[:, i].tolist() for i in range(4)}
    cols[4] = [str(v) for v in y.tolist()]
    t = from_arrays(schema, cols)
    gb = GradientBoostedTrees(schema, GBTParams(n_estimators=15, max_depth=3)).fit(t)
    pr = gb.predict_proba(t)
    assert pr.shape == (1500, 3)
    assert float((pr.argmax(1) == y).float().mean()) > 0.8


# ------------------------------------------------------------------------------------------------
@pytest.mark.gpu
def test_tree_gpu_matches_cpu(cuda, tmp_path):
    _, schema, t = _hangup(tmp_path, 50_000, seed=11)
    params = TreeParams(max_depth=4, attr_selection="all", algorithm="entropy")
    cpu = DecisionTreeBuilder(schema, params).fit(t).state()
    gpu_tree = DecisionTreeBuilder(schema, params).fit(t.to(cuda))
    gpu = gpu_tree.state()
    assert [n["predicates"] for n in gpu["nodes"]] == [n["predicates"] for n in cpu["nodes"]]
    assert [n["population"] for n in gpu["nodes"]] == [n["population"] for n in cpu["nodes"]]
    tg = t.to(cuda)
    pg = TreeEnsemble([gpu_tree]).predict_proba(tg).cpu()
    pc = TreeEnsemble([DecisionTree.from_state(cpu, schema)]).predict_proba(t)
    assert torch.allclose(pg, pc, atol=1e-6)


@pytest.mark.gpu
def test_forest_and_gbt_gpu(cuda):
    schema, t, x, y = _blobs(20_000, 6, seed=3)
    tg = t.to(cuda)
    rf = RandomForest(schema, n_trees=4, params=TreeParams(binary=True, max_depth=5, sub_sampling="none",
                                                           attr_selection="all")).fit(tg)
    rfc = RandomForest(schema, n_trees=4, params=TreeParams(binary=True, max_depth=5, sub_sampling="none",
                                                            attr_selection="all")).fit(t)
    assert torch.equal(rf.predict(tg).cpu(), rfc.predict(t))
    votes_g = rf.ensemble().predict_votes(tg).cpu()
    votes_c = rfc.ensemble().predict_votes(t)
    assert torch.equal(votes_g, votes_c)
    gb = GradientBoostedTrees(schema, GBTParams(n_estimators=10, max_depth=3)).fit(tg)
    gbc = GradientBoostedTrees(schema, GBTParams(n_estimators=10, max_depth=3)).fit(t)
    assert torch.allclose(gb.predict_proba(tg).cpu(), gbc.predict_proba(t), atol=1e-4)


@pytest.mark.gpu
def test_node_histogram_kernels_match_oracle(cuda):
    """Raw K9 kernels against the CPU oracle: ragged n (not a multiple of the 4-row quads), rows of
    other frontier nodes / left nodes (-1) / nodes past the chunk, zero weights, missing codes."""
    from avenir_amd.ops import tree_ops as TO
    g = torch.Generator().manual_seed(5)
    n, ld = 100_003, 100_016
    bins = [5, 9, 2, 17, 3, 8, 4, 11, 6, 1]
    codes = torch.full((len(bins), ld), 255, dtype=torch.uint8)
    for f, b in enumerate(bins):
        codes[f, :n] = torch.randint(0, b + 1, (n,), generator=g).to(torch.uint8)   # b = missing
    A = 37
    node = torch.randint(-1, A + 3, (ld,), generator=g, dtype=torch.int32)
    labels = torch.randint(0, 3, (ld,), generator=g).to(torch.uint8)
    weight = torch.randint(0, 3, (ld,), generator=g).to(torch.uint8)
    ref = TO.node_histogram(codes, n, labels, node, weight, bins, 3, A)
    got = TO.node_histogram(codes.to(cuda), n, labels.to(cuda), node.to(cuda), weight.to(cuda), bins, 3, A)
    assert torch.equal(got.cpu(), ref)
    gr = torch.randn(ld, generator=g).clamp(-1, 1)          # GBT gradients: |g| <= 1, 0 <= h <= 1
    hs = torch.rand(ld, generator=g)
    ref = TO.node_grad_histogram(codes, n, node, gr, hs, bins, A)
    got = TO.node_grad_histogram(codes.to(cuda), n, node.to(cuda), gr.to(cuda), hs.to(cuda), bins, A)
    assert torch.equal(got.cpu(), ref)
    # packed-sum extremes (every row at |g| = 1, h = 1 in one node), the total slot, left children only
    bt = bins + [1]
    for gv, even, ts in ((1.0, False, sum(bins)), (-1.0, True, sum(bins)), (0.5, False, -1)):
        gg, hh = torch.full((ld,), gv), torch.ones(ld)
        nd = torch.zeros(ld, dtype=torch.int32) if not even else node.abs() % 4
        ref = TO.node_grad_histogram(codes, n, nd, gg, hh, bt, A, even_only=even, tot_slot=ts)
        got = TO.node_grad_histogram(codes.to(cuda), n, nd.to(cuda), gg.to(cuda), hh.to(cuda), bt, A,
                                     even_only=even, tot_slot=ts)
        assert torch.equal(got.cpu(), ref), (gv, even, ts)


# ------------------------------------------------------------------------------------------------
# batched reference-semantics forest (DecisionTreeBuilder.fit_many)
def _tree_sig(tr):
    return [(n.predicates, n.population, n.children) for n in tr.nodes]


REF_PARAMS = dict(stopping="maxDepth", max_depth=3, sub_sampling="withReplace", attr_selection="randomNotUsedYet",
                  random_attr_count=3, split_selection="randomAmongTop", top_split_count=3)


def test_fit_many_equals_one_tree_builds(tmp_path):
    """Every tree of a batched build equals the tree built alone with its seed (the batch shares
    launches, not random streams), multi-way numeric + categorical partition splits."""
    _, schema, t = _hangup(tmp_path, 4000, seed=3)
    for f in schema.feature_fields:
        f.max_split = 3                        # up to 3-way splits (SplitManager maxSplit)
    seeds = [11, 12, 13, 14]
    many = DecisionTreeBuilder(schema, TreeParams(**REF_PARAMS)).fit_many(t, seeds)
    for s, tr in zip(seeds, many):
        one = DecisionTreeBuilder(schema, TreeParams(**REF_PARAMS)).fit_many(t, [s])[0]
        assert _tree_sig(tr) == _tree_sig(one)
    assert any(len(n.children) > 2 for tr in many for n in tr.nodes)   # multi-way splits occur


def test_reference_forest_uses_batched_builder(tmp_path):
    _, schema, t = _hangup(tmp_path, 3000, seed=4)
    rf = RandomForest(schema, 5, TreeParams(**REF_PARAMS), "all").fit(t)
    assert len(rf.trees) == 5 and rf.build_stats["levels"] >= 1
    assert float((rf.predict(t) == t.labels[: t.n].long()).float().mean()) > 0.6


@pytest.mark.gpu
def test_fit_many_gpu_equals_cpu(cuda, tmp_path):
    _, schema, t = _hangup(tmp_path, 60_000, seed=5)
    for extra in ({}, {"algorithm": "entropy", "split_selection": "best", "attr_selection": "notUsedYet"}):
        prm = dict(REF_PARAMS, **extra)
        cpu = DecisionTreeBuilder(schema, TreeParams(**prm)).fit_many(t, [1, 2, 3])
        gpu = DecisionTreeBuilder(schema, TreeParams(**prm)).fit_many(t.to(cuda), [1, 2, 3])
        assert [_tree_sig(x) for x in gpu] == [_tree_sig(x) for x in cpu]


@pytest.mark.gpu
def test_k7_split_kernel_equals_torch_scoring(cuda, tmp_path, monkeypatch):
    """K7 device scoring (csrc/kernels/split.hip) against the torch scoring path on the same device:
    identical trees, node impurities equal to 1e-12."""
    _, schema, t = _hangup(tmp_path, 40_000, seed=8)
    for f in schema.feature_fields:
        f.max_split = 3
    for extra in ({}, {"algorithm": "entropy", "split_selection": "best"}):
        prm = dict(REF_PARAMS, **extra)
        got = DecisionTreeBuilder(schema, TreeParams(**prm)).fit_many(t.to(cuda), [5, 6, 7])
        monkeypatch.setenv("AVMI_TREE_K7", "0")
        ref = DecisionTreeBuilder(schema, TreeParams(**prm)).fit_many(t.to(cuda), [5, 6, 7])
        monkeypatch.delenv("AVMI_TREE_K7")
        assert [_tree_sig(x) for x in got] == [_tree_sig(x) for x in ref]
        for a, b in zip(got, ref):
            for na, nb in zip(a.nodes, b.nodes):
                assert abs(na.info - nb.info) < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("C,algo", [(2, 1), (5, 0), (17, 1)])
def test_k7_kernel_scores_random_histograms(cuda, C, algo):
    """The kernel's k best splits, segment counts and impurities against a float64 host oracle on
    random histograms (multi-class, multi-way segment maps, invalid and non-candidate rows)."""
    from avenir_amd import _native
    from avenir_amd.models.tree import impurity
    g = torch.Generator().manual_seed(C)
    A, F, B = 7, 4, 9
    TB = F * B + 1
    hist = torch.randint(0, 50, (A, C, TB), generator=g, dtype=torch.int64)
    hist[:, :, 3] = 0                                           # an empty bin
    rows, segb = [], []
    for f in range(F):
        for s in range(6):
            ns = 2 + s % 3
            sm = torch.randint(0, ns, (B,), generator=g).tolist()
            sm[:ns] = list(range(ns))
            rows.append([f, f * B, B, ns, int(s != 5), len(segb)])
            segb += sm
    sp = torch.tensor(rows, dtype=torch.int32)
    seg = torch.tensor(segb, dtype=torch.int8)
    cand = (torch.rand(A, F, generator=g) > 0.3).to(torch.uint8)
    k, G2 = 3, 4
    top, topv, segc, cinfo = _native.C().ref_split_score(hist.to(cuda), sp.to(cuda), seg.to(cuda), cand.to(cuda),
                                                         algo, k, G2)
    name = "entropy" if algo == 0 else "giniIndex"
    R = len(rows)
    scores = torch.full((A, R), float("inf"), dtype=torch.float64)
    segs = torch.zeros((A, R, G2, C), dtype=torch.float64)
    for r, (f, col, nb, ns, valid, off) in enumerate(rows):
        for gg in range(ns):
            m = torch.tensor([segb[off + b] == gg for b in range(nb)])
            segs[:, r, gg] = hist[:, :, col:col + nb][:, :, m].double().sum(-1)
        cnt = segs[:, r].sum(-1)
        w = (impurity(segs[:, r], name) * cnt).sum(-1) / cnt.sum(-1).clamp_min(1)
        ok = ((cnt > 0).sum(-1) >= 2) & bool(valid) & cand[:, f].bool()
        scores[:, r] = torch.where(ok, w, scores[:, r])
    order = torch.sort(scores, dim=1, stable=True).indices[:, :k]
    assert torch.equal(top.cpu(), order)
    assert torch.allclose(topv.cpu(), torch.gather(scores, 1, order), rtol=1e-12, atol=0, equal_nan=False) or \
        bool((torch.isinf(topv.cpu()) == torch.isinf(torch.gather(scores, 1, order))).all())
    ref_segc = segs[torch.arange(A).view(-1, 1), order]
    assert torch.equal(segc.cpu(), ref_segc)
    assert torch.allclose(cinfo.cpu(), impurity(ref_segc, name), rtol=1e-12, atol=1e-15)
