"""Multi-rank equivalence at world sizes 1, 2, 4 and 8 (gloo, CPU processes): every distributed
model trained on row shards must give the single-process result — counts bit-exact, floats within
tolerance.  One spawn per world size runs all models."""
import json
import os
import tempfile

import numpy as np
import pytest
import torch

from _dist import run_world
from avenir_amd.data import synth


def _data():
    d = tempfile.mkdtemp(prefix="avmi_ws_")
    churn = os.path.join(d, "churn.csv")
    synth.write_churn(churn, 3001, seed=5)
    hang = os.path.join(d, "hangup.csv")
    with open(hang, "w") as fh:
        fh.write("\n".join(synth.call_hangup_lines(2003, seed=8)) + "\n")
    rng = np.random.default_rng(7)
    seqs = [[str(x) for x in rng.integers(0, 4, 12)] for _ in range(401)]
    tagged = [[f"{'ab'[int(s) % 2]}:{'HL'[int(s) // 2]}" for s in row] for row in seqs]
    tx = [sorted({f"i{int(v)}" for v in rng.integers(0, 9, 5)}) for _ in range(503)]
    return churn, hang, seqs, tagged, tx


def _shard(xs, rank, world):
    n = len(xs)
    return xs[rank * n // world:(rank + 1) * n // world]


def _all_models(rank, world, churn, hang, seqs, tagged, tx, dev="cpu"):
    from avenir_amd.data.table import load_csv
    from avenir_amd.models import tree as T
    from avenir_amd.models.association import Apriori
    from avenir_amd.models.bayes import NaiveBayes
    from avenir_amd.models.cluster import KMeans
    from avenir_amd.models.explore import MutualInformation, categorical_correlation
    from avenir_amd.models.forest import ForestBuilder
    from avenir_amd.models.linear import LogisticRegression
    from avenir_amd.models.markov import (HiddenMarkovModelBuilder, MarkovStateTransitionModel,
                                          ProbabilisticSuffixTree)
    from avenir_amd.ops import distance as D
    from avenir_amd.ops import sequence_ops as SO
    from avenir_amd.parallel.comm import get_comm
    from avenir_amd.utils.schema import FeatureSchema
    comm = get_comm()
    out = {}
    # ---- counting models: bit-exact -----------------------------------------------------------
    cs = FeatureSchema.from_json(synth.CHURN_SCHEMA)
    t = load_csv(churn, cs, rank=rank, world=world, device=dev)
    nb = NaiveBayes(cs, comm=comm).fit(t)
    out["nb"] = (nb.counts.tolist(), nb.class_n.tolist())
    mi = MutualInformation(comm=comm)
    r = mi.fit(t)
    out["mi"] = sorted((k, round(v, 12)) for k, v in r.feature_class.items())
    out["cramer"] = sorted((k, round(v, 12)) for k, v in categorical_correlation(t, comm=comm).items())
    m = MarkovStateTransitionModel(["0", "1", "2", "3"], comm=comm)
    m.fit(m.encode(_shard(seqs, rank, world)).to(dev))
    out["markov"] = m.counts.tolist()
    hb = HiddenMarkovModelBuilder(["H", "L"], ["a", "b"], comm=comm)
    ob, st = hb.encode(_shard(tagged, rank, world))
    ob, st = ob.to(dev), st.to(dev)
    hmm = hb.fit(ob, st)
    out["hmm"] = (hmm.A.tolist(), hmm.B.tolist(), hmm.pi.tolist())
    pst = ProbabilisticSuffixTree(4, 3).fit(m.encode(_shard(seqs, rank, world)).to(dev), comm=comm)
    out["pst"] = [(tok, ch.count) for tok, ch in sorted(pst.root.children.items())]
    fi = Apriori(0.08, max_len=3, comm=comm).fit_transactions(_shard(tx, rank, world), device=dev)
    out["apriori"] = sorted((tuple(fi.items[i] for i in s), c) for lvl in fi.levels.values() for s, c in lvl)
    # ---- trees: level-wise builder (data parallel), forest data-parallel and tree-parallel ----
    hs = FeatureSchema.from_json(synth.CALL_HANGUP_SCHEMA)
    th = load_csv(hang, hs, rank=rank, world=world, raw_numeric=True, device=dev)
    full = load_csv(hang, hs, raw_numeric=True, device=dev)
    tr = T.DecisionTreeBuilder(hs, T.TreeParams(max_depth=3), comm=comm).fit(th)
    out["tree"] = [(n.predicates, n.population) for n in tr.nodes]
    prm = T.TreeParams(binary=True, stopping="maxDepth", max_depth=4, attr_selection="all", sub_sampling="none")
    space = T.build_split_space(hs, full, binary=True, max_bins=32)
    fb = ForestBuilder(hs, 2, prm, comm=comm).fit(th, space=space, codes=T.encode_for_tree(space, th))
    out["forest_dp"] = [[(n.predicates, n.population) for n in x.nodes] for x in fb]
    rf = T.RandomForest(hs, 6, T.TreeParams(binary=True, stopping="maxDepth", max_depth=4,
                                            sub_sampling="withReplace", attr_selection="randomAll", seed=3),
                        "sqrt", comm=comm, tree_parallel=True).fit(full)
    out["forest_tp"] = [[(n.predicates, n.population) for n in x.nodes] for x in rf.trees]
    # reference split semantics (multi-way numeric, categorical partitions, notUsedYet), data parallel
    rr = T.RandomForest(hs, 3, T.TreeParams(stopping="maxDepth", max_depth=3, sub_sampling="withReplace",
                                            attr_selection="randomNotUsedYet", random_attr_count=3, seed=5),
                        "all", comm=comm).fit(th)
    out["forest_ref"] = [[(n.predicates, n.population) for n in x.nodes] for x in rr.trees]
    # ---- float models: tolerance ------------------------------------------------------------
    g = torch.Generator().manual_seed(4)
    X = torch.randn(2000, 3, generator=g) + torch.randint(0, 3, (2000, 1), generator=g) * 6.0
    km = KMeans(3, seed=5, comm=comm).fit(_shard(X, rank, world).to(dev))
    out["kmeans"] = float(km.best[3].sse)
    w = torch.tensor([1.0, -2.0, 0.5])
    y = ((X @ w + 2.0 * torch.randn(2000, generator=g)) > 0).double()     # non-separable: finite optimum
    lr = LogisticRegression(max_iter=10).fit(_shard(X, rank, world).to(dev), _shard(y, rank, world).to(dev))
    out["logit"] = lr.coef.tolist()
    Q = torch.randn(64, 3, generator=g)
    lo = rank * 2000 // world
    d, i = D.distributed_knn(Q.to(dev), _shard(X, rank, world).contiguous().to(dev), 5, comm, r_base=lo)
    out["knn"] = (d.tolist(), i.tolist())
    # ---- cascade SVM (same global shard partition at every world size), Relief, GBT -----------
    from avenir_amd.models.sampling import relief
    from avenir_amd.models.svm import CascadeSVM
    gs = torch.Generator().manual_seed(12)
    Xs = torch.randn(640, 2, generator=gs)
    ys = (Xs[:, 0] * Xs[:, 1] > 0).long()
    cs_ = CascadeSVM(shards=8 // world, comm=comm, gamma=0.5, C=1.0).fit(_shard(Xs, rank, world).to(dev),
                                                                       _shard(ys, rank, world).to(dev))
    probe = torch.randn(64, 2, generator=gs)
    out["cascade"] = (cs_.n_cascade_sv, cs_.decision_function(probe.to(dev)).tolist())
    Xr = torch.randn(600, 5, generator=gs)
    yr = ((Xr[:, 0] + 0.5 * Xr[:, 3]) > 0).long()
    out["relief"] = relief(_shard(Xr, rank, world).to(dev), _shard(yr, rank, world).to(dev), k=2, comm=comm).tolist()
    gbt = T.GradientBoostedTrees(hs, T.GBTParams(n_estimators=6, max_depth=3, max_bins=32), comm=comm).fit(th)
    out["gbt"] = gbt.decision_function(full).tolist()
    # ---- sequence parallel Viterbi -----------------------------------------------------------
    gh = torch.Generator().manual_seed(9)
    norm = lambda mm: torch.log(mm / mm.sum(-1, keepdim=True))
    lA = norm(torch.rand(5, 5, generator=gh, dtype=torch.float64) + 0.05)
    lB = norm(torch.rand(5, 4, generator=gh, dtype=torch.float64) + 0.05)
    lp = norm(torch.rand(5, generator=gh, dtype=torch.float64) + 0.05)
    obs = torch.randint(0, 4, (1601,), generator=gh).to(torch.int16)
    path, score = SO.viterbi_long(_shard(obs, rank, world).to(dev), lA.to(dev), lB.to(dev), lp.to(dev), chunk=64)
    out["viterbi"] = (path.tolist(), round(float(score), 6))
    comm.check()
    out["p2p_calls"] = comm.p2p_calls             # small device sums that took the peer-mapped kernel
    return out


@pytest.fixture(scope="module")
def reference():
    args = _data()
    return args, run_world(_all_models, 1, *args, timeout=300)[0]


def _compare(res, ref, world, score_rel=1e-9):
    for r, got in enumerate(res):
        for key in ("nb", "mi", "cramer", "markov", "hmm", "pst", "apriori", "tree", "forest_dp", "forest_tp",
                    "forest_ref"):
            assert got[key] == ref[key], f"rank {r}/{world}: {key} differs"
        assert got["kmeans"] == pytest.approx(ref["kmeans"], rel=1e-5)
        # device: the fp32 K13 gradient partials depend on the row sharding (fp64 across ranks)
        assert np.allclose(got["logit"], ref["logit"], rtol=max(1e-7, score_rel * 2), atol=1e-9)
        assert np.allclose(got["knn"][0], ref["knn"][0], atol=1e-5)
        assert got["knn"][1] == ref["knn"][1]
        assert got["viterbi"][1] == pytest.approx(ref["viterbi"][1], rel=score_rel)
        assert got["cascade"][0] == ref["cascade"][0]
        assert np.allclose(got["cascade"][1], ref["cascade"][1], atol=1e-5)
        assert np.allclose(got["relief"], ref["relief"], rtol=1e-6, atol=1e-7)
        assert np.allclose(got["gbt"], ref["gbt"], rtol=1e-6, atol=1e-6)
    # Viterbi is sequence-parallel: the rank segments concatenate to the single-rank path
    assert sum((g["viterbi"][0] for g in res), []) == ref["viterbi"][0]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_world_size_equivalence(reference, world):
    args, ref = reference
    res = run_world(_all_models, world, *args, timeout=600)
    _compare(res, ref, world)


@pytest.mark.parametrize("world", [2, 4])
def test_world_size_equivalence_emulated_rccl(reference, world):
    """The RCCL-only code paths (backend == "nccl": device collective buffers, all_to_all_single,
    batched P2P ring) over a gloo group on the CPU."""
    args, ref = reference
    _compare(run_world(_all_models, world, *args, timeout=600, comm="rccl-emul:cpu"), ref, world)


@pytest.mark.gpu
@pytest.mark.parametrize("comm", ["gloo:cuda", "rccl-emul:cuda"])
def test_world_size_equivalence_device_tensors(comm):
    """Every model of the set with DEVICE tensors at world 2 and 4: separate rank processes sharing
    cuda:0 (the HIP kernels under row sharding, the _prep copy path, and with rccl-emul the NB
    side-stream all-reduce overlap), against the same set at world 1 on the device."""
    args = _data()
    ref = run_world(_all_models, 1, *args, "cuda", timeout=600, comm=comm)[0]
    for world in (2, 4):
        # the device Viterbi scan accumulates in fp32 per chunk: the score depends on the chunking
        res = run_world(_all_models, world, *args, "cuda", timeout=600, comm=comm)
        _compare(res, ref, world, score_rel=1e-6)
        # the default small-sum selection took the hand-written kernel on every rank
        assert all(r["p2p_calls"] > 0 for r in res), [r["p2p_calls"] for r in res]


def _cli_ranks(rank, world, data, schema, model, out_dir, out_file):
    from avenir_amd.cli import main
    from avenir_amd.parallel import comm as C
    assert main(["bayesianPredictor", "-i", data, "-o", out_dir, "--schema", schema, "--model", model,
                 "--device", "cpu"]) == 0
    C.get_comm().barrier()
    assert main(["bayesianPredictor", "-i", data, "-o", out_file, "--schema", schema, "--model", model,
                 "--device", "cpu"]) == 0
    return rank


@pytest.mark.parametrize("world", [2, 4])
def test_cli_map_output_per_rank(tmp_path, world):
    """Map-side CLI jobs under several ranks: one part file per rank in a directory output, or the
    rank-ordered lines gathered into a single file; either way every input row appears once."""
    from avenir_amd.cli import main
    data, schema = tmp_path / "churn.csv", tmp_path / "churn.json"
    synth.write_churn(data, 1001, seed=2, schema_path=schema)
    model = tmp_path / "nb.txt"
    assert main(["bayesianDistribution", "-i", str(data), "-o", str(model), "--schema", str(schema),
                 "--device", "cpu"]) == 0
    out_dir, out_file = tmp_path / "pred", tmp_path / "pred.txt"
    run_world(_cli_ranks, world, str(data), str(schema), str(model), str(out_dir), str(out_file))
    parts = sorted(out_dir.glob("part-*"))
    assert len(parts) == world
    rows = [l for p in parts for l in p.read_text().splitlines() if l]
    src = [l for l in data.read_text().splitlines() if l]
    assert [r.rsplit(",", 2)[0] for r in rows] == src
    single = [l for l in out_file.read_text().splitlines() if l]
    assert single == rows


def _domain():
    from avenir_amd.optimize.domain import AssignmentDomain
    g = torch.Generator().manual_seed(21)
    cost = torch.rand((20, 8), generator=g) * 100
    conf = torch.rand((20, 20), generator=g) < 0.12
    return AssignmentDomain(cost, conf | conf.T, invalid_cost=1e3)


def _optimisers(rank, world, seed):
    from avenir_amd.optimize.search import GeneticAlgorithm, SimulatedAnnealing
    from avenir_amd.parallel.comm import get_comm
    comm = get_comm()
    sa = SimulatedAnnealing(_domain(), n_chains=16, iters=200, t0=5.0, cooling=0.97, seed=seed, comm=comm).run()
    ga = GeneticAlgorithm(_domain(), islands=2, pool=12, mating=6, replacement=6, generations=15, seed=seed,
                          comm=comm).run()
    sal = SimulatedAnnealing(_domain(), n_chains=16, iters=100, t0=5.0, cooling=0.97, seed=seed, comm=comm,
                             locally_optimize=True, local_iters=20).run()
    return float(sa.best_cost), float(ga.best_cost), float(sal.best_cost)


@pytest.mark.parametrize("world", [2, 4])
def test_optimiser_islands_equal_independent_runs(world):
    """SA chains / GA islands are global (their random streams are keyed by global chain / island
    index; the reference runs independent optimisers per Spark partition): the W-rank result is the
    single-process run of W times as many chains / islands."""
    got = run_world(_optimisers, world, 5)
    from avenir_amd.optimize.search import GeneticAlgorithm, SimulatedAnnealing
    sa_ref = float(SimulatedAnnealing(_domain(), n_chains=16 * world, iters=200, t0=5.0, cooling=0.97,
                                      seed=5).run().best_cost)
    ga_ref = float(GeneticAlgorithm(_domain(), islands=2 * world, pool=12, mating=6, replacement=6, generations=15,
                                    seed=5).run().best_cost)
    # local search after the walk: keyed by global chain too
    sal_ref = float(SimulatedAnnealing(_domain(), n_chains=16 * world, iters=100, t0=5.0, cooling=0.97, seed=5,
                                       locally_optimize=True, local_iters=20).run().best_cost)
    for sa_c, ga_c, sal_c in got:
        assert sa_c == pytest.approx(sa_ref, rel=1e-6)
        assert ga_c == pytest.approx(ga_ref, rel=1e-6)
        assert sal_c == pytest.approx(sal_ref, rel=1e-6)
