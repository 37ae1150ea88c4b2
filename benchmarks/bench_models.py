#!/usr/bin/env python3
"""End-to-end model training / inference throughput on one GPU (JSON line per model).

    python benchmarks/bench_models.py --only rf,gbt,kmeans,logit,svm,knn,sa,mlp
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def emit(**kw):
    print(json.dumps(kw), flush=True)


def timed(fn, reps=1):
    fn()                                  # warm-up (compiles / caches)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps, out


def _numeric_table(n, d, seed=0, classes=2):
    from avenir_amd.data.table import Table, pad16
    from avenir_amd.models.supervised import array_schema
    g = torch.Generator(device="cuda").manual_seed(seed)
    X = torch.randn((d, pad16(n)), device="cuda", generator=g)
    w = torch.randn(d, device="cuda", generator=g)
    y = ((w @ X[:, :n]) + 0.5 * torch.randn(n, device="cuda", generator=g) > 0).to(torch.uint8)
    lab = torch.full((pad16(n),), 255, dtype=torch.uint8, device="cuda")
    lab[:n] = y
    schema = array_schema(d, [0, 1])
    t = Table(schema, n, torch.zeros((0, pad16(n)), dtype=torch.uint8, device="cuda"), [], X,
              schema.feature_fields, lab, schema.find_class_attr_field())
    return t


def bench_rf(a):
    from avenir_amd.models.tree import RandomForest, TreeParams
    n, d = a.rows, 16
    t = _numeric_table(n, d)
    for trees, depth in ((10, 8),):
        p = TreeParams(binary=True, stopping="maxDepth", max_depth=depth, sub_sampling="withReplace",
                       attr_selection="randomAll", max_bins=32)
        sec, rf = timed(lambda: RandomForest(t.schema, trees, p, "sqrt").fit(t), reps=3)
        emit(model="random_forest", rows=n, features=d, trees=trees, depth=depth, seconds=sec,
             rows_x_trees_per_s=n * trees / sec, build=getattr(rf, "build_stats", None))
        ps, _ = timed(lambda: rf.predict_proba(t), 3)
        emit(model="random_forest_predict", rows=n, trees=trees, seconds=ps, rows_per_s=n / ps)


def bench_gbt(a):
    from avenir_amd.models.tree import GBTParams, GradientBoostedTrees
    n, d = a.rows, 16
    t = _numeric_table(n, d, 1)
    for rounds, depth in ((120, 3), (50, 4)):
        p = GBTParams(n_estimators=rounds, learning_rate=0.1, max_depth=depth, max_bins=64)
        sec, m = timed(lambda: GradientBoostedTrees(t.schema, p).fit(t))
        acc = float((m.predict(t) == t.labels[:n].long()).float().mean())
        emit(model="gbt", rows=n, features=d, rounds=rounds, depth=depth, seconds=sec, ms_per_round=1e3 * sec / rounds,
             rows_x_rounds_per_s=n * rounds / sec, graph=m.graph_used, train_acc=acc,
             loss_first_last=[m.train_loss[0], m.train_loss[-1]])


def bench_rf_ref(a):
    """Random forest with the reference's split semantics (explicit multi-point numeric splits up to
    maxSplit, randomNotUsedYet attributes, randomAmongTop): all trees in one batched level-wise build."""
    from avenir_amd.models.tree import RandomForest, TreeParams
    n, d = a.rows, 16
    t = _numeric_table(n, d, 2)
    for f in t.schema.feature_fields:
        f.max_split = 3
    p = TreeParams(binary=False, stopping="maxDepth", max_depth=5, sub_sampling="withReplace",
                   attr_selection="randomNotUsedYet", random_attr_count=4, split_selection="randomAmongTop",
                   top_split_count=3, max_bins=8)
    sec, rf = timed(lambda: RandomForest(t.schema, 10, p, "all").fit(t), reps=3)
    acc = float((rf.predict(t) == t.labels[:n].long()).float().mean())
    emit(model="random_forest_reference_splits", rows=n, features=d, trees=10, depth=5, max_split=3, seconds=sec,
         rows_x_trees_per_s=n * 10 / sec, train_acc=acc, build=getattr(rf, "build_stats", None))


def bench_apriori(a):
    """Apriori with device candidate generation / pruning / support (models/association.py): the
    tutorial case (resource/freq_items_apriori_tutorial.txt: 50,000 items, 3 seeded triplets,
    2,000 transactions, support 0.1) and 10^6 transactions x 10^4 items (Zipf items)."""
    import tempfile
    from avenir_amd.data import fixtures, synth_text
    from avenir_amd.data.records import read_records
    from avenir_amd.models.association import Apriori, association_rules
    d = tempfile.mkdtemp()
    cases = []
    p1 = f"{d}/tut.txt"
    with open(p1, "w") as fh:
        fh.write("\n".join(fixtures.freq_items(50000, 3, 2000, seed=1)) + "\n")
    cases.append(("tutorial_50k_items_2k_tx", p1, 2, 0.1, 4))
    p2 = f"{d}/big.txt"
    synth_text.transactions(p2, 1_000_000, n_items=10_000, per_tx=12, seed=2)
    cases.append(("1M_tx_10k_items", p2, 1, 0.002, 4))
    for name, path, skip, sup, ml in cases:
        rec = read_records(path, device="cuda", modes="x" * skip)
        torch.cuda.synchronize()
        sec, fi = timed(lambda: Apriori(sup, ml).fit_records(rec, skip))
        rs, rules = timed(lambda: association_rules(fi, 0.5))
        emit(model="apriori", case=name, transactions=rec.n_lines, items=len(rec.vocab), support=sup,
             seconds=sec, levels={k: int(v.shape[0]) for k, v in fi.sets.items()}, rules=len(rules), rules_seconds=rs)


def bench_kmeans(a):
    from avenir_amd.models.cluster import KMeans
    n, d, k = a.rows, 16, 16
    X = torch.randn((n, d), device="cuda")
    sec, km = timed(lambda: KMeans(k, n_init=1, max_iter=20, tol=0).fit(X))
    it = km.best[k].iterations
    emit(model="kmeans", rows=n, dim=d, k=k, iterations=it, seconds=sec, rows_x_iters_per_s=n * it / sec)


def bench_logit(a):
    from avenir_amd.models.linear import LogisticRegression
    n, d = a.rows * 4, 15
    X = torch.randn((n, d), device="cuda")
    y = (X[:, 0] - X[:, 1] > 0).float()
    sec, m = timed(lambda: LogisticRegression(max_iter=10, criteria="iterLimit", tol=0).fit(X, y))
    emit(model="logistic_regression_newton", rows=n, features=d, iterations=10, seconds=sec,
         rows_x_iters_per_s=n * 10 / sec)


def bench_svm(a):
    from avenir_amd.models.svm import SVC
    n = 16384
    X = torch.randn((n, 8), device="cuda")
    y = (X[:, 0] * X[:, 1] > 0).long()
    sec, m = timed(lambda: SVC("rbf", C=1.0, gamma=0.5).fit(X, y))
    emit(model="svm_rbf_smo", rows=n, seconds=sec, iterations=m.iters, support_vectors=len(m.support_))


def bench_knn(a):
    from avenir_amd.models.knn import NearestNeighbor
    n, d = 1 << 20, 16
    X = torch.randn((n, d), device="cuda")
    y = (X[:, 0] > 0).long()
    Q = torch.randn((1 << 16, d), device="cuda")
    nn = NearestNeighbor(k=10).fit(X, y, 2)
    sec, _ = timed(lambda: nn.predict(Q))
    emit(model="knn_classify", train_rows=n, queries=Q.shape[0], dim=d, k=10, seconds=sec,
         pairs_per_s=n * Q.shape[0] / sec)


def bench_sa(a):
    from avenir_amd.optimize import AssignmentDomain, SimulatedAnnealing
    g = torch.Generator().manual_seed(0)
    d = AssignmentDomain(torch.rand((64, 16), generator=g) * 100,
                         (torch.rand((64, 64), generator=g) < 0.05)).to("cuda")
    sec, r = timed(lambda: SimulatedAnnealing(d, n_chains=1 << 16, iters=1000, t0=5.0).run())
    emit(model="simulated_annealing_chains", chains=1 << 16, iters=1000, seconds=sec,
         moves_per_s=(1 << 16) * 1000 / sec, best_cost=r.best_cost)


def bench_mlp(a):
    from avenir_amd.nn import FeedForwardNetwork
    n = 1 << 18
    X = torch.randn((n, 16), device="cuda")
    y = (X[:, 0] * X[:, 1] > 0).long()
    for graph in (False, True):
        m = FeedForwardNetwork("64:relu:false:false:0,64:relu:false:false:0,2:none:false:false:0", 16, loss="ce",
                               optimizer="adam", lr=1e-3, batch_size=1024, num_iter=1, device="cuda", graph=graph)
        sec, _ = timed(lambda: m.fit(X, y, num_iter=2))
        emit(model="mlp_train", graph=graph, rows=n, batch=1024, epochs=2, seconds=sec,
             steps_per_s=2 * (n // 1024) / sec)


BENCHES = {"rf": bench_rf, "rf_ref": bench_rf_ref, "gbt": bench_gbt, "apriori": bench_apriori, "kmeans": bench_kmeans, "logit": bench_logit, "svm": bench_svm,
           "knn": bench_knn, "sa": bench_sa, "mlp": bench_mlp}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    ap.add_argument("--rows", type=int, default=1 << 24)
    a = ap.parse_args()
    import avenir_amd
    for name, fn in BENCHES.items():
        if a.only and name not in a.only.split(","):
            continue
        avenir_amd.freeze_startup_objects()   # earlier benches' objects out of the timed GC passes
        try:
            fn(a)
        except Exception as e:  # noqa: BLE001
            emit(model=name, error=f"{type(e).__name__}: {e}")


if __name__ == "__main__":
    main()
