#!/usr/bin/env python3
"""avenir_amd on one MI355X vs the reference's own CPU implementations, same data and settings.

The reference publishes no numbers, and its Python estimators are thin wrappers
over scikit-learn / PyTorch-CPU (P/supv/rf.py, gbt.py, svm.py, lrd.py, P/unsupv/cluster.py,
P/supv/lstm.py with ``common.device=cpu``).  This script runs those same library calls on the
host CPU (``--threads`` workers) and the avenir_amd estimator on the GPU on identical synthetic
data, and prints one JSON line per model: fit seconds for both, the speedup, and held-out
accuracy for both (a sanity check that the two fit the same model class).  The Java/Hadoop
jobs of the reference cannot be run here (no JVM/Hadoop), so they have no row.

    python benchmarks/bench_vs_reference.py --only rf,gbt,kmeans,logit,svm,knn,nb,lstm
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import avenir_amd  # noqa: E402


def emit(**kw):
    print(json.dumps(kw), flush=True)


def gpu_time(fn, reps=1):
    fn()                                  # warm-up (kernel caches, allocator)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps, out


def cpu_time(fn):
    t0 = time.perf_counter()
    out = fn()
    return time.perf_counter() - t0, out


def linear_data(n, d, seed, w):
    g = torch.Generator(device="cuda").manual_seed(seed)
    X = torch.randn((n, d), device="cuda", generator=g)
    y = ((X @ w) + 0.5 * torch.randn(n, device="cuda", generator=g) > 0).long()
    return X, y


def as_table(X, y):
    """Row-major device arrays -> avenir_amd Table (feature-major SoA, padded)."""
    from avenir_amd.data.table import Table, pad16
    from avenir_amd.models.supervised import array_schema
    n, d = X.shape
    Xs = torch.zeros((d, pad16(n)), device=X.device)
    Xs[:, :n] = X.t()
    lab = torch.full((pad16(n),), 255, dtype=torch.uint8, device=X.device)
    lab[:n] = y.to(torch.uint8)
    schema = array_schema(d, [0, 1])
    return Table(schema, n, torch.zeros((0, pad16(n)), dtype=torch.uint8, device=X.device), [], Xs,
                 schema.feature_fields, lab, schema.find_class_attr_field())


def acc(pred, y):
    return float((torch.as_tensor(pred).to(y.device).long() == y.long()).float().mean())


def tree_data(a, d=16):
    g = torch.Generator(device="cuda").manual_seed(7)
    w = torch.randn(d, device="cuda", generator=g)
    Xtr, ytr = linear_data(a.tree_rows, d, 1, w)
    # a non-linear target so depth matters: XOR of two half-spaces
    ytr = ((Xtr[:, 0] * Xtr[:, 1] > 0) ^ (Xtr @ w > 0)).long()
    Xte, _ = linear_data(a.tree_rows // 4, d, 2, w)
    yte = ((Xte[:, 0] * Xte[:, 1] > 0) ^ (Xte @ w > 0)).long()
    return Xtr, ytr, Xte, yte


def bench_rf(a):
    from sklearn.ensemble import RandomForestClassifier
    from avenir_amd.models.tree import RandomForest, TreeParams
    Xtr, ytr, Xte, yte = tree_data(a)
    trees, depth = 10, 8
    p = TreeParams(binary=True, stopping="maxDepth", max_depth=depth, sub_sampling="withReplace",
                   attr_selection="randomAll", max_bins=32)
    ttr, tte = as_table(Xtr, ytr), as_table(Xte, yte)
    g_s, rf = gpu_time(lambda: RandomForest(ttr.schema, trees, p, "sqrt").fit(ttr))
    g_acc = acc(rf.predict(tte), yte)
    xn, yn = Xtr.cpu().numpy(), ytr.cpu().numpy()
    c_s, sk = cpu_time(lambda: RandomForestClassifier(trees, max_depth=depth, max_features="sqrt",
                                                      n_jobs=a.threads, random_state=0).fit(xn, yn))
    c_acc = float((sk.predict(Xte.cpu().numpy()) == yte.cpu().numpy()).mean())
    emit(model="random_forest", reference="sklearn RandomForestClassifier (P/supv/rf.py)", rows=len(yn),
         features=Xtr.shape[1], trees=trees, depth=depth, ref_cpu_s=c_s, avenir_gpu_s=g_s, speedup=c_s / g_s,
         ref_acc=c_acc, avenir_acc=g_acc)


def bench_gbt(a):
    from sklearn.ensemble import GradientBoostingClassifier
    from avenir_amd.models.tree import GBTParams, GradientBoostedTrees
    Xtr, ytr, Xte, yte = tree_data(a)
    n = min(a.gbt_rows, Xtr.shape[0])
    Xtr, ytr = Xtr[:n], ytr[:n]
    # reference defaults, R/gb.properties:12-13,17: 120 estimators, depth 3, learning rate 0.12
    p = GBTParams(n_estimators=120, learning_rate=0.12, max_depth=3, max_bins=64)
    ttr, tte = as_table(Xtr, ytr), as_table(Xte, yte)
    g_s, gb = gpu_time(lambda: GradientBoostedTrees(ttr.schema, p).fit(ttr))
    g_acc = acc(gb.predict(tte), yte)
    xn, yn = Xtr.cpu().numpy(), ytr.cpu().numpy()
    c_s, sk = cpu_time(lambda: GradientBoostingClassifier(n_estimators=120, learning_rate=0.12, max_depth=3,
                                                          random_state=0).fit(xn, yn))
    c_acc = float((sk.predict(Xte.cpu().numpy()) == yte.cpu().numpy()).mean())
    emit(model="gbt", reference="sklearn GradientBoostingClassifier (P/supv/gbt.py, R/gb.properties)", rows=n,
         features=Xtr.shape[1], estimators=120, depth=3, ref_cpu_s=c_s, avenir_gpu_s=g_s, speedup=c_s / g_s,
         ref_acc=c_acc, avenir_acc=g_acc)


def bench_kmeans(a):
    """R/cluster.properties: 10 k-means++ inits, up to 300 iterations (our 10 runs share one fused
    launch per iteration; scikit-learn runs them one after another)."""
    from sklearn.cluster import KMeans as SKKMeans
    from avenir_amd.models.cluster import KMeans
    n, d, k, inits, it = a.rows, 16, 16, 10, 300
    g = torch.Generator(device="cuda").manual_seed(3)
    centers = torch.randn((k, d), device="cuda", generator=g) * 4
    X = centers[torch.randint(0, k, (n,), device="cuda", generator=g)] + torch.randn((n, d), device="cuda",
                                                                                      generator=g)
    g_s, km = gpu_time(lambda: KMeans(k, n_init=inits, max_iter=it, tol=1e-4, tol_mode="sklearn").fit(X))
    run = km.best[k]
    xn = X.cpu().numpy()
    c_s, sk = cpu_time(lambda: SKKMeans(k, n_init=inits, max_iter=it, tol=1e-4, random_state=0).fit(xn))
    emit(model="kmeans", reference="sklearn KMeans (P/unsupv/cluster.py, R/cluster.properties)", rows=n, dim=d, k=k,
         n_init=inits, max_iter=it, ref_cpu_s=c_s, avenir_gpu_s=g_s, speedup=c_s / g_s, ref_sse=float(sk.inertia_),
         avenir_sse=float(run.sse), ref_iters=int(sk.n_iter_), avenir_iters=int(run.iterations))


def bench_logit(a):
    from sklearn.linear_model import LogisticRegression as SKLR
    from avenir_amd.models.linear import LogisticRegression
    n, d = a.rows, 15
    g = torch.Generator(device="cuda").manual_seed(5)
    w = torch.randn(d, device="cuda", generator=g)
    Xtr, ytr = linear_data(n, d, 11, w)
    Xte, yte = linear_data(n // 4, d, 12, w)
    g_s, m = gpu_time(lambda: LogisticRegression(max_iter=25, tol=1e-8).fit(Xtr, ytr.float()))
    g_acc = acc(m.predict(Xte), yte)
    xn, yn = Xtr.cpu().numpy(), ytr.cpu().numpy()
    c_s, sk = cpu_time(lambda: SKLR(C=1e6, max_iter=200).fit(xn, yn))
    c_acc = float((sk.predict(Xte.cpu().numpy()) == yte.cpu().numpy()).mean())
    emit(model="logistic_regression", reference="sklearn LogisticRegression lbfgs (P/supv/lrd.py)", rows=n,
         features=d, ref_cpu_s=c_s, avenir_gpu_s=g_s, speedup=c_s / g_s, ref_acc=c_acc, avenir_acc=g_acc)


def bench_svm(a):
    from sklearn.svm import SVC as SKSVC
    from avenir_amd.models.svm import SVC
    n = a.svm_rows
    g = torch.Generator(device="cuda").manual_seed(9)
    X = torch.randn((n, 8), device="cuda", generator=g)
    y = (X[:, 0] * X[:, 1] > 0).long()
    Xte = torch.randn((n // 4, 8), device="cuda", generator=g)
    yte = (Xte[:, 0] * Xte[:, 1] > 0).long()
    g_s, m = gpu_time(lambda: SVC("rbf", C=1.0, gamma=0.5).fit(X, y))
    g_acc = acc(m.predict(Xte), yte)
    xn, yn = X.cpu().numpy(), y.cpu().numpy()
    c_s, sk = cpu_time(lambda: SKSVC(C=1.0, kernel="rbf", gamma=0.5, cache_size=2000).fit(xn, yn))
    c_acc = float((sk.predict(Xte.cpu().numpy()) == yte.cpu().numpy()).mean())
    emit(model="svm_rbf", reference="sklearn SVC / libsvm (P/supv/svm.py)", rows=n, features=8, ref_cpu_s=c_s,
         avenir_gpu_s=g_s, speedup=c_s / g_s, ref_acc=c_acc, avenir_acc=g_acc,
         ref_support_vectors=int(sk.n_support_.sum()), avenir_support_vectors=len(m.support_))


def bench_knn(a):
    from sklearn.neighbors import KNeighborsClassifier
    from avenir_amd.models.knn import NearestNeighbor
    n, q, d, k = a.knn_rows, a.knn_rows // 16, 16, 5          # top-k = 5, R/knn.properties:35
    g = torch.Generator(device="cuda").manual_seed(13)
    w = torch.randn(d, device="cuda", generator=g)
    X, y = linear_data(n, d, 14, w)
    Q, yq = linear_data(q, d, 15, w)
    nn = NearestNeighbor(k=k).fit(X, y, 2)
    g_s, r = gpu_time(lambda: nn.predict(Q))
    g_acc = acc(r.pred, yq)
    xn, yn, qn = X.cpu().numpy(), y.cpu().numpy(), Q.cpu().numpy()
    sk = KNeighborsClassifier(k, algorithm="brute", n_jobs=a.threads).fit(xn, yn)
    c_s, pred = cpu_time(lambda: sk.predict(qn))
    c_acc = float((pred == yq.cpu().numpy()).mean())
    emit(model="knn_classify", reference="sklearn KNeighborsClassifier brute (J/knn/NearestNeighbor semantics)",
         train_rows=n, queries=q, dim=d, k=k, ref_cpu_s=c_s, avenir_gpu_s=g_s, speedup=c_s / g_s, ref_acc=c_acc,
         avenir_acc=g_acc)


def bench_nb(a):
    from sklearn.naive_bayes import CategoricalNB
    from avenir_amd.data.synth import CHURN_SCHEMA, churn_device
    from avenir_amd.data.table import Table
    from avenir_amd.models.bayes import NaiveBayes
    from avenir_amd.utils.schema import FeatureSchema
    n = a.nb_rows
    schema = FeatureSchema.from_json(CHURN_SCHEMA)
    codes, labels = churn_device(n, seed=21, device=torch.device("cuda"))
    t = Table(schema, n, codes, schema.feature_fields, torch.zeros((0, codes.shape[1]), device="cuda"), [],
              labels, schema.find_class_attr_field())
    g_s, nb = gpu_time(lambda: NaiveBayes(schema).fit(t), 3)
    pr = nb.predict(t)
    g_acc = acc(pr.pred, labels[:n])
    xn = codes[:, :n].t().contiguous().cpu().numpy()
    yn = labels[:n].cpu().numpy()
    c_s, sk = cpu_time(lambda: CategoricalNB(alpha=1.0).fit(xn, yn))
    c_acc = float((sk.predict(xn) == yn).mean())
    emit(model="naive_bayes", reference="sklearn CategoricalNB (BayesianDistribution semantics, R/churn.json)",
         rows=n, features=int(codes.shape[0]), ref_cpu_s=c_s, avenir_gpu_s=g_s, speedup=c_s / g_s,
         ref_train_acc=c_acc, avenir_train_acc=g_acc)


def bench_lstm(a):
    """P/supv/lstm.py on ``common.device=cpu`` (R/lstm_ct.properties: input 5, hidden 100, 2 layers,
    seq_len 5, 1000 sequences) vs the fused-kernel LSTM with a graph-captured step."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from bench_lstm import CONFIGS, run
    cfg = dict(CONFIGS[0])
    gpu = run(cfg, "fused_graph", 20, 3)
    B, T, I, H, L, O = (cfg[k] for k in "BTIHLO")
    torch.manual_seed(0)

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lstm = torch.nn.LSTM(I, H, L, batch_first=True)
            self.head = torch.nn.Linear(H, O)

        def forward(self, x):
            return self.head(self.lstm(x)[0][:, -1])

    net = Net()
    opt = torch.optim.Adam(net.parameters(), lr=2e-3)
    x = torch.randn(B, T, I)
    y = torch.randint(0, O, (B,))
    lossf = torch.nn.CrossEntropyLoss()

    def step():
        opt.zero_grad()
        lossf(net(x), y).backward()
        opt.step()

    step()
    steps = 10
    c_s, _ = cpu_time(lambda: [step() for _ in range(steps)])
    c_ms = c_s / steps * 1e3
    emit(model="lstm_train_step", reference="torch.nn.LSTM on CPU (P/supv/lstm.py, common.device=cpu)",
         config=cfg["name"], batch=B, seq_len=T, hidden=H, layers=L, ref_cpu_ms=c_ms, avenir_gpu_ms=gpu["train_ms"],
         speedup=c_ms / gpu["train_ms"])


BENCHES = {"nb": bench_nb, "rf": bench_rf, "gbt": bench_gbt, "kmeans": bench_kmeans, "logit": bench_logit,
           "svm": bench_svm, "knn": bench_knn, "lstm": bench_lstm}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--rows", type=int, default=1 << 20)
    ap.add_argument("--tree-rows", type=int, default=1 << 20)
    ap.add_argument("--gbt-rows", type=int, default=1 << 16)
    ap.add_argument("--svm-rows", type=int, default=8192)
    ap.add_argument("--knn-rows", type=int, default=1 << 18)
    ap.add_argument("--nb-rows", type=int, default=1 << 23)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    os.environ.setdefault("OMP_NUM_THREADS", str(a.threads))
    for name, fn in BENCHES.items():
        if a.only and name not in a.only.split(","):
            continue
        # objects alive now (torch, sklearn modules imported by earlier benches, their results)
        # go to the GC's permanent generation: a generation-2 pass over them inside a timed fit
        # cost 150 ms (GBT: 0.03 -> 0.13 s) — harness hygiene, the same for both columns
        avenir_amd.freeze_startup_objects()
        try:
            fn(a)
        except Exception as e:  # noqa: BLE001
            emit(model=name, error=f"{type(e).__name__}: {e}")


if __name__ == "__main__":
    main()
