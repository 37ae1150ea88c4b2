#!/usr/bin/env python3
"""Kernel micro-benchmarks (hipEvent timing, interleaved rounds in one process).

Prints one JSON line per kernel variant with achieved bandwidth / throughput, e.g.

    python benchmarks/bench_kernels.py --only hist
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = []
    for _ in range(iters):
        s.record()
        fn()
        e.record()
        e.synchronize()
        times.append(s.elapsed_time(e))
    times.sort()
    return times[len(times) // 2], times[0]


def emit(**kw):
    print(json.dumps(kw), flush=True)


def bench_hist(args):
    from avenir_amd.data.synth import churn_device
    from avenir_amd.ops import histogram as H
    n = args.rows
    codes, labels = churn_device(n, seed=1, device="cuda")
    bins = [4, 3, 3, 3, 5]
    nbytes = n * 6
    for name, mode in (("split(auto)", 0), ("packed-idx", 3), ("lds", 1)):
        out = torch.zeros((2, sum(bins) + 1), dtype=torch.int64, device="cuda")

        def f():
            out.zero_()
            H.class_histogram(codes, n, bins, labels, 2, out=out, mode=mode, count_labels=True)
        med, best = timeit(f)
        emit(kernel="class_histogram", variant=name, rows=n, ms=med, best_ms=best,
             gbps=nbytes / (med / 1e3) / 1e9, rows_per_s=n / (med / 1e3))
    # larger-cardinality features -> LDS path
    g = torch.Generator(device="cuda").manual_seed(0)
    big = torch.randint(0, 40, (8, codes.shape[1]), generator=g, device="cuda", dtype=torch.int32).to(torch.uint8)
    out = torch.zeros((2, 8 * 40 + 1), dtype=torch.int64, device="cuda")

    def f2():
        out.zero_()
        H.class_histogram(big, n, [40] * 8, labels, 2, out=out, count_labels=True)
    med, best = timeit(f2, iters=5)
    emit(kernel="class_histogram", variant="lds 8x40 bins", rows=n, ms=med,
         gbps=n * 9 / (med / 1e3) / 1e9)


def bench_nb_predict(args):
    from avenir_amd.data.synth import CHURN_SCHEMA, churn_device
    from avenir_amd.data.table import Table
    from avenir_amd.models.bayes import NaiveBayes
    from avenir_amd.utils.schema import FeatureSchema
    n = min(args.rows, 1 << 27)
    schema = FeatureSchema.from_json(CHURN_SCHEMA)
    codes, labels = churn_device(n, seed=2, device="cuda")
    t = Table(schema, n, codes, schema.feature_fields, torch.zeros((0, 16), device="cuda"), [],
              labels, schema.find_class_attr_field())
    nb = NaiveBayes(schema).fit(t)
    for prob in (False, True):
        med, _ = timeit(lambda: nb.predict(t, with_prob=prob), iters=10)
        emit(kernel="nb_predict", with_prob=prob, rows=n, ms=med, rows_per_s=n / (med / 1e3))


def bench_glm(args):
    """K13 fused GLM gradient vs the unfused torch path (GEMV, sigmoid, GEMV)."""
    from avenir_amd.models.linear import DenseSoA, MODE_LOGISTIC, glm_gradient
    n = min(args.rows, 1 << 27)
    for d in (7, 15):
        X = torch.randn((d, n), device="cuda")
        data = DenseSoA.__new__(DenseSoA)
        data.n, data.d_in, data.intercept, data.D = n, d, True, d + 1
        data.Dp = 8 if d == 7 else 16
        data.ld = n
        data.X = torch.zeros((data.Dp, n), device="cuda")
        data.X[0] = 1
        data.X[1:d + 1] = X
        del X
        y = (torch.rand(n, device="cuda") < 0.5).float()
        w = torch.randn(d + 1, device="cuda") * 0.1
        med, best = timeit(lambda: glm_gradient(data, y, w, MODE_LOGISTIC), iters=10)
        nbytes = n * (data.Dp + 1) * 4
        emit(kernel="glm_grad", variant=f"fused D={data.Dp}", rows=n, ms=med, best_ms=best,
             gbps=nbytes / (med / 1e3) / 1e9, rows_per_s=n / (med / 1e3))
        Xr = data.X[: d + 1]

        def unfused():
            p = torch.sigmoid(w @ Xr)
            return Xr @ (y - p)
        med2, _ = timeit(unfused, iters=10)
        emit(kernel="glm_grad", variant=f"torch GEMV+sigmoid+GEMV D={d + 1}", rows=n, ms=med2,
             gbps=n * (d + 2) * 4 / (med2 / 1e3) / 1e9, speedup_fused=med2 / med)
        del data, y


def bench_smo(args):
    from avenir_amd.models.svm import kernel_matrix, smo_batch
    g = torch.Generator(device="cuda").manual_seed(0)
    for N, B in ((4096, 1), (4096, 16)):
        X = torch.randn((N, 8), device="cuda", generator=g)
        y = torch.where((X[:, 0] * X[:, 1] + 0.3 * X[:, 2]) > 0, 1.0, -1.0)
        K = kernel_matrix(X, X, "rbf", 0.25)
        Kb = K.unsqueeze(0).expand(B, -1, -1).contiguous()
        yb = y.unsqueeze(0).expand(B, -1).contiguous()
        torch.cuda.synchronize()
        out = {}

        def run():
            out["r"] = smo_batch(Kb, yb, 1.0, 1e-3)
        med, _ = timeit(run, iters=3, warmup=1)
        its = int(out["r"][2][0])
        emit(kernel="smo", N=N, problems=B, ms=med, iterations=its, us_per_iter=med * 1e3 / max(its, 1))


def bench_sa(args):
    from avenir_amd.optimize import AssignmentDomain, sa_assign
    g = torch.Generator().manual_seed(0)
    L, V, P, iters = 64, 16, 1 << 16, 1000
    cost = torch.rand((L, V), generator=g) * 100
    conf = torch.rand((L, L), generator=g) < 0.05
    d = AssignmentDomain(cost, conf | conf.T).to("cuda")
    sol, _ = d.random(P)
    c = d.cost(sol)
    med, _ = timeit(lambda: sa_assign(d, sol, c, iters, 5.0, 0.99, 4, True, 3, 1, 0), iters=3, warmup=1)
    emit(kernel="sa_assign", chains=P, L=L, V=V, iters=iters, ms=med, moves_per_s=P * iters / (med / 1e3))


def bench_knn(args):
    from avenir_amd.ops import distance as Dm
    g = torch.Generator(device="cuda").manual_seed(0)
    for M, R, D in ((65536, 65536, 16), (16384, 1 << 20, 32), (16384, 1 << 18, 64), (16384, 1 << 18, 256)):
        Q = torch.randn((M, D), device="cuda", generator=g)
        Rt = torch.randn((R, D), device="cuda", generator=g)
        med, _ = timeit(lambda: Dm.knn(Q, Rt, 10), iters=5, warmup=1)
        emit(kernel="knn_topk", M=M, R=R, D=D, k=10, ms=med, tflops=2.0 * M * R * D / (med / 1e3) / 1e12,
             pairs_per_s=M * R / (med / 1e3))


def bench_sampler(args):
    from avenir_amd.ops import samplers as S
    n = 1 << 28
    for dist, params, name in ((S.NORMAL, [0, 1], "normal"), (S.GAMMA, [2.0, 1.0], "gamma"),
                               (S.POISSON, [4.0], "poisson")):
        med, _ = timeit(lambda: S.device_sample(dist, n, params, "cuda", seed=1), iters=5)
        emit(kernel="sample", dist=name, n=n, ms=med, samples_per_s=n / (med / 1e3), gbps=n * 4 / (med / 1e3) / 1e9)


def bench_mlp(args):
    """K27 fused Linear+bias+act vs torch (addmm + activation), forward and forward+backward."""
    from avenir_amd.ops.mlp_ops import linear_act
    g = torch.Generator(device="cuda").manual_seed(0)
    for M, K, N in ((65536, 64, 64), (65536, 256, 256), (8192, 32, 16)):
        x = torch.randn((M, K), device="cuda", generator=g, requires_grad=True)
        W = torch.randn((N, K), device="cuda", generator=g, requires_grad=True)
        b = torch.randn((N,), device="cuda", generator=g, requires_grad=True)
        gy = torch.randn((M, N), device="cuda", generator=g)
        for name, fn in (("fused", lambda: linear_act(x, W, b, "relu")),
                         ("torch", lambda: torch.relu(torch.nn.functional.linear(x, W, b)))):
            with torch.no_grad():
                fwd, _ = timeit(fn, iters=20)
            fb, _ = timeit(lambda: fn().backward(gy), iters=20)
            emit(kernel="linear_relu", variant=name, M=M, K=K, N=N, fwd_ms=fwd, fwd_bwd_ms=fb,
                 fwd_tflops=2.0 * M * K * N / (fwd / 1e3) / 1e12)


BENCHES = {"hist": bench_hist, "nbpred": bench_nb_predict, "glm": bench_glm, "smo": bench_smo, "sa": bench_sa,
           "knn": bench_knn, "sample": bench_sampler, "mlp": bench_mlp}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    ap.add_argument("--rows", type=int, default=1 << 30)
    args = ap.parse_args()
    for name, fn in BENCHES.items():
        if args.only and name not in args.only.split(","):
            continue
        fn(args)


if __name__ == "__main__":
    main()
