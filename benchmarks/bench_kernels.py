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


BENCHES = {"hist": bench_hist, "nbpred": bench_nb_predict}


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
