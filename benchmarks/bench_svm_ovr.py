#!/usr/bin/env python3
"""Batched one-vs-rest SVM on one MI355X (the batched solve must fill the chip):
``--classes`` one-vs-rest problems of N x d RBF solved as ONE batch (smo_batch over the stacked
label vectors), dense and implicit kernel paths.  One JSON line per (N, classes, path); run under
``rocprofv3 --pmc SQ_WAVES ...`` for the per-launch wave counts.

    python benchmarks/bench_svm_ovr.py [--n 8192] [--d 16] [--classes 16] [--paths dense,implicit]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from avenir_amd.models import svm as S  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--d", type=int, default=16)
    ap.add_argument("--classes", type=int, default=16)
    ap.add_argument("--paths", default="dense,implicit")
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(3)
    X = torch.randn((args.n, args.d), device="cuda", generator=g)
    W = torch.randn((args.d, args.classes), device="cuda", generator=g)
    y = (X @ W + 0.3 * torch.randn((args.n, args.classes), device="cuda", generator=g)).argmax(1)
    for path in args.paths.split(","):
        S.DENSE_MAX_N = 0 if path == "implicit" else 1 << 30
        S.SVC(kernel="rbf", C=1.0, gamma=0.1).fit(X[:512], y[:512])      # warm-up
        best = None
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m = S.SVC(kernel="rbf", C=1.0, gamma=0.1).fit(X, y)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        acc = float((m.predict(X) == y).float().mean())
        print(json.dumps({"bench": "svm_ovr", "N": args.n, "d": args.d, "classes": args.classes, "path": path,
                          "seconds": round(best, 5), "solver": S.LAST_SOLVE.get("solver"),
                          "outer_steps": S.LAST_SOLVE.get("outer"), "support_vectors": int(m.support_.numel()),
                          "train_acc": acc}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
