#!/usr/bin/env python3
"""SVM fit at production sizes on one MI355X: the dense-K working-set path
against the implicit-kernel path (no N x N matrix), RBF, d features, XOR-like labels.  One JSON
line per (N, d, path): fit seconds (kernel build + solve, end to end), outer steps, support
vectors, peak device memory above the inputs, and — with ``--sklearn`` — sklearn's fit time on the
box CPU for the same problem (N <= 32768).

    python benchmarks/bench_svm_implicit.py [--sizes 8192,32768,262144] [--d 8] [--paths dense,implicit]
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


def problem(N, d, seed=9):
    """XOR labels.  d <= 16: on two of d standard-normal features (the earlier profiles' problem);
    wider: the rows lie near an 8-dimensional subspace (X = Z A + 0.1 noise) and the label is the
    XOR of two latent coordinates, so an RBF kernel on all d features can learn it."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    if d <= 16:
        X = torch.randn((N, d), device="cuda", generator=g)
        return X, (X[:, 0] * X[:, 1] > 0).long()
    ga = torch.Generator(device="cuda").manual_seed(1234)       # one subspace for train and test
    A = torch.randn((8, d), device="cuda", generator=ga) / 8 ** 0.5
    Z = torch.randn((N, 8), device="cuda", generator=g)
    X = Z @ A + 0.1 * torch.randn((N, d), device="cuda", generator=g)
    return X, (Z[:, 0] * Z[:, 1] > 0).long()


def fit(X, y, path, gamma):
    S.DENSE_MAX_N = 0 if path == "implicit" else 1 << 30
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()
    t0 = time.perf_counter()
    m = S.SVC(kernel="rbf", C=1.0, gamma=gamma, eps=1e-3).fit(X, y)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return m, dt, torch.cuda.max_memory_allocated() - base


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="8192,32768")
    ap.add_argument("--d", type=int, default=8)
    ap.add_argument("--paths", default="dense,implicit")
    ap.add_argument("--sklearn", action="store_true")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--cache", default=None, help="kernel-row cache: auto | 0 | slots (models/svm.py ROW_CACHE)")
    ap.add_argument("--sklearn-sub", type=int, default=0,
                    help="also fit sklearn on a random subsample of this many rows and compare held-out accuracy")
    ap.add_argument("--gamma", type=float, default=0.5)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    if args.cache is not None:
        S.ROW_CACHE = args.cache
    gamma = args.gamma
    Xw, yw = problem(512, args.d)
    for path in args.paths.split(","):
        fit(Xw, yw, path, gamma)                     # warm-up: kernels, graphs, allocator
    for N in [int(v) for v in args.sizes.split(",")]:
        X, y = problem(N, args.d)
        sk = None
        if args.sklearn and N <= 32768:
            from sklearn.svm import SVC as SKSVC
            Xh, yh = X.cpu().numpy(), y.cpu().numpy()
            t0 = time.perf_counter()
            skm = SKSVC(C=1.0, kernel="rbf", gamma=gamma, tol=1e-3).fit(Xh, yh)
            sk = {"sklearn_s": time.perf_counter() - t0, "sklearn_sv": int(skm.n_support_.sum()),
                  "sklearn_acc": float((skm.predict(Xh) == yh).mean())}
        for path in args.paths.split(","):
            if path == "dense" and 4.0 * N * N > 0.4 * torch.cuda.mem_get_info()[0]:
                continue
            best = None
            for _ in range(args.reps):
                m, dt, peak = fit(X, y, path, gamma)
                best = (dt, m, peak) if best is None or dt < best[0] else best
            dt, m, peak = best
            acc = float((m.predict(X) == y).float().mean())
            Xt, yt = problem(20000, args.d, seed=11)
            held = float((m.predict(Xt) == yt).float().mean())
            rec = {"bench": "svm_fit", "N": N, "d": args.d, "path": path, "seconds": round(dt, 5),
                   "outer_steps": S.LAST_SOLVE.get("outer"), "solver": S.LAST_SOLVE.get("solver"),
                   "support_vectors": int(m.support_.numel()), "train_acc": acc,
                   "heldout_acc": held, "inner_steps": int(sum(m.iters)),
                   "cache": {k: v for k, v in S.LAST_SOLVE.items() if k.startswith("cache")},
                   "inner_per_outer": sum(m.iters) / max(1, S.LAST_SOLVE.get("outer") or 1),
                   "peak_bytes": int(peak), "dense_matrix_bytes": 4 * N * N}
            if args.sklearn_sub:
                from sklearn.svm import SVC as SKSVC
                sub = torch.randperm(N, generator=torch.Generator().manual_seed(3))[:args.sklearn_sub].to(X.device)
                t0 = time.perf_counter()
                skm = SKSVC(C=1.0, kernel="rbf", gamma=gamma, tol=1e-3).fit(X[sub].cpu().numpy(), y[sub].cpu().numpy())
                rec["sklearn_sub_rows"] = args.sklearn_sub
                rec["sklearn_sub_s"] = time.perf_counter() - t0
                rec["sklearn_sub_heldout_acc"] = float((skm.predict(Xt.cpu().numpy()) == yt.cpu().numpy()).mean())
            if sk:
                rec.update(sk)
                rec["speedup_vs_sklearn"] = sk["sklearn_s"] / dt
            print(json.dumps(rec), flush=True)
            if args.out:
                with open(args.out, "a") as fh:
                    fh.write(json.dumps(rec) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
