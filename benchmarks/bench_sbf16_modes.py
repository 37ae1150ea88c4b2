#!/usr/bin/env python3
"""gemm.hip ``gemm_tn`` (the LSTM weight-gradient Aᵀ B) and distance.hip ``knn_topk`` (squared
euclidean top-k) in each arithmetic mode — fp32 MFMA (0), split-bf16 x3 (3), x6 (6) — with the
error of each against an fp64 oracle and the library (hipBLASLt) time for the GEMM.  One JSON line
per (kernel, shape, mode)."""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avenir_amd import _native  # noqa: E402
from avenir_amd.ops import distance as Dm  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def gemm():
    C = _native.C()
    g = torch.Generator(device="cuda").manual_seed(0)
    for K, M, N in ((5000, 400, 106), (40000, 400, 106), (327680, 400, 106), (65536, 400, 201)):
        A = torch.randn(K, M, generator=g, device="cuda")
        B = torch.randn(K, N, generator=g, device="cuda")
        t_r = timed(lambda: A.t() @ B)
        sub = min(K, 40000)                      # fp64 oracle on the first rows (host memory / time)
        ref = (A[:sub].double().t() @ B[:sub].double())
        e_t = float(((A[:sub].t() @ B[:sub]).double() - ref).abs().max())
        for mode in (0, 3, 6):
            t_k = timed(lambda: C.gemm_tn(A, B, prec=mode))
            e_k = float((C.gemm_tn(A[:sub].contiguous(), B[:sub].contiguous(), prec=mode).double() - ref).abs().max())
            print(json.dumps({"op": "gemm_tn", "mode": {0: "f32", 3: "bf16x3", 6: "bf16x6"}[mode], "K": K, "M": M,
                              "N": N, "us": t_k * 1e6, "torch_us": t_r * 1e6, "speedup_vs_torch": t_r / t_k,
                              "TFLOPs": 2 * M * N * K / t_k / 1e12, "err_fp64_first_rows": e_k,
                              "torch_err_fp64_first_rows": e_t, "oracle_rows": sub}), flush=True)


def knn():
    g = torch.Generator(device="cuda").manual_seed(1)
    for M, N, D, k in ((65536, 65536, 16, 10), (16384, 1048576, 32, 10), (16384, 262144, 64, 10),
                       (8192, 131072, 256, 10)):
        Q = torch.randn(M, D, generator=g, device="cuda")
        R = torch.randn(N, D, generator=g, device="cuda")
        qs = Q[:512]
        ref = torch.cdist(qs.double(), R.double())
        bd, bi = torch.topk(ref, k, dim=1, largest=False)
        for mode in (0, 3, 6):
            t = timed(lambda: Dm.knn(Q, R, k, prec=mode), reps=5)
            d, i = Dm.knn(qs, R, k, prec=mode)
            print(json.dumps({"op": "knn_topk", "mode": {0: "f32", 3: "bf16x3", 6: "bf16x6"}[mode], "M": M, "N": N,
                              "D": D, "k": k, "ms": t * 1e3, "pairs_per_s": M * N / t,
                              "TFLOPs": 2 * M * N * D / t / 1e12,
                              "max_dist_err_fp64": float((d.double() - bd).abs().max()),
                              "index_agreement": float((i == bi).float().mean())}), flush=True)


if __name__ == "__main__":
    for w in sys.argv[1:] or ["gemm", "knn"]:
        globals()[w]()
