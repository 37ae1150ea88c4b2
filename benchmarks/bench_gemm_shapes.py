#!/usr/bin/env python3
"""fp32 GEMM shapes of the framework's hand-written MFMA kernels against torch (hipBLASLt) on the
same GPU: mlp.hip ``linear_act_fwd`` (Y = act(X Wᵀ + b)) at the BERT query shapes (128 rows) and the
LSTM shapes, gemm.hip ``gemm_tn`` (Aᵀ B) at the LSTM weight-gradient shapes.  One JSON line each."""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avenir_amd import _native  # noqa: E402

MODE = os.environ.get("AVMI_F32_GEMM", "bf16x3")


def timed(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    C = _native.C()
    g = torch.Generator(device="cuda").manual_seed(0)
    for M, N, K, act in ((128, 2304, 768, 0), (128, 768, 768, 0), (128, 3072, 768, 6), (128, 768, 3072, 0),
                         (1, 3072, 768, 6), (4096, 3072, 768, 6), (4096, 2304, 768, 0), (4096, 768, 768, 0), (4096, 768, 3072, 0),
                         (16384, 768, 768, 0), (8192, 2304, 768, 0), (2048, 3072, 768, 6),
                         (8192, 1024, 1024, 1), (5000, 400, 5, 0), (5000, 100, 400, 0)):
        X = torch.randn(M, K, generator=g, device="cuda")
        W = torch.randn(N, K, generator=g, device="cuda") / K ** 0.5
        b = torch.randn(N, generator=g, device="cuda")
        t_k = timed(lambda: C.linear_act_fwd(X, W, b, act))
        # with the weight's term planes split once (inference: weights fixed), when the call takes the
        # pre-split planes path
        P = C.sbf16_weight_planes(W) if C.linear_act_fwd_planes_bytes(M, N, K) else None
        t_kc = timed(lambda: C.linear_act_fwd(X, W, b, act, -1, P)) if P is not None else None
        if act == 6:
            ref = lambda: torch.nn.functional.gelu(torch.nn.functional.linear(X, W, b))
        elif act == 1:
            ref = lambda: torch.relu(torch.nn.functional.linear(X, W, b))
        else:
            ref = lambda: torch.nn.functional.linear(X, W, b)
        t_r = timed(ref)
        err = float((C.linear_act_fwd(X, W, b, act) - ref()).abs().max())
        # error against an fp64 oracle, for the kernel and for the library's fp32 GEMM
        z64 = torch.nn.functional.linear(X.double(), W.double(), b.double())
        y64 = (torch.nn.functional.gelu(z64) if act == 6 else torch.relu(z64) if act == 1 else z64)
        e_k = float((C.linear_act_fwd(X, W, b, act).double() - y64).abs().max())
        e_t = float((ref().double() - y64).abs().max())
        print(json.dumps({"op": "linear_act_fwd", "mode": MODE, "M": M, "N": N, "K": K, "act": act, "us": t_k * 1e6,
                          "torch_us": t_r * 1e6, "speedup": t_r / t_k, "TFLOPs": 2 * M * N * K / t_k / 1e12,
                          "us_cached_w": None if t_kc is None else t_kc * 1e6,
                          "speedup_cached_w": None if t_kc is None else t_r / t_kc,
                          "max_abs_diff": err, "err_fp64": e_k, "torch_err_fp64": e_t,
                          "err_over_sqrtK": e_k / K ** 0.5}), flush=True)
    for K, M, N in ((5000, 400, 106), (327680, 400, 106), (65536, 400, 201)):
        A = torch.randn(K, M, generator=g, device="cuda")
        B = torch.randn(K, N, generator=g, device="cuda")
        t_k = timed(lambda: C.gemm_tn(A, B), reps=20)
        t_r = timed(lambda: A.t() @ B, reps=20)
        err = float((C.gemm_tn(A, B) - A.t() @ B).abs().max())
        print(json.dumps({"op": "gemm_tn", "mode": MODE, "K": K, "M": M, "N": N, "us": t_k * 1e6, "torch_us": t_r * 1e6,
                          "speedup": t_r / t_k, "TFLOPs": 2 * M * N * K / t_k / 1e12, "max_abs_diff": err}), flush=True)


if __name__ == "__main__":
    main()
