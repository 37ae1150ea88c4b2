#!/usr/bin/env python3
"""Micro-benchmark of one working-set SMO sub-problem solve (gather + smo_ws_solve_kernel) at a
mid-solve state: time per call against the iteration cap, so the fixed cost (launch, K-block
staging, state loads, write-back) and the per-iteration cost separate."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from avenir_amd import _native  # noqa: E402
from avenir_amd.models.svm import _WorkingSetSMO, kernel_matrix  # noqa: E402


def main(N=8192, warm_steps=60, reps=50):
    g = torch.Generator(device="cuda").manual_seed(9)
    X = torch.randn((N, 8), device="cuda", generator=g)
    y = torch.where(X[:, 0] * X[:, 1] > 0, 1.0, -1.0).view(1, -1)
    K = kernel_matrix(X, X, "rbf", 0.5).unsqueeze(0).contiguous()
    st = _WorkingSetSMO(K, y, 1.0, 1e-3, 2048, 128, True, 0.3)
    for _ in range(warm_steps):
        st.step()
    C_ = _native.C()
    C_.smo_ws_select(st.alpha, st.G, st.yf, st.C, 64, st.ws_buf, st.ok_buf, st.gap)
    a0, g0 = st.alpha.clone(), st.G.clone()
    torch.cuda.synchronize()
    for cap in (0, 1, 4, 16, 64, 2048):
        ts, its = [], []
        for r in range(reps):
            st.alpha.copy_(a0)
            st.G.copy_(g0)
            before = int(st.inner_total[0])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            C_.smo_ws_solve_fused(K, st.ws_buf, st.ok_buf, st.alpha, st.G, st.yf, st.gap, st.C, st.eps, cap,
                                  st.dA_buf, st.inner_total, 0.3)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
            its.append(int(st.inner_total[0]) - before)
        ts.sort()
        print(json.dumps({"bench": "smo_solve_call", "N": N, "cap": cap, "iters": its[0],
                          "us_median": ts[len(ts) // 2], "us_min": ts[0]}), flush=True)


if __name__ == "__main__":
    main()
