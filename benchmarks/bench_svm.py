#!/usr/bin/env python3
"""K12 SVM solvers on one MI355X: full single-workgroup SMO vs the working-set decomposition
(one wavefront per Q=128 sub-problem, K block in LDS), RBF kernel, XOR-like labels."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from avenir_amd.models.svm import SVC, kernel_matrix, smo_batch  # noqa: E402


def run(N, solver):
    g = torch.Generator(device="cuda").manual_seed(9)
    X = torch.randn((N, 8), device="cuda", generator=g)
    y = torch.where(X[:, 0] * X[:, 1] > 0, 1.0, -1.0)
    K = kernel_matrix(X, X, "rbf", 0.5).unsqueeze(0).contiguous()
    smo_batch(K[:, :256, :256].contiguous(), y[:256].view(1, -1), 1.0, 1e-3, solver=solver)   # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    a, rho, it = smo_batch(K, y.view(1, -1), 1.0, 1e-3, solver=solver)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ya = a[0] * y
    dual = float(0.5 * ya.double() @ K[0].double() @ ya.double() - a[0].double().sum())
    from avenir_amd.models.svm import LAST_SOLVE
    print(json.dumps({"bench": "svm_solver", "N": N, "solver": solver, "seconds": dt, "inner_iters": int(it[0]),
                      "outer_steps": LAST_SOLVE.get("outer") if solver == "ws" else None,
                      "rel_tol": float(os.environ.get("AVMI_SMO_REL_TOL", "0.3")),
                      "support_vectors": int((a[0] > 0).sum()), "dual": dual}), flush=True)


if __name__ == "__main__":
    sizes = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else ("2048", "8192", "32768"))]
    solvers = sys.argv[2].split(",") if len(sys.argv) > 2 else ("full", "ws")
    for N in sizes:
        for solver in solvers:
            if solver == "full" and N > 8192:
                continue
            run(N, solver)
