#!/usr/bin/env python3
"""Small driver programs for hardware-counter passes (scripts/gpu_pmc.sh): each target runs a
handful of launches of ONE hot kernel at a roofline-relevant size, so a ``rocprofv3 --pmc`` pass
over it is short and its counters belong to that kernel.

    python benchmarks/pmc_targets.py {rowpack,columns,knn16,knn64,knn256,smo_ws,forest}
"""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rowpack():
    from avenir_amd.data.synth import churn_device
    from avenir_amd.ops import histogram as H
    n = 1 << 30
    codes, labels = churn_device(n, seed=1, device="cuda")
    rp = H.pack_rows(codes, n, [4, 3, 3, 3, 5], labels, 2)
    del codes, labels
    for _ in range(4):
        H.class_histogram_packed(rp)
    torch.cuda.synchronize()


def columns():
    from avenir_amd.data.synth import churn_device
    from avenir_amd.ops import histogram as H
    n = 1 << 29
    codes, labels = churn_device(n, seed=1, device="cuda")
    bins = [4, 3, 3, 3, 5]
    out = torch.zeros((2, sum(bins) + 1), dtype=torch.int64, device="cuda")
    for _ in range(4):
        out.zero_()
        H.class_histogram(codes, n, bins, labels, 2, out=out, mode=0, count_labels=True)
    torch.cuda.synchronize()


def _knn(D):
    from avenir_amd.ops import distance as Dm
    g = torch.Generator(device="cuda").manual_seed(0)
    Q = torch.randn((16384, D), device="cuda", generator=g)
    R = torch.randn((1 << 18, D), device="cuda", generator=g)
    for _ in range(3):
        Dm.knn(Q, R, 10)
    torch.cuda.synchronize()


def smo_ws():
    from avenir_amd.models.svm import kernel_matrix, smo_batch
    g = torch.Generator(device="cuda").manual_seed(9)
    X = torch.randn((8192, 8), device="cuda", generator=g)
    y = torch.where(X[:, 0] * X[:, 1] > 0, 1.0, -1.0)
    K = kernel_matrix(X, X, "rbf", 0.5).unsqueeze(0).contiguous()
    smo_batch(K, y.view(1, -1), 1.0, 1e-3, solver="ws")
    torch.cuda.synchronize()


def forest():
    import numpy as np
    from avenir_amd.models.forest import ForestBuilder
    from avenir_amd.ops import forest_ops as FO
    dev = torch.device("cuda")
    R, F, A = 1 << 25, 16, 256
    g = torch.Generator(device=dev).manual_seed(0)
    codes = torch.randint(0, 32, (F, R), generator=g, device=dev, dtype=torch.uint8)
    lab = torch.randint(0, 2, (R,), generator=g, device=dev, dtype=torch.uint8)
    wt = torch.randint(1, 4, (R,), generator=g, device=dev, dtype=torch.uint8)
    dc, dl, dw = torch.empty_like(codes), torch.empty_like(lab), torch.empty_like(wt)
    cnt = np.full(A, R // A, dtype=np.int64)
    start = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    feat = torch.randint(0, F, (A,), generator=g, device=dev, dtype=torch.int32)
    thr = torch.full((A,), 15, dtype=torch.int32, device=dev)
    bins = [32] * F
    bd = torch.tensor(bins, dtype=torch.int32, device=dev)
    od = torch.tensor(list(np.cumsum([0] + bins[:-1])), dtype=torch.int32, device=dev)
    inode, istart, ilen, nch = ForestBuilder(None, 1, None)._chunks(np.arange(A), start, cnt, 26000)
    il = FO.forest_part_count(codes, inode, istart, ilen, feat, thr).cpu().numpy().astype(np.int64)
    ends = np.cumsum(nch)
    first = ends - nch
    csum = np.concatenate([[0], np.cumsum(il)])
    nleft = csum[ends] - csum[first]
    rsum = np.concatenate([[0], np.cumsum(ilen.astype(np.int64) - il)])
    owner = inode.astype(np.int64)
    lbase = start[owner] + (csum[:-1] - csum[first[owner]])
    rbase = start[owner] + nleft[owner] + (rsum[:-1] - rsum[first[owner]])
    hist = torch.zeros((A, 2, sum(bins) + 1), dtype=torch.int64, device=dev)
    for _ in range(3):
        FO.forest_part_scatter(codes, lab, wt, dc, dl, dw, inode, istart, ilen, lbase, rbase, il, feat, thr)
        FO.forest_hist(codes, lab, wt, inode, istart, ilen, bd, od, bins, sum(bins) + 1, 2, hist)
        FO.forest_bootstrap(codes[:, : R // 4].contiguous(), lab, R // 4, list(range(4)), 0, 1, 0)
    torch.cuda.synchronize()


def kmeans():
    """K16 Lloyd pass at 16.7 M rows x 16 dims x 16 centroids."""
    from avenir_amd.models.cluster import kmeans_step
    g = torch.Generator(device="cuda").manual_seed(0)
    n, D, k = 1 << 24, 16, 16
    X = torch.randn((n, D), device="cuda", generator=g)
    C = X[torch.randint(0, n, (k,), device="cuda", generator=g)].clone()
    for _ in range(6):
        kmeans_step(X, [C])
    torch.cuda.synchronize()


TARGETS = {"kmeans": kmeans, "rowpack": rowpack, "columns": columns, "knn16": lambda: _knn(16), "knn64": lambda: _knn(64),
           "knn256": lambda: _knn(256), "smo_ws": smo_ws, "forest": forest}

if __name__ == "__main__":
    TARGETS[sys.argv[1]]()
