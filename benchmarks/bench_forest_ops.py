#!/usr/bin/env python3
"""Micro-benchmark of the forest builder kernels (forest.hip) on one GPU: the stable partition
(scatter), the segment histogram and the partition count, at the row / feature counts of the RF
benchmark (106 M bootstrap rows x 16 features), with achieved bandwidth per kernel.

    python benchmarks/bench_forest_ops.py [--rows 106000000] [--feat 16] [--chunk 26000]
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


def main():
    from avenir_amd.ops import forest_ops as FO
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=106_000_000)
    ap.add_argument("--feat", type=int, default=16)
    ap.add_argument("--nodes", type=int, default=640)
    ap.add_argument("--chunks", default="8192,26000,65536")
    a = ap.parse_args()
    dev = torch.device("cuda")
    R, F, A = a.rows, a.feat, a.nodes
    g = torch.Generator(device=dev).manual_seed(0)
    codes = torch.randint(0, 32, (F, R), generator=g, device=dev, dtype=torch.uint8)
    lab = torch.randint(0, 2, (R,), generator=g, device=dev, dtype=torch.uint8)
    wt = torch.randint(1, 4, (R,), generator=g, device=dev, dtype=torch.uint8)
    dc, dl, dw = torch.empty_like(codes), torch.empty_like(lab), torch.empty_like(wt)
    # A equal segments
    cnt = np.full(A, R // A, dtype=np.int64)
    cnt[-1] += R - cnt.sum()
    start = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    feat = torch.randint(0, F, (A,), generator=g, device=dev, dtype=torch.int32)
    thr = torch.full((A,), 15, dtype=torch.int32, device=dev)
    bins = [32] * F
    bd = torch.tensor(bins, dtype=torch.int32, device=dev)
    od = torch.tensor(list(np.cumsum([0] + bins[:-1])), dtype=torch.int32, device=dev)
    TB = sum(bins) + 1
    from avenir_amd.models.forest import ForestBuilder
    fb = ForestBuilder(None, 1, None)
    for chunk in [int(c) for c in a.chunks.split(",")]:
        inode, istart, ilen, nch = fb._chunks(np.arange(A), start, cnt, chunk)
        il = FO.forest_part_count(codes, inode, istart, ilen, feat, thr)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            il = FO.forest_part_count(codes, inode, istart, ilen, feat, thr)
        torch.cuda.synchronize()
        t_count = (time.perf_counter() - t0) / 5
        il_h = il.cpu().numpy().astype(np.int64)
        ends = np.cumsum(nch)
        first = ends - nch
        csum = np.concatenate([[0], np.cumsum(il_h)])
        nleft = csum[ends] - csum[first]
        rsum = np.concatenate([[0], np.cumsum(ilen.astype(np.int64) - il_h)])
        owner = inode.astype(np.int64)
        lbase = start[owner] + (csum[:-1] - csum[first[owner]])
        rbase = start[owner] + nleft[owner] + (rsum[:-1] - rsum[first[owner]])
        FO.forest_part_scatter(codes, lab, wt, dc, dl, dw, inode, istart, ilen, lbase, rbase, il_h, feat, thr)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            FO.forest_part_scatter(codes, lab, wt, dc, dl, dw, inode, istart, ilen, lbase, rbase, il_h, feat, thr)
        torch.cuda.synchronize()
        t_sc = (time.perf_counter() - t0) / 5
        hist = torch.zeros((A, 2, TB), dtype=torch.int64, device=dev)
        FO.forest_hist(codes, lab, wt, inode, istart, ilen, bd, od, bins, TB, 2, hist)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            FO.forest_hist(codes, lab, wt, inode, istart, ilen, bd, od, bins, TB, 2, hist)
        torch.cuda.synchronize()
        t_h = (time.perf_counter() - t0) / 5
        mb = R * (F + 2)
        print(json.dumps({"chunk": chunk, "items": int(inode.size), "rows": R, "features": F,
                          "scatter_ms": t_sc * 1e3, "scatter_TBps": 2 * mb / t_sc / 1e12,
                          "hist_ms": t_h * 1e3, "hist_TBps": mb / t_h / 1e12,
                          "count_ms": t_count * 1e3, "count_TBps": R / t_count / 1e12}), flush=True)


if __name__ == "__main__":
    main()
