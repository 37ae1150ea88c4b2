#!/usr/bin/env python3
"""Latency of the hand-written peer-mapped all-reduce (csrc/kernels/comm.hip) with W processes
sharing one GPU (the gloo:cuda rehearsal harness of tests/_dist.py): per-call time of back-to-back
device sums at 8 KB .. 4 MB, one-shot and two-shot, next to the gloo library all-reduce of the
same device tensor (host round trip).  One JSON line per (world, bytes, algo) on stdout.

Usage: python benchmarks/bench_p2p.py [--worlds 2,4] [--iters 500]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _measure(rank, world, iters):
    import torch
    from avenir_amd.parallel.comm import get_comm
    comm = get_comm()
    dev = comm.device
    rows = []
    for nbytes in (8 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20):
        for algo in ("oneshot", "twoshot"):
            x = torch.ones(nbytes // 4, device=dev)
            for _ in range(20):
                comm.p2p().all_reduce(x, algo=algo)
            torch.cuda.synchronize()
            comm.barrier()
            t0 = time.perf_counter()
            for _ in range(iters):
                comm.p2p().all_reduce(x, algo=algo)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / iters
            rows.append({"bytes": nbytes, "algo": algo, "us": dt * 1e6})
    comm.p2p().check()
    # the gloo library all-reduce of the same device tensor, for scale (host round trip)
    x = torch.ones(2048, device=dev)
    for _ in range(5):
        comm.all_reduce(x)
    comm.barrier()
    k = 50
    t0 = time.perf_counter()
    for _ in range(k):
        comm.all_reduce(x)
    torch.cuda.synchronize()
    rows.append({"bytes": 8 << 10, "algo": "gloo_library", "us": (time.perf_counter() - t0) / k * 1e6})
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="2,4")
    ap.add_argument("--iters", type=int, default=500)
    a = ap.parse_args()
    from _dist import run_world
    for w in (int(v) for v in a.worlds.split(",")):
        res = run_world(_measure, w, a.iters, timeout=600, comm="gloo:cuda")
        for i, row in enumerate(res[0]):
            worst = max(r[i]["us"] for r in res)
            print(json.dumps({"bench": "p2p_all_reduce_shared_gpu", "world": w, **row, "us_max_rank": worst,
                              "note": f"{w} processes on ONE MI355X; peers mapped through hipIpcOpenMemHandle"}),
                  flush=True)


if __name__ == "__main__":
    main()
