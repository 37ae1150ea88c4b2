"""Host-side profile of one GBT fit (120 x depth 3, the reference's defaults) at --rows rows:
wall time of three fits, then cProfile of a fourth sorted by internal time."""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 16)
    ap.add_argument("--bins", type=int, default=64)
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from bench_vs_reference import as_table, tree_data
    from avenir_amd.models.tree import GBTParams, GradientBoostedTrees

    class A:
        rows = a.rows
        tree_rows = a.rows
    Xtr, ytr, _, _ = tree_data(A)
    t = as_table(Xtr[: a.rows], ytr[: a.rows])
    p = GBTParams(n_estimators=120, learning_rate=0.12, max_depth=3, max_bins=a.bins)
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m = GradientBoostedTrees(t.schema, p).fit(t)
        torch.cuda.synchronize()
        print(f"fit {time.perf_counter() - t0:.4f} s graph={getattr(m, 'graph_used', None)}", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    GradientBoostedTrees(t.schema, p).fit(t)
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue(), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
