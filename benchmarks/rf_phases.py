#!/usr/bin/env python3
"""Phase timing of one RandomForest.fit on the bench_vs_reference data shape (1 M rows x 16)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from benchmarks.bench_vs_reference import as_table, tree_data
    from avenir_amd.models import tree as T
    from avenir_amd.models.forest import ForestBuilder

    class A:
        tree_rows = 1 << 20
    Xtr, ytr, _, _ = tree_data(A())
    t = as_table(Xtr, ytr)
    p = T.TreeParams(binary=True, stopping="maxDepth", max_depth=8, sub_sampling="withReplace",
                     attr_selection="randomAll", max_bins=32)
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        space = T.build_split_space(t.schema, t, binary=True, max_bins=32)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        codes = T.encode_for_tree(space, t)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        p.random_attr_count = 4
        fb = ForestBuilder(t.schema, 10, p)
        trees = fb.fit(t, space=space, codes=codes)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        rf = T.RandomForest(t.schema, 10, p, "sqrt").fit(t)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        print(json.dumps({"rep": rep, "space_ms": (t1 - t0) * 1e3, "encode_ms": (t2 - t1) * 1e3,
                          "builder_ms": (t3 - t2) * 1e3, "builder_internal_ms": fb.stats["seconds"] * 1e3,
                          "rf_fit_ms": (t4 - t3) * 1e3, "levels_ms": [round(x * 1e3, 2) for x in fb.level_times]}),
              flush=True)


if __name__ == "__main__":
    main()
