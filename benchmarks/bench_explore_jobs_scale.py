#!/usr/bin/env python3
"""End-to-end (file -> output file) throughput of the record-wise exploration / encoding / sampling
CLI jobs at scale, with the configurations of tests/test_native_explore_jobs.py and its record
layout (id, three categoricals, a class, two numbers) scaled to ``--rows`` records.  One JSON line
per job: seconds of the second (warm) run and records/s.

    python benchmarks/bench_explore_jobs_scale.py --rows 2097152 [--device cuda] [jobs ...]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import test_native_explore_jobs as T  # noqa: E402

from avenir_amd.cli import main  # noqa: E402

DATA_CASES = ["nuc", "rue", "usb", "abe", "abu", "hash", "loo", "loo_test", "dummy", "dummy_ci", "spc", "kmc",
              "bag", "nor", "pro", "tra", "uvc", "nads"]


def big_rows(n: int, seed: int = 3) -> list[str]:
    """The test's record layout, vectorised: r<i>,a,b,c,cls,uniform,normal."""
    rng = np.random.default_rng(seed)
    cats = np.array(["x", "y", "z", "Y"])
    a = cats[rng.integers(0, 4, n)]
    b = np.where(rng.random(n) < 0.7, a, cats[rng.integers(0, 3, n)])
    c = np.array(["p", "q"])[rng.integers(0, 2, n)]
    cls = np.where(((a == "x") & (rng.random(n) < 0.8)) | (rng.random(n) < 0.2), "T", "F")
    u = np.char.mod("%.4f", rng.random(n))
    z = np.char.mod("%.5f", rng.normal(size=n))
    ids = np.char.add("r", np.arange(n).astype(str))
    parts = [ids, a, b, c, cls, u, z]
    out = parts[0]
    for p in parts[1:]:
        out = np.char.add(np.char.add(out, ","), p)
    return out.tolist()


def main_(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 21)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("jobs", nargs="*")
    args = ap.parse_args(argv)
    rows = big_rows(args.rows)
    T._cat_rows = lambda n=700, seed=3: rows          # the harness writes d.csv from this
    tmp = Path(tempfile.mkdtemp(prefix="avmi_explore_scale_"))
    try:
        for name in args.jobs or DATA_CASES:
            d = tmp / name
            d.mkdir()
            argv_, cfg = T._setup(d, name, False)
            nbytes = os.path.getsize(d / "d.csv")
            cmd = [str(a) for a in argv_] + ["-c", str(cfg), "--device", args.device]
            times = []
            for rep in range(2):
                out = d / f"out{rep}"
                t0 = time.perf_counter()
                rc = main(cmd + ["-o", str(out)])
                times.append(time.perf_counter() - t0)
                if rc != 0:
                    raise SystemExit(f"{name}: rc {rc}")
            print(json.dumps({"bench": "explore_job_scale", "case": name, "job": str(argv_[0]), "rows": args.rows,
                              "file_bytes": nbytes, "cold_s": times[0], "warm_s": times[1],
                              "rows_per_s": args.rows / times[1]}), flush=True)
            shutil.rmtree(d, ignore_errors=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(main_())
