#!/usr/bin/env python3
"""End-to-end (file -> output file) throughput of the keyed / data-parallel CLI jobs at scale: the
configurations of tests/test_data_parallel_jobs.py on inputs of ``--scale`` x their test sizes
(layouts generated vectorised here).  One JSON line per job: seconds of the second (warm) run and
input lines/s.

    python benchmarks/bench_keyed_jobs_scale.py [--scale 400] [--device cuda] [jobs ...]
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

import test_data_parallel_jobs as T  # noqa: E402

from avenir_amd.cli import main  # noqa: E402

CASES = ["gr", "nr", "sg", "td", "kpp", "mab", "gb", "smb", "rfb", "cgs"]


def _join(*cols) -> list[str]:
    out = np.asarray(cols[0]).astype(str)
    for c in cols[1:]:
        out = np.char.add(np.char.add(out, ","), np.asarray(c).astype(str))
    return out.tolist()


def _write(path: Path, lines: list[str]) -> int:
    path.write_text("\n".join(lines) + "\n")
    return len(lines)


def make_input(name: str, path: Path, scale: int) -> int:
    """The test's layout for ``name`` at ``scale`` x its size; returns the line count."""
    rng = np.random.default_rng(7)
    f = lambda a, p: np.char.mod(p, a)
    if name == "gr":                       # groups of points: pairs stay within a group (~100 per group)
        n = 900 * scale
        g = np.char.add("g", rng.integers(0, n // 100, n).astype(str))
        ids = np.char.add("p", np.arange(n).astype(str))
        return _write(path, _join(g, ids, f(rng.normal(size=n), "%.4f"), f(rng.normal(size=n), "%.4f"),
                                  rng.integers(0, 10, n)))
    if name == "nr":
        n = 3000 * scale
        ents = 400 * scale
        return _write(path, _join(np.char.add("e", rng.integers(0, ents, n).astype(str)),
                                  np.char.add("e", rng.integers(0, ents, n).astype(str)), rng.integers(0, 51, n)))
    if name == "sg":
        n = 2500 * scale
        i = np.arange(n)
        return _write(path, _join(np.char.add("k", rng.integers(0, 150 * scale, n).astype(str)),
                                  np.array(["a", "b"])[rng.integers(0, 2, n)], rng.integers(0, 61, n),
                                  np.char.add("v", (i % 7).astype(str)), np.char.add("w", (i % 5).astype(str))))
    if name == "td":
        n = 3000 * scale
        i = np.arange(n)
        return _write(path, _join(np.char.add("k", rng.integers(0, 60 * scale, n).astype(str)), i * 7 % 1000,
                                  np.array(["L", "M", "H", "HH"])[rng.integers(0, 4, n)]))
    if name == "kpp":
        n = 1200 * scale
        c = rng.integers(0, 3, n)
        return _write(path, _join(np.char.add("g", rng.integers(0, 7, n).astype(str)),
                                  f(c * 4 + rng.normal(0, .3, n), "%.4f"), f(c * 3 + rng.normal(0, .3, n), "%.4f")))
    if name == "mab":
        n = 3000 * scale
        return _write(path, _join(np.char.add("grp", rng.integers(0, 40 * scale, n).astype(str)),
                                  np.array(["a1", "a2", "a3"])[rng.integers(0, 3, n)], rng.integers(0, 101, n)))
    if name in ("gb", "smb", "rfb"):
        G = 45 * scale
        k = rng.integers(1, 10, G)
        g = np.repeat(np.arange(G), k)
        it = np.concatenate([np.arange(m) for m in k])
        n = len(g)
        return _write(path, _join(np.char.add("grp", g.astype(str)), np.char.add("item", it.astype(str)),
                                  rng.integers(1, 31, n), f(rng.random(n) * 5, "%.3f")))
    if name == "cgs":
        n = 2000 * scale
        sym = np.array([f"i{j}" for j in range(40)])
        return _write(path, _join(sym[rng.integers(0, 40, n)], sym[rng.integers(0, 40, n)], sym[rng.integers(0, 40, n)],
                                  np.full(n, "0.1")))
    raise KeyError(name)


def main_(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=400)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("jobs", nargs="*")
    args = ap.parse_args(argv)
    tmp = Path(tempfile.mkdtemp(prefix="avmi_keyed_scale_"))
    try:
        for name in args.jobs or CASES:
            d = tmp / name
            d.mkdir()
            argv_, text, data = T._setup(d, name)
            lines = make_input(name, Path(data), args.scale)
            cfg = T._conf(d, text)
            cmd = [str(a) for a in argv_] + T._app([str(a) for a in argv_]) + ["-c", str(cfg), "--device", args.device]
            times = []
            for rep in range(2):
                t0 = time.perf_counter()
                rc = main(cmd + ["-o", str(d / f"out{rep}")])
                times.append(time.perf_counter() - t0)
                if rc != 0:
                    raise SystemExit(f"{name}: rc {rc}")
            print(json.dumps({"bench": "keyed_job_scale", "case": name, "job": str(argv_[0]), "lines": lines,
                              "file_bytes": os.path.getsize(data), "cold_s": times[0], "warm_s": times[1],
                              "lines_per_s": lines / times[1]}), flush=True)
            shutil.rmtree(d, ignore_errors=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(main_())
