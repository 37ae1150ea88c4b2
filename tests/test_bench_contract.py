"""bench.py's driver contract (one JSON line from rank 0 with the required keys; ``value`` is the
whole-job rate; the max over ranks is the step time) and its multi-rank extras — the count-table
all-reduce choice and the checked collective self-test — on CPU ranks over gloo."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

from tests._dist import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _run(cmd, timeout=600):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", MASTER_ADDR="127.0.0.1")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.strip().startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_single_rank_contract():
    d = _run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--ingest-rows", "0"])
    assert KEYS <= set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["value"] > 0 and d["config"]["parallelism"] == "dp1"


def test_bench_two_ranks_selftest():
    port = free_port()
    d = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
              "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
              "--steps", "2", "--warmup", "1", "--probe-allreduce", "--ingest-rows", "0"])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["global_batch"] == 2 * d["config"]["rows_per_gpu"]
    st = d["extra"]["comm_selftest"]
    assert st["ok"], st
    for k in ("ring_batch_isend_irecv", "ring_iter", "all_to_all_v", "all_gather_v", "barrier"):
        assert st[k]["ok"], (k, st[k])
    assert d["extra"]["count_allreduce"]["chosen"] == "rccl"       # no GPU: the library collective
