"""featureCondProbJoiner (J/knn/FeatureCondProbJoiner.java:105-178) on the native data-parallel path.

* the native join equals a plain-Python oracle of the reference's map + reduce (prob-file record
  keyed by training id, its ``classVal`` = last field and the posterior of that class; every
  distance pair of the id -> ``testId,testClass,trainId,dist,classVal,prob``), including ragged
  prob lines, a prob line whose class is missing from its pairs and pairs with no posterior;
* world 2 / 4 (gloo ranks): each rank reads only its byte range of the pair files (the prob file is
  read whole by every rank, as a side file), and the union of the part files equals world 1;
* GPU: the device tokenizer + device formatter give the same lines as the CPU path.
"""
from __future__ import annotations

import os
import random
from pathlib import Path

import pytest

from avenir_amd.cli import main
from avenir_amd.jobs import common as JC

from _dist import run_world


def _lines(p):
    p = Path(p)
    if p.is_dir():
        return [l for f in sorted(p.iterdir()) if f.is_file() for l in f.read_text().splitlines() if l.strip()]
    return [l for l in p.read_text().splitlines() if l.strip()]


def _make(tmp: Path, n_train=120, n_test=40, seed=3):
    rnd = random.Random(seed)
    classes = ["pass", "fail", "hold"]
    pairs = tmp / "pairs"
    pairs.mkdir()
    with open(pairs / "part-00000", "w") as f:
        for te in range(n_test):
            for tr in range(n_train + 5):                    # ids tr >= n_train have no posterior
                f.write(f"T{tr},Q{te},{rnd.randint(0, 5000)},{rnd.choice(classes)},{rnd.choice(classes)}\n")
    prob = tmp / "prob"
    prob.mkdir()
    with open(prob / "prDistr-00000", "w") as f:
        for tr in range(n_train):
            k = 2 if tr % 7 else 3                           # ragged: 2 or 3 (class, prob) pairs
            cls = classes[:k]
            ps = [f"{rnd.random():.6f}" for _ in cls]
            actual = rnd.choice(cls) if tr % 11 else "other"  # 'other': no matching class -> dropped
            body = ",".join(f"{c},{p}" for c, p in zip(cls, ps))
            f.write(f"T{tr},{rnd.random():.4f},{body},{actual}\n")
    cfg = tmp / "fcb.properties"
    cfg.write_text("fcb.feature.cond.prob.split.prefix=prDistr\n")
    return pairs, prob, cfg


def _oracle(pairs: Path, prob: Path) -> list[str]:
    post = {}
    for l in _lines(prob):
        p = l.split(",")
        cls = p[-1]
        for i in range(2, len(p) - 1, 2):
            if p[i] == cls:
                post.setdefault(p[0], (cls, p[i + 1]))
                break
    out = []
    for l in _lines(pairs):
        p = l.split(",")
        if p[0] in post:
            c, pr = post[p[0]]
            out.append(",".join([p[1], p[4], p[0], p[2], c, pr]))
    return out


def test_native_join_matches_reference_semantics(tmp_path):
    pairs, prob, cfg = _make(tmp_path)
    out = tmp_path / "join.txt"
    assert main(["featureCondProbJoiner", "-i", f"{pairs},{prob}", "-o", str(out), "-c", str(cfg),
                 "--device", "cpu"]) == 0
    got, ref = _lines(out), _oracle(pairs, prob)
    assert len(ref) > 1000
    assert got == ref


def _world(rank, world, argv, out, cfg):
    JC.IO_STATS["bytes_read"] = 0
    assert main(argv + ["-o", out, "-c", cfg, "--device", "cpu"]) == 0
    return JC.IO_STATS["bytes_read"]


@pytest.mark.parametrize("world", [2, 4])
def test_join_byte_ranges_and_world_invariance(tmp_path, world):
    pairs, prob, cfg = _make(tmp_path, n_train=200, n_test=50)
    argv = ["featureCondProbJoiner", "-i", f"{pairs},{prob}"]
    out = tmp_path / f"w{world}"
    read = run_world(_world, world, argv, str(out), str(cfg), timeout=300)
    assert sorted(_lines(out)) == sorted(_oracle(pairs, prob))
    pbytes = os.path.getsize(prob / "prDistr-00000")
    tbytes = os.path.getsize(pairs / "part-00000")
    pair_read = [r - pbytes for r in read]                 # every rank reads the prob file whole
    assert sum(pair_read) == tbytes                        # every pair byte read exactly once
    assert max(pair_read) <= tbytes / world * 1.05 + 200   # each rank about its share


@pytest.mark.gpu
def test_join_gpu_equals_cpu(cuda, tmp_path, monkeypatch):
    from avenir_amd.data import records as R
    monkeypatch.setattr(R, "DEVICE_MIN_BYTES", 0)          # device tokenizer on small files too
    monkeypatch.setattr(R, "DEVICE_FORMAT_MIN_ROWS", 0)    # device output formatter too
    pairs, prob, cfg = _make(tmp_path, n_train=300, n_test=80)
    outs = {}
    for d in ("cpu", "cuda"):
        out = tmp_path / f"{d}.txt"
        assert main(["featureCondProbJoiner", "-i", f"{pairs},{prob}", "-o", str(out), "-c", str(cfg),
                     "--device", d]) == 0
        outs[d] = _lines(out)
    assert outs["cuda"] == outs["cpu"] == _oracle(pairs, prob)
