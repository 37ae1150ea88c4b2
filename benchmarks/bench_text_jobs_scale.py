#!/usr/bin/env python3
"""Wall time of the text CLI drivers (tests/test_text_jobs.py commands) on a corpus of ``--per``
documents per topic (3 topics, 6 sentences of 9 words each), on the job's device.  One JSON line
per stage (second run, warm process).

    python benchmarks/bench_text_jobs_scale.py [--per 2000] [--device cuda]
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

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import test_text_jobs as T  # noqa: E402

from avenir_amd.cli import main  # noqa: E402


def main_(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--per", type=int, default=2000)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("stages", nargs="*", help="stage names (default: all)")
    args = ap.parse_args(argv)
    tmp = Path(tempfile.mkdtemp(prefix="avmi_text_scale_"))
    try:
        d = T._corpus(tmp, n_per=args.per)
        ndocs = 3 * args.per
        dev = ["--device", args.device]
        stages = {
            "topicModel_train": ["topicModel", "--mode", "train", "--input", str(d), "--model", str(tmp / "lda.st"),
                                 "--output", str(tmp / "topics.txt"), "-D", "train.num.topics=3",
                                 "-D", "train.num.iter=40"],
            "termDistribution_base": ["termDistribution", "--mode", "buildBaseTf", "--input", str(d), "--model",
                                      str(tmp / "base.json")],
            "textEncoder_vectorise": ["textEncoder", "--mode", "vectorise", "--kind", "bi", "--input", str(d),
                                      "--output", str(tmp / "vec.csv")],
            "docToVec_train": ["docToVec", "--mode", "train", "--input", str(d), "--model", str(tmp / "d2v.st"),
                               "-D", "train.vector.size=32", "-D", "train.epochs=5"],
            "wordToVec_train": ["wordToVec", "--mode", "train", "--input", str(d), "--model", str(tmp / "w2v.st"),
                                "-D", "train.vector.size=32", "-D", "train.epochs=5"],
            "semanticSearch_corpus": ["semanticSearch", "--mode", "tokenAvMax", "--input", str(d), "--name",
                                      "rocket orbit moon", "--k", "5", "--output", str(tmp / "ss.txt"),
                                      "-D", "embed.epochs=3"],
        }
        for name, cmd in stages.items():
            if args.stages and name not in args.stages:
                continue
            times = []
            for _ in range(2):
                t0 = time.perf_counter()
                main(cmd + dev)
                times.append(time.perf_counter() - t0)
            print(json.dumps({"bench": "text_job_scale", "stage": name, "docs": ndocs, "cold_s": times[0],
                              "warm_s": times[1], "docs_per_s": ndocs / times[1]}), flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(main_())
