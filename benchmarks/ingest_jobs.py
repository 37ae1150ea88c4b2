"""End-to-end (file -> output file) timings of the text-layout CLI jobs, in-process
(benchmarks/bench_ingest.py --jobs).  Configs match data/synth_text.py's layouts."""
from __future__ import annotations

import os
import time

import torch

from avenir_amd.cli import main
from avenir_amd.data import synth_text as S

JOBS = {
    "mst": ("markovStateTransitionModel",
            "mst.model.states=" + ",".join(S.STATES) + "\nmst.skip.field.count=1\nmst.class.label.field.ord=1\n"),
    "apriori": ("frequentItemsApriori", "fia.support.threshold=0.01\nfia.max.item.set.length=3\nfia.skip.field.count=1\n"),
    "hmm": ("hiddenMarkovModelBuilder", "hmmb.model.states=S,T,U\nhmmb.model.observations=a,b,c,d\n"
            "hmmb.skip.field.count=1\n"),
    "tmc": ("topMatchesByClass", "tmc.class.attr.ord=1\ntmc.top.match.count=10\ntmc.compact.output=true\n"),
    "nen": ("nearestNeighbor", "nen.top.match.count=10\nnen.kernel.function=none\nnen.validation.mode=true\n"),
    "str": ("stateTransitionRate", None),
}


def _config(fmt: str, d: str) -> str:
    job, text = JOBS[fmt]
    if fmt == "str":
        p = os.path.join(d, "str.conf")
        with open(p, "w") as fh:
            fh.write("stateTransitionRate {\n key.field.ordinals = [0]\n time.field.ordinal = 1\n"
                     " state.field.ordinal = 2\n state.values = [A,B,C,D]\n rate.time.unit = hour\n}\n")
        return p
    p = os.path.join(d, f"{fmt}.properties")
    with open(p, "w") as fh:
        fh.write(text)
    return p


def run_job(fmt: str, path: str, d: str, reps: int = 3) -> dict:
    job, _ = JOBS[fmt]
    cfg = _config(fmt, d)
    out = os.path.join(d, f"{fmt}.out")
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    args = [job, "-i", path, "-o", out, "-c", cfg, "--device", dev]
    if fmt == "str":
        args += ["--app", "stateTransitionRate"]
    best = None
    n_out = 0
    for _ in range(reps):
        if dev == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        assert main(args) == 0
        if dev == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    with open(out, "rb") as fh:
        n_out = sum(1 for _ in fh)
    os.remove(out)
    with open(path, "rb") as fh:
        n_in = sum(1 for _ in fh)
    return {"job": job, "records": n_in, "seconds": round(best, 4), "records_per_s": n_in / best,
            "output_lines": n_out}
