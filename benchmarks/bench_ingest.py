"""Ingest-inclusive benchmarks of the text-layout jobs.

For each reference layout (data/synth_text.py) a file of ``--records`` records is written, then
timed on one device:

* ``tokenize``: file -> CSR token table (``read_records``; device tokenizer on a GPU, the
  multi-threaded host TextShard otherwise);
* ``job``: the whole CLI job, file -> output file (``python -m avenir_amd <job>`` semantics,
  in-process), records per second end to end.

One JSON line per (format, stage) on stdout; ``--out`` appends them to a file.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from avenir_amd.data import records as R  # noqa: E402
from avenir_amd.data import synth_text as S  # noqa: E402

TOKENIZE = {  # read_records options per layout
    "mst": dict(modes="xd"),
    "apriori": dict(modes="x"),
    "hmm": dict(modes="x", sub_delim=":"),
    "tmc": dict(modes="dddddd", tail_mode="n", numeric=True),
    "nen": dict(modes="xdnd", tail_mode="d", numeric=True),
    "str": dict(modes="dnd", numeric=True),
}


def sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 24)
    ap.add_argument("--formats", default=",".join(TOKENIZE))
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--host", action="store_true", help="also time the host tokenizer on a GPU box")
    ap.add_argument("--jobs", action="store_true", help="also time the full CLI jobs")
    ap.add_argument("--out", default=None)
    ap.add_argument("--dir", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    d = args.dir or tempfile.mkdtemp(prefix="avmi_ingest_")
    results = []

    def emit(rec):
        results.append(rec)
        print(json.dumps(rec), flush=True)

    for fmt in args.formats.split(","):
        path = os.path.join(d, f"{fmt}.txt")
        t0 = time.perf_counter()
        nbytes = S.write(fmt, path, args.records)
        gen_s = time.perf_counter() - t0
        opts = TOKENIZE[fmt]
        devices = [dev] + ([torch.device("cpu")] if args.host and dev.type == "cuda" else [])
        for dv in devices:
            best = None
            for _ in range(args.reps):
                sync()
                t0 = time.perf_counter()
                rec = R.read_records(path, device=dv, **opts)
                sync()
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            emit({"bench": "tokenize", "format": fmt, "device": str(dv), "path": rec.stats.get("path"),
                  "records": rec.n_lines, "tokens": rec.n_tokens, "vocab": len(rec.vocab), "bytes": nbytes,
                  "seconds": round(best, 4), "records_per_s": rec.n_lines / best, "GB_per_s": nbytes / best / 1e9,
                  "gen_s": round(gen_s, 2)})
            del rec
        if args.jobs:
            sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
            from ingest_jobs import run_job  # noqa: E402
            for _ in range(1):
                r = run_job(fmt, path, d, reps=args.reps)
                r.update({"bench": "job", "format": fmt, "device": str(dev), "bytes": nbytes})
                emit(r)
        os.remove(path)
    if args.out:
        with open(args.out, "a") as fh:
            for r in results:
                fh.write(json.dumps(r) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
