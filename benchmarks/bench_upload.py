"""Sweep of the K1 device-CSV upload (page cache -> pinned staging ring -> HBM): source mode
(``AVMI_UPLOAD_MODE`` pread / mmap) x host threads (``AVMI_UPLOAD_THREADS``) x DMA queues (``AVMI_UPLOAD_STREAMS``, setting
``mode:threads:streams``) on the bench's
2^26-record churn CSV.  Prints one JSON line per setting: best-of-``--reps`` ``load_csv`` seconds,
file GB/s and records/s, and the NB fit + model-lines time on the loaded table.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 26)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--settings", default="mmap:4,pread:4,pread:8,pread:16")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from avenir_amd.data import synth
    from avenir_amd.data.synth import CHURN_SCHEMA
    from avenir_amd.data.table import load_csv
    from avenir_amd.models.bayes import NaiveBayes
    from avenir_amd.utils.schema import FeatureSchema

    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    schema = FeatureSchema.from_json(CHURN_SCHEMA)
    d = "/dev/shm" if os.path.isdir("/dev/shm") else "/tmp"
    path = os.path.join(d, f"avmi_upload_{os.getpid()}.csv")
    out = []
    try:
        nbytes = synth.write_churn_native(path, args.rows, seed=99)
        with open(path, "rb") as fh:
            while fh.read(1 << 26):
                pass
        ref = None
        for s in args.settings.split(","):
            mode, th, *ns = s.split(":")
            os.environ["AVMI_UPLOAD_MODE"] = mode
            os.environ["AVMI_UPLOAD_THREADS"] = th
            os.environ["AVMI_UPLOAD_STREAMS"] = ns[0] if ns else "1"
            best = float("inf")
            t = None
            for _ in range(args.reps + 1):
                if dev.type == "cuda":
                    torch.cuda.synchronize()
                t0 = time.perf_counter()
                t = load_csv(path, schema, device=dev, rank=0, world=1)
                if dev.type == "cuda":
                    torch.cuda.synchronize()
                best = min(best, time.perf_counter() - t0)
            nb = NaiveBayes(schema).fit(t)
            counts = nb.counts.cpu()
            if ref is None:
                ref = counts
            assert torch.equal(ref, counts), f"counts differ under {s}"
            rec = {"bench": "csv_upload", "mode": mode, "threads": int(th), "streams": int(ns[0]) if ns else 1, "rows": args.rows,
                   "bytes": nbytes, "load_s": best, "GB_per_s": nbytes / best / 1e9,
                   "rows_per_s": args.rows / best, "device": str(dev)}
            out.append(rec)
            print(json.dumps(rec), flush=True)
    finally:
        if os.path.exists(path):
            os.remove(path)
    if args.out:
        with open(args.out, "a") as fh:
            for r in out:
                fh.write(json.dumps(r) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
