"""cProfile of one end-to-end run of each prediction job at ``--records`` records (the phases
behind benchmarks/bench_predict_jobs.py): top functions by cumulative time, one block per job."""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from bench_predict_jobs import _run, setup  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 24)
    ap.add_argument("--jobs", default="vit,nbp")
    ap.add_argument("--top", type=int, default=30)
    args = ap.parse_args()
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    d = tempfile.mkdtemp(prefix="avmi_prof_")
    for job in args.jobs.split(","):
        argv, _ = setup(job, d, args.records, dev)
        out = os.path.join(d, f"{job}.out")
        _run(argv + ["-o", out, "--device", dev])          # warm-up (first-load costs)
        pr = cProfile.Profile()
        if dev == "cuda":
            os.environ["AVMI_SYNC_PROFILE"] = "1"
        pr.enable()
        _run(argv + ["-o", out, "--device", dev])
        if dev == "cuda":
            torch.cuda.synchronize()
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(args.top)
        print(f"===== {job} =====\n" + s.getvalue(), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
