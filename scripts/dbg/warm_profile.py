"""Run a benchmarks/bench_*_scale.py script with cProfile enabled for the WARM (second) call of
each job only: python scripts/dbg/warm_profile.py OUTDIR benchmarks/bench_x.py [args...]."""
import cProfile
import os
import runpy
import sys

out_dir, script, rest = sys.argv[1], sys.argv[2], sys.argv[3:]
os.makedirs(out_dir, exist_ok=True)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import avenir_amd.cli as cli  # noqa: E402

_orig = cli.main
_seen = {}


def main(argv=None):
    job = (argv or ["?"])[0]
    _seen[job] = _seen.get(job, 0) + 1
    if _seen[job] != 2:
        return _orig(argv)
    pr = cProfile.Profile()
    pr.enable()
    try:
        return _orig(argv)
    finally:
        pr.disable()
        pr.dump_stats(os.path.join(out_dir, f"warm_{job}.prof"))


cli.main = main
sys.argv = [script] + rest
runpy.run_path(script, run_name="__main__")
