"""cProfile of one exploration job at scale on the GPU (benchmarks/bench_explore_jobs_scale.py cases)."""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
import bench_explore_jobs_scale as B  # noqa: E402

case = sys.argv[1]
rows = sys.argv[2] if len(sys.argv) > 2 else str(1 << 21)
out = os.path.join(ROOT, "gpurun_out", f"prof_{case}.txt")
pr = cProfile.Profile()
pr.enable()
B.main_(["--rows", rows, "--device", "cuda", case])
pr.disable()
with open(out, "w") as fh:
    pstats.Stats(pr, stream=fh).sort_stats("cumulative").print_stats(40)
