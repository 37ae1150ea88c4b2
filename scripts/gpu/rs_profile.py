"""Host-side phase profile of the recordSimilarity job (cProfile, 3 runs after a warm-up)."""
import cProfile
import os
import pstats
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "benchmarks"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import bench_predict_jobs as B  # noqa: E402
from avenir_amd.cli import main  # noqa: E402

d = tempfile.mkdtemp(prefix="avmi_rsprof_")
argv, data = B.setup_rs(d, 1 << 17)
for rep in range(2):
    out = os.path.join(d, f"w{rep}.out")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    main(argv + ["-o", out, "--device", "cuda"])
    torch.cuda.synchronize()
    print("warm run", rep, round(time.perf_counter() - t0, 4), flush=True)
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
for rep in range(3):
    main(argv + ["-o", os.path.join(d, f"p{rep}.out"), "--device", "cuda"])
torch.cuda.synchronize()
pr.disable()
print("3 profiled runs", round(time.perf_counter() - t0, 4), flush=True)
pstats.Stats(pr).sort_stats("cumulative").print_stats(35)
