#!/bin/bash
# Final-tree rehearsal of the round-end tiers + a kernel-trace profile of the 1-GPU bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/suite.log 2>&1 \
  || { tail -40 gpurun_out/suite.log; exit 1; }
tail -1 gpurun_out/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log | grep smoke
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/benchprof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 > gpurun_out/benchprof.log 2>&1 || exit 1
find gpurun_out/benchprof -name "*kernel_stats.csv" | head -1
