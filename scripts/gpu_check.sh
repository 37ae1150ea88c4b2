#!/bin/bash
# One GPU validation pass: tests, smoke, bench, rocprof kernel stats.  Each GPU step has its own
# time limit; the script stops at the first failure.
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/pytest_gpu.log
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee gpurun_out/smoke.log
echo "== bench"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --predict 2>&1 | tee gpurun_out/bench.log
if [ "${PROFILE:-1}" = "1" ]; then
  echo "== rocprof"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 > gpurun_out/prof.log 2>&1
  find gpurun_out/prof -name "*kernel_stats.csv" | head -5
fi
echo "== done"
