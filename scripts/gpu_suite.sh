#!/bin/bash
# Full GPU rehearsal of the round-end tiers: pytest -m gpu, smoke(), a 1-GPU bench.  Each step has
# its own time limit; the script stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/suite.log 2>&1 \
  || { tail -40 gpurun_out/suite.log; exit 1; }
tail -3 gpurun_out/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
