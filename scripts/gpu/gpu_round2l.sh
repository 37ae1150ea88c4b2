#!/bin/bash
# joint kernel with bank-spreading slot map
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rowpack.py tests/test_bayes.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2l_tests.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/r2l_bench.log 2>&1
PMC_TARGETS="rowpack" bash scripts/gpu_pmc.sh > gpurun_out/r2l_pmc.log 2>&1
tail -3 gpurun_out/r2l_tests.log; cat gpurun_out/r2l_bench.log
