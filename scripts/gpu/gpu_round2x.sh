#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_svm_ws.py tests/test_linear.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2x_tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_svm3 -o run --output-format csv -- python3 benchmarks/bench_svm.py 8192 ws > gpurun_out/prof_svm3.log 2>&1
tail -2 gpurun_out/r2x_tests.log; grep '^{' gpurun_out/prof_svm3.log
