#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_svm_ws.py tests/test_linear.py tests/test_forest.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2t_tests.log 2>&1
timeout -k 10 300 python -u benchmarks/bench_svm.py 8192,32768 ws > gpurun_out/r2t_svm.log 2>&1
timeout -k 10 300 python -u benchmarks/rf_phases.py > gpurun_out/r2t_rf.log 2>&1
timeout -k 10 900 python -u benchmarks/bench_vs_reference.py > gpurun_out/r2t_vsref.log 2>&1
tail -2 gpurun_out/r2t_tests.log; cat gpurun_out/r2t_svm.log gpurun_out/r2t_rf.log; grep '^{' gpurun_out/r2t_vsref.log
