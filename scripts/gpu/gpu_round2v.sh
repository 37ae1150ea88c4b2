#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_distance.py tests/test_tree.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2v_tests.log 2>&1
timeout -k 10 600 python -u benchmarks/bench_vs_reference.py --only kmeans,gbt > gpurun_out/r2v_vsref.log 2>&1
tail -2 gpurun_out/r2v_tests.log; grep '^{' gpurun_out/r2v_vsref.log
