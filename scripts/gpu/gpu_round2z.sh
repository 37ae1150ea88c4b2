#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_csv_device.py tests/test_wide.py tests/test_bayes.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2z_tests.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/r2z_bench.log 2>&1
tail -3 gpurun_out/r2z_tests.log; cat gpurun_out/r2z_bench.log
