#!/bin/bash
# fused bootstrap + node assembly: forest tests, RF bench + kernel profile, bench.py with extras
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_forest.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2c_tests.log 2>&1
timeout -k 10 300 python -u benchmarks/bench_models.py --only rf > gpurun_out/r2c_forest_bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_forest2 -o run --output-format csv -- python3 benchmarks/bench_models.py --only rf > gpurun_out/prof_forest2.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/r2c_bench.log 2>&1
cat gpurun_out/r2c_forest_bench.log gpurun_out/r2c_bench.log
