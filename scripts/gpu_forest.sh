#!/bin/bash
# Forest builder on the GPU: kernel/oracle tests, model bench (16.7M x 16, 10 trees, depth 8),
# sklearn comparison at 1M rows, kernel stats of the bench.
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_forest.py -x -v -m gpu --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/forest_tests.log
timeout -k 10 300 python -u benchmarks/bench_models.py --only rf 2>&1 | tee gpurun_out/forest_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_forest -o run --output-format csv -- python3 benchmarks/bench_models.py --only rf > gpurun_out/prof_forest.log 2>&1
timeout -k 10 400 python -u benchmarks/bench_vs_reference.py --only rf 2>&1 | tee gpurun_out/forest_vsref.log
