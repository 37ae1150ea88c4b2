#!/bin/bash
# kNN metric kernels + ingest path + PMC passes
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_distance.py tests/test_forest.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2d_tests.log 2>&1
timeout -k 10 300 python -u benchmarks/bench_kernels.py --only knn > gpurun_out/r2d_knn.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/r2d_bench.log 2>&1
bash scripts/gpu_pmc.sh > gpurun_out/r2d_pmc.log 2>&1
tail -3 gpurun_out/r2d_tests.log; cat gpurun_out/r2d_knn.log gpurun_out/r2d_bench.log
