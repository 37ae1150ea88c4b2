#!/bin/bash
# forest kernels + SVM determinism + bench; each GPU step bounded
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_forest.py tests/test_svm_ws.py tests/test_gpu_jobs.py -x -v -m gpu --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/r2b_tests.log
timeout -k 10 300 python -u benchmarks/bench_forest_ops.py 2>&1 | tee gpurun_out/forest_ops.log
timeout -k 10 300 python -u benchmarks/bench_models.py --only rf 2>&1 | tee gpurun_out/forest_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_forest -o run --output-format csv -- python3 benchmarks/bench_models.py --only rf > gpurun_out/prof_forest.log 2>&1
