#!/bin/bash
# kNN prefetch restructure, LDS binary-forest predict
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_distance.py tests/test_forest.py tests/test_tree.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2g_tests.log 2>&1
timeout -k 10 300 python -u benchmarks/bench_kernels.py --only knn > gpurun_out/r2g_knn.log 2>&1
timeout -k 10 300 python -u benchmarks/bench_models.py --only rf > gpurun_out/r2g_rf.log 2>&1
PMC_TARGETS="knn16 knn64 knn256" bash scripts/gpu_pmc.sh > gpurun_out/r2g_pmc.log 2>&1
tail -3 gpurun_out/r2g_tests.log; cat gpurun_out/r2g_knn.log gpurun_out/r2g_rf.log
