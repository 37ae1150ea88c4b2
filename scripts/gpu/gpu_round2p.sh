#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_distance.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2p_tests.log 2>&1
timeout -k 10 300 python -u benchmarks/bench_kernels.py --only knn > gpurun_out/r2p_knn.log 2>&1
PMC_TARGETS="knn16 knn64 knn256" bash scripts/gpu_pmc.sh > gpurun_out/r2p_pmc.log 2>&1
tail -2 gpurun_out/r2p_tests.log; cat gpurun_out/r2p_knn.log
