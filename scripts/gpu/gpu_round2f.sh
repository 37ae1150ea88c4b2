#!/bin/bash
# kNN norms-from-LDS, prefetching fused linear, vs-reference refresh
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_nn.py tests/test_distance.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2f_tests.log 2>&1
timeout -k 10 300 python -u benchmarks/bench_kernels.py --only knn,mlp > gpurun_out/r2f_kern.log 2>&1
PMC_TARGETS="knn16 knn256" bash scripts/gpu_pmc.sh > gpurun_out/r2f_pmc.log 2>&1
timeout -k 10 900 python -u benchmarks/bench_vs_reference.py > gpurun_out/r2f_vsref.log 2>&1
tail -3 gpurun_out/r2f_tests.log; cat gpurun_out/r2f_kern.log; grep '^{' gpurun_out/r2f_vsref.log
