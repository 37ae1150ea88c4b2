#!/bin/bash
# full GPU suite, kNN bench + counters, headline bench
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2j_tests.log 2>&1 || true
timeout -k 10 300 python -u benchmarks/bench_kernels.py --only knn,mlp > gpurun_out/r2j_kern.log 2>&1
PMC_TARGETS="knn16 knn64 knn256" bash scripts/gpu_pmc.sh > gpurun_out/r2j_pmc.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/r2j_bench.log 2>&1
tail -3 gpurun_out/r2j_tests.log; grep -E "FAILED|ERROR" gpurun_out/r2j_tests.log | head; cat gpurun_out/r2j_kern.log gpurun_out/r2j_bench.log
