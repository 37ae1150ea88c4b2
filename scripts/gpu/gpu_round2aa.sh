#!/bin/bash
# refresh every kernel micro-benchmark and model throughput for profiles/
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u benchmarks/bench_kernels.py > gpurun_out/r2aa_kernels.log 2>&1
timeout -k 10 600 python -u benchmarks/bench_models.py > gpurun_out/r2aa_models.log 2>&1
grep '^{' gpurun_out/r2aa_kernels.log gpurun_out/r2aa_models.log | cut -c1-250
