#!/bin/bash
# Quick GPU pass: gpu tests + kernel micro-benchmarks + bench.
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/pytest_gpu.log
timeout -k 10 300 python benchmarks/bench_kernels.py ${KB_ARGS:-} 2>&1 | tee gpurun_out/kernels.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 2>&1 | tee gpurun_out/bench.log
