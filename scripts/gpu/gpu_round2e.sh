#!/bin/bash
# K27 fused linear+act, grouped similarity GPU, MLP micro-bench
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_nn.py tests/test_distance.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2e_tests.log 2>&1
timeout -k 10 300 python -u benchmarks/bench_kernels.py --only mlp > gpurun_out/r2e_mlp.log 2>&1
tail -3 gpurun_out/r2e_tests.log; cat gpurun_out/r2e_mlp.log
