#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_linear.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/svm_tests.log
timeout -k 10 300 python -u benchmarks/bench_svm.py 2048,8192,32768 full,ws 2>&1 | tee gpurun_out/svm_bench.jsonl
