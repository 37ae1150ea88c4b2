#!/bin/bash
# Chunked long-sequence Viterbi on the GPU: tests, then sequential vs chunked timing.
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_viterbi_long.py tests/test_markov.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/viterbi_tests.log
timeout -k 10 400 python -u benchmarks/bench_viterbi_long.py 2>&1 | tee gpurun_out/viterbi_long.jsonl
