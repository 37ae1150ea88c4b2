#!/bin/bash
# rocprofv3 kernel statistics of the fused-LSTM benchmark (fused implementation only).
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/lstmprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lstmprof -o run --output-format csv -- python3 benchmarks/bench_lstm.py --configs ${LSTM_CFG:-b64k_t32_h128} --impls fused --steps 5 --warmup 1 > gpurun_out/lstmprof/log.txt 2>&1
