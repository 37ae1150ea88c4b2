#!/bin/bash
# LSTM kernel pass: gpu tests for the fused LSTM, then the fused-vs-MIOpen benchmark.
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rnn.py -x -v -m gpu --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/pytest_rnn.log
timeout -k 10 300 python -u benchmarks/bench_lstm.py ${LSTM_ARGS:-} 2>&1 | tee gpurun_out/bench_lstm.log
