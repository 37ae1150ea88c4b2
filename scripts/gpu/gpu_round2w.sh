#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_svm2 -o run --output-format csv -- python3 benchmarks/bench_svm.py 8192 ws > gpurun_out/prof_svm2.log 2>&1
grep '^{' gpurun_out/prof_svm2.log
