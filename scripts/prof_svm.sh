#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
cd gpurun_out && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d prof_svm -o run -- python3 ../benchmarks/bench_svm.py 8192 ws > prof_svm.log 2>&1
tail -3 prof_svm.log
