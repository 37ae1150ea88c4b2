#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_km -o run --output-format csv -- python3 benchmarks/bench_vs_reference.py --only kmeans > gpurun_out/prof_km.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gbt -o run --output-format csv -- python3 benchmarks/bench_vs_reference.py --only gbt > gpurun_out/prof_gbt.log 2>&1
grep '^{' gpurun_out/prof_km.log gpurun_out/prof_gbt.log
