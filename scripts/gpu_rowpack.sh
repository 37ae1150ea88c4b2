#!/bin/bash
# Row-packed NB path on the GPU: numerics tests, bench in both layouts, kernel profile.
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rowpack.py tests/test_bayes.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/rowpack_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 2>&1 | tee gpurun_out/bench_rowpacked.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --layout columns 2>&1 | tee gpurun_out/bench_columns.log
cd gpurun_out && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d prof_rowpack -o run -- python3 ../bench.py --steps 10 --warmup 2 > prof_rowpack.log 2>&1
