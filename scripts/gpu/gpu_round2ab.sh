#!/bin/bash
# kernel trace of the headline step: which launches sit between the histogram kernels
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r2ab
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2ab/prof -o run -- python3 bench.py --steps 10 --warmup 2 --ingest-rows 0 > gpurun_out/r2ab/bench.log 2>&1
timeout -k 10 300 python3 -m pytest tests/test_outlier.py -m gpu -x -q --timeout 120 > gpurun_out/r2ab/pytest.log 2>&1
find gpurun_out/r2ab/prof -name '*kernel_stats.csv' -exec head -20 {} \;
tail -2 gpurun_out/r2ab/bench.log | cut -c1-300
