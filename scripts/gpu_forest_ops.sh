#!/bin/bash
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/bench_forest_ops.py 2>&1 | tee gpurun_out/forest_ops.log
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE SQ_WAVES SQ_BUSY_CYCLES -d gpurun_out/pmc_forest -o run --output-format csv -- python3 benchmarks/bench_forest_ops.py --chunks 26000 > gpurun_out/pmc_forest.log 2>&1
