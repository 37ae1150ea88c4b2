#!/bin/bash
# joint-table row-packed histogram: correctness, headline bench (joint vs nibble), counters
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rowpack.py tests/test_bayes.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2k_tests.log 2>&1
timeout -k 10 300 python -u bench.py --ingest-rows 0 > gpurun_out/r2k_bench_joint.log 2>&1
AVMI_ROWPACK_KERNEL=nibble timeout -k 10 300 python -u bench.py --ingest-rows 0 > gpurun_out/r2k_bench_nibble.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_joint -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --ingest-rows 0 > gpurun_out/prof_joint.log 2>&1
PMC_TARGETS="rowpack" bash scripts/gpu_pmc.sh > gpurun_out/r2k_pmc.log 2>&1
tail -3 gpurun_out/r2k_tests.log; cat gpurun_out/r2k_bench_joint.log gpurun_out/r2k_bench_nibble.log
