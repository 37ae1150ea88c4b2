#!/bin/bash
# dense B-bit record stream for the joint-table histogram
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rowpack.py tests/test_bayes.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2m_tests.log 2>&1
timeout -k 10 300 python -u bench.py --ingest-rows 0 > gpurun_out/r2m_bench_dense.log 2>&1
AVMI_ROWPACK_KERNEL=joint timeout -k 10 300 python -u bench.py --ingest-rows 0 > gpurun_out/r2m_bench_joint.log 2>&1
PMC_TARGETS="rowpack" bash scripts/gpu_pmc.sh > gpurun_out/r2m_pmc.log 2>&1
tail -3 gpurun_out/r2m_tests.log; cat gpurun_out/r2m_bench_dense.log gpurun_out/r2m_bench_joint.log
