#!/bin/bash
# replicated joint tables: correctness + bench at R = 1, 2, 4 + counters at the default
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rowpack.py tests/test_bayes.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2o_tests.log 2>&1
for r in 1 2 4; do
  echo "== R=$r" >> gpurun_out/r2o_bench.log
  AVMI_JOINT_REPLICAS=$r timeout -k 10 300 python -u bench.py --ingest-rows 0 >> gpurun_out/r2o_bench.log 2>&1
done
PMC_TARGETS="rowpack" bash scripts/gpu_pmc.sh > gpurun_out/r2o_pmc.log 2>&1
tail -2 gpurun_out/r2o_tests.log; cat gpurun_out/r2o_bench.log
