#!/bin/bash
# NB fit with the multi-GPU reduce on a side stream: ordering test (stub 2-rank comm), headline
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r2ad
timeout -k 10 300 python3 -u -m pytest tests/test_bayes.py tests/test_rowpack.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2ad/pytest.log 2>&1
timeout -k 10 300 python3 bench.py --ingest-rows 0 > gpurun_out/r2ad/bench.log 2>&1
tail -3 gpurun_out/r2ad/pytest.log
grep '^{' gpurun_out/r2ad/bench.log | cut -c1-300
