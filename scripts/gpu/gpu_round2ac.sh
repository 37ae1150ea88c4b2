#!/bin/bash
# headline step without the blocking bins/offs read-back; K10 vote kernel and outlier GPU tests
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/r2ac
timeout -k 10 300 python3 -u -m pytest tests/test_distance.py tests/test_outlier.py tests/test_rowpack.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2ac/pytest.log 2>&1
timeout -k 10 300 python3 bench.py --ingest-rows 0 > gpurun_out/r2ac/bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2ac/prof -o run -- python3 bench.py --steps 10 --warmup 2 --ingest-rows 0 > gpurun_out/r2ac/bench_prof.log 2>&1
tail -3 gpurun_out/r2ac/pytest.log
grep '^{' gpurun_out/r2ac/bench.log | cut -c1-400
