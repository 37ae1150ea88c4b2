#!/bin/bash
# full GPU suite + smoke + headline bench on the current tree
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2y_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r2y_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; tail -5 gpurun_out/r2y_tests.log; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2y_smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/r2y_bench.log 2>&1 || exit $?
tail -3 gpurun_out/r2y_tests.log; grep -E "FAILED|ERROR" gpurun_out/r2y_tests.log | head -20 || true; tail -2 gpurun_out/r2y_smoke.log; cat gpurun_out/r2y_bench.log
