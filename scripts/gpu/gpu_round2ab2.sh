#!/bin/bash
# K23/K26 encode.hip: GPU tests, micro-benchmark, per-kernel stats
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_encode_ops.py tests/test_wide.py tests/test_analytics.py -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/enc_tests.log 2>&1
rc=$?; tail -15 gpurun_out/enc_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/bench_encode.py > gpurun_out/enc_bench.log 2>&1 || exit $?
cat gpurun_out/enc_bench.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/enc_prof -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_encode.py > $GRAFT_REPO_ROOT/gpurun_out/enc_prof.log 2>&1 || exit $?
find $GRAFT_REPO_ROOT/gpurun_out/enc_prof -name "*kernel_stats.csv" | head -1 | xargs cut -c1-200 | head -20
