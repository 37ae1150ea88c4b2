#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_nn.py tests/test_nn_graphs.py tests/test_rnn.py > gpurun_out/rl_ab_tests.log 2>&1 || { tail -30 gpurun_out/rl_ab_tests.log; exit 1; }
tail -1 gpurun_out/rl_ab_tests.log
for m in 64; do
  AVMI_FUSED_BWD_MAX=$m timeout -k 10 300 python -u benchmarks/bench_rl_unsup.py > gpurun_out/rl_ab_$m.jsonl 2>&1 || exit 1
  echo "== fused bwd max $m"; grep '"us_per' gpurun_out/rl_ab_$m.jsonl | cut -c1-200
done
AVMI_FUSED_BWD_MAX=512 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/dqnprof2 -o trace --output-format csv -- python3 benchmarks/pmc_targets.py dqn > gpurun_out/dqnprof2.log 2>&1 || exit 1
