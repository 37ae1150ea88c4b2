#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_nn.py tests/test_nn_graphs.py tests/test_rnn.py tests/test_gemm.py > gpurun_out/rl_kc_tests.log 2>&1 || { tail -30 gpurun_out/rl_kc_tests.log; exit 1; }
tail -1 gpurun_out/rl_kc_tests.log
for k in 1 0 1 0; do
  AVMI_SBF16_SMALLK_KC64=$k timeout -k 10 300 python -u benchmarks/bench_rl_unsup.py dqn autoencoder > gpurun_out/rl_kc_$k.jsonl 2>&1 || exit 1
  echo "== kc64 $k"; grep 'graph' gpurun_out/rl_kc_$k.jsonl | cut -c1-160
done
