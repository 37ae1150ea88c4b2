# round-5 batch 22: fused optimisers for the NN estimators (A/B by AVMI_FUSED_OPT)
set -o pipefail
mkdir -p gpurun_out/r5b22
export TMPDIR=/tmp
O=gpurun_out/r5b22
timeout -k 10 100 python -u scripts/diag/fused_adam_eager.py > $O/diag.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_nn.py tests/test_rnn.py tests/test_lstm_data_parallel.py tests/test_gemm.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
AVMI_FUSED_OPT=0 timeout -k 10 300 python -u benchmarks/bench_lstm_network.py > $O/lstm_net_foreach.jsonl 2> $O/a.err || exit $?
AVMI_FUSED_OPT=1 timeout -k 10 300 python -u benchmarks/bench_lstm_network.py > $O/lstm_net_fused.jsonl 2> $O/b.err || exit $?
