# round-5 batch 15: data-parallel LSTM on the GPU, BERT kernels, BERT bench
set -o pipefail
mkdir -p gpurun_out/r5b15
export TMPDIR=/tmp
O=gpurun_out/r5b15
timeout -k 10 400 python -u -m pytest tests/test_lstm_data_parallel.py tests/test_bert.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 400 python -u benchmarks/bench_bert.py > $O/bert_bench.jsonl 2> $O/bert_bench.err || exit $?
