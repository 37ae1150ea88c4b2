# round-5 batch 17: split-K linear_act_fwd + long-K gemm_tn slices; tests, shape bench, BERT bench, kernel-row benches
set -o pipefail
mkdir -p gpurun_out/r5b17
export TMPDIR=/tmp
O=gpurun_out/r5b17
timeout -k 10 400 python -u -m pytest tests/test_gemm.py tests/test_bert.py tests/test_nn.py tests/test_rnn.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python -u benchmarks/bench_gemm_shapes.py > $O/gemm_shapes.jsonl 2> $O/gemm_shapes.err || exit $?
timeout -k 10 300 python -u benchmarks/bench_bert.py > $O/bert_bench.jsonl 2> $O/bert_bench.err || exit $?
timeout -k 10 400 python -u benchmarks/bench_r5_kernels.py > $O/r5_kernels.jsonl 2> $O/r5_kernels.err || exit $?
