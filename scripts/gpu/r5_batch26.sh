# round-5 batch 26: batched corpus encoding for semantic search
set -o pipefail
mkdir -p gpurun_out/r5b26
export TMPDIR=/tmp
O=gpurun_out/r5b26
timeout -k 10 400 python -u -m pytest tests/test_bert.py tests/test_gemm.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 500 python -u benchmarks/bench_bert.py > $O/bert_bench.jsonl 2> $O/bert_bench.err || exit $?
