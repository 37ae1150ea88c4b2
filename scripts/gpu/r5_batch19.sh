# round-5 batch 19: BERT attention kernel + fused split-K LayerNorm
set -o pipefail
mkdir -p gpurun_out/r5b19
export TMPDIR=/tmp
O=gpurun_out/r5b19
timeout -k 10 400 python -u -m pytest tests/test_bert.py tests/test_gemm.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/bench_bert.py > $O/bert_bench.jsonl 2> $O/bert_bench.err || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_bert -o k -- python3 $GRAFT_REPO_ROOT/benchmarks/pmc_targets.py bert > $GRAFT_REPO_ROOT/$O/prof_bert.log 2>&1 || exit $?
find $GRAFT_REPO_ROOT/$O/prof_* -name "*kernel_trace.csv" -delete
