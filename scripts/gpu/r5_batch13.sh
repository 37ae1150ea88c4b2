# round-5 batch 13: BERT encoder kernels + bench; k-means uniform loop
set -o pipefail
mkdir -p gpurun_out/r5b13
export TMPDIR=/tmp
O=gpurun_out/r5b13
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_bert.py tests/test_distance.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 400 python -u benchmarks/bench_bert.py > $O/bert_bench.jsonl 2> $O/bert_bench.err || exit $?
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_km -o km -- python3 $R/benchmarks/pmc_targets.py kmeans > $R/$O/prof_km.log 2>&1 || exit $?
find $R/$O/prof_* -name "*kernel_trace.csv" -delete
