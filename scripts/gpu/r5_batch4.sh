# round-5 batch 4: LSTM (in-kernel projection, one dW GEMM), k-means three-tile rotation,
# pairs_within prefilter, SVM row cache at wide rows
set -o pipefail
mkdir -p gpurun_out/r5b4
export TMPDIR=/tmp
O=gpurun_out/r5b4
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_rnn.py tests/test_distance.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/bench_lstm.py --configs reference_ct --impls fused,fused_graph,miopen,miopen_graph --steps 30 > $O/lstm_bench.jsonl 2> $O/lstm_bench.err || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_lstm -o l -- python3 $R/benchmarks/bench_lstm.py --configs reference_ct --impls fused --steps 20 > $R/$O/prof_lstm.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_km -o km -- python3 $R/benchmarks/pmc_targets.py kmeans > $R/$O/prof_km.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_pairs -o p -- python3 $R/benchmarks/pmc_targets.py pairs > $R/$O/prof_pairs.log 2>&1 || exit $?
find $R/$O/prof_* -name "*kernel_trace.csv" -delete
cd $R
timeout -k 10 300 python -u benchmarks/bench_predict_jobs.py --jobs rs > $O/rs_bench.jsonl 2> $O/rs_bench.err || exit $?
for c in 0 auto; do
  timeout -k 10 300 python -u benchmarks/bench_svm_implicit.py --sizes 16384 --d 512 --gamma 0.002 --paths implicit --reps 2 --cache $c >> $O/svm_wide.jsonl 2>> $O/svm_wide.err || exit $?
done
