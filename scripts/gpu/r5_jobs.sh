# recordSimilarity diagonal skip + featureCondProbJoiner end to end + tie-aware kNN GPU tests
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_data_parallel_jobs.py tests/test_native_predictors.py tests/test_cond_prob_joiner.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r5/jobs_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u benchmarks/bench_predict_jobs.py --jobs rs,fcb --records 16777216 --rs-records 131072 --reps 3 --dir /tmp > gpurun_out/r5/jobs_bench.jsonl 2> gpurun_out/r5/jobs_bench.err || exit $?
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5/prof_rs -o rs -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_predict_jobs.py --jobs rs --rs-records 131072 --reps 2 --dir /tmp > $GRAFT_REPO_ROOT/gpurun_out/r5/prof_rs.log 2>&1
rc=$?
find $GRAFT_REPO_ROOT/gpurun_out/r5/prof_rs -name "*kernel_trace.csv" -delete
exit $rc
