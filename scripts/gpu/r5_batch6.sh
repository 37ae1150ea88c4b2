# round-5 batch 6: pairs_within with per-workgroup LDS lists + segmented counters
set -o pipefail
mkdir -p gpurun_out/r5b6
export TMPDIR=/tmp
O=gpurun_out/r5b6
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_distance.py tests/test_data_parallel_jobs.py -m gpu -x -v --timeout 300 --timeout-method thread -k "pairs or similarity or Similarity" > $O/tests.log 2>&1 || exit $?
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_pairs -o p -- python3 $R/benchmarks/pmc_targets.py pairs > $R/$O/prof_pairs.log 2>&1 || exit $?
find $R/$O/prof_* -name "*kernel_trace.csv" -delete
cd $R
timeout -k 10 300 python -u benchmarks/bench_predict_jobs.py --jobs rs > $O/rs_bench.jsonl 2> $O/rs_bench.err || exit $?
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_rs -o rs -- python3 $R/benchmarks/bench_predict_jobs.py --jobs rs --reps 1 > $R/$O/prof_rs.log 2>&1 || exit $?
find $R/$O/prof_* -name "*kernel_trace.csv" -delete
