# round-5 batch 5: pairs_within (packed math, 256-row workgroups), k-means v3 counters, SVM cache test at d=256
set -o pipefail
mkdir -p gpurun_out/r5b5
export TMPDIR=/tmp
O=gpurun_out/r5b5
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_distance.py tests/test_data_parallel_jobs.py tests/test_svm_large.py -m gpu -x -v --timeout 300 --timeout-method thread -k "pairs or similarity or Similarity or cache or kmeans" > $O/tests.log 2>&1 || exit $?
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_pairs -o p -- python3 $R/benchmarks/pmc_targets.py pairs > $R/$O/prof_pairs.log 2>&1 || exit $?
find $R/$O/prof_* -name "*kernel_trace.csv" -delete
cd $R
timeout -k 10 300 python -u benchmarks/bench_predict_jobs.py --jobs rs > $O/rs_bench.jsonl 2> $O/rs_bench.err || exit $?
PMC_OUT=$O/pmc PMC_TARGETS="kmeans pairs" timeout -k 10 600 bash scripts/gpu_pmc.sh > $O/pmc.log 2>&1
