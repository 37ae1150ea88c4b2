# round-5 batch 14: kNN one threshold test per 16 candidates
set -o pipefail
mkdir -p gpurun_out/r5b14
export TMPDIR=/tmp
O=gpurun_out/r5b14
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_distance.py tests/test_native_predictors.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
cd /tmp
for t in knn16 knn64; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$t -o k -- python3 $R/benchmarks/pmc_targets.py $t > $R/$O/prof_$t.log 2>&1 || exit $?
done
find $R/$O/prof_* -name "*kernel_trace.csv" -delete
