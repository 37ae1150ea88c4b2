# round-5 batch 12: k-means branch-free prefetch
set -o pipefail
mkdir -p gpurun_out/r5b12
export TMPDIR=/tmp
O=gpurun_out/r5b12
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_distance.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
cd /tmp
for nb in 2 3; do
  AVMI_KMEANS_NBUF=$nb timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_km$nb -o km -- python3 $R/benchmarks/pmc_targets.py kmeans > $R/$O/prof_km$nb.log 2>&1 || exit $?
done
find $R/$O/prof_* -name "*kernel_trace.csv" -delete
