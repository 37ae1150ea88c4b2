# k-means MFMA scoring: tests, A/B kernel traces (score vs packed-FMA kernel), PMC pass, sklearn SSE parity
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_distance.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r5/kmeans_tests.log 2>&1 || exit $?
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5/prof_km_score -o km -- python3 $R/benchmarks/pmc_targets.py kmeans > $R/gpurun_out/r5/prof_km_score.log 2>&1 || exit $?
AVMI_KMEANS_SCORE=valu timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5/prof_km_valu -o km -- python3 $R/benchmarks/pmc_targets.py kmeans > $R/gpurun_out/r5/prof_km_valu.log 2>&1 || exit $?
find $R/gpurun_out/r5/prof_km_* -name "*kernel_trace.csv" -delete
cd $R
PMC_OUT=gpurun_out/r5/pmc_score PMC_TARGETS=kmeans timeout -k 10 400 bash scripts/gpu_pmc.sh > gpurun_out/r5/pmc_score.log 2>&1 || exit $?
timeout -k 10 600 python -u benchmarks/bench_vs_reference.py --only kmeans > gpurun_out/r5/kmeans_vsref.log 2>&1
