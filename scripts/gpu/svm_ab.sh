# A/B: fused two-level selection on / off, plus kernel statistics of each at N = 8192
set -o pipefail
P=$GRAFT_REPO_ROOT/gpurun_out/prof
mkdir -p $P
timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768 ws > gpurun_out/ab_fused.log 2>&1 &&
AVMI_SMO_SELECT_FUSED=0 timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768 ws > gpurun_out/ab_unfused.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o ab_fused -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_svm.py 8192 ws > $GRAFT_REPO_ROOT/gpurun_out/ab_prof1.log 2>&1 &&
AVMI_SMO_SELECT_FUSED=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o ab_unfused -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_svm.py 8192 ws > $GRAFT_REPO_ROOT/gpurun_out/ab_prof2.log 2>&1
rc=$?
find $P -name "*kernel_trace.csv" -delete
find $P -name "*.db" -delete
exit $rc
