# working-set SMO kernel stats at N = 32768 (dense) and the fit times at 8192 / 32768
set -o pipefail
P=$GRAFT_REPO_ROOT/gpurun_out/prof_svm
mkdir -p $P
timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768 ws > gpurun_out/r4_svm_times.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o svm32k -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_svm.py 32768 ws > $GRAFT_REPO_ROOT/gpurun_out/r4_svmprof.log 2>&1
rc=$?
find $P -name "*kernel_trace.csv" -delete
find $P -name "*.db" -delete
exit $rc
