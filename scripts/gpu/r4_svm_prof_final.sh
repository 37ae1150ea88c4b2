# kernel stats of the final SMO step at N = 8192 and 32768
set -o pipefail
P=$GRAFT_REPO_ROOT/gpurun_out/prof_svm_final
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o s8k -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_svm.py 8192 ws > $GRAFT_REPO_ROOT/gpurun_out/r4_svmprof_final.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o s32k -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_svm.py 32768 ws >> $GRAFT_REPO_ROOT/gpurun_out/r4_svmprof_final.log 2>&1
rc=$?
find $P -name "*kernel_trace.csv" -delete
find $P -name "*.db" -delete
exit $rc
