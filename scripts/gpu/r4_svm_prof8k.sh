# kernel stats at N = 8192: radix parts (default) and top-k parts with HP = 8
set -o pipefail
P=$GRAFT_REPO_ROOT/gpurun_out/prof_svm8k
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o radix -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_svm.py 8192 ws > $GRAFT_REPO_ROOT/gpurun_out/r4_svmprof8k.log 2>&1 || exit $?
export AVMI_SMO_TOPK_MIN_N=4097 AVMI_SMO_TOPK_HP=8
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o topk8 -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_svm.py 8192 ws >> $GRAFT_REPO_ROOT/gpurun_out/r4_svmprof8k.log 2>&1
rc=$?
find $P -name "*kernel_trace.csv" -delete
find $P -name "*.db" -delete
exit $rc
