# working-set SMO kernel timeline at N = 8192: busy vs idle time between kernels
set -o pipefail
P=$GRAFT_REPO_ROOT/gpurun_out/prof
mkdir -p $P
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $P -o svmgap -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_svm.py 8192 ws > $GRAFT_REPO_ROOT/gpurun_out/gap_run.log 2>&1
rc=$?
f=$(find $P -name "svmgap*kernel_trace.csv" | head -1)
[ $rc -eq 0 ] && python3 $GRAFT_REPO_ROOT/tools/trace_gaps.py "$f" --from select_part --skip 20 --to smo_ws_update > $GRAFT_REPO_ROOT/gpurun_out/svm_gaps.txt 2>&1
rc=$?
find $P -name "*kernel_trace.csv" -delete
find $P -name "*.db" -delete
exit $rc
