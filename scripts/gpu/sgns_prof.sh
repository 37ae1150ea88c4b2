# SGNS kernel statistics (word2vec epoch of bench_r3_kernels.py)
set -o pipefail
P=$GRAFT_REPO_ROOT/gpurun_out/prof
mkdir -p $P
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o sgns -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_r3_kernels.py sgns > $GRAFT_REPO_ROOT/gpurun_out/sgns_prof.log 2>&1
rc=$?
find $P -name "*kernel_trace.csv" -delete
find $P -name "*.db" -delete
exit $rc
