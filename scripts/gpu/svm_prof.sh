# working-set SMO: timings and a kernel-stat profile at N = 32768
set -o pipefail
P=$GRAFT_REPO_ROOT/gpurun_out/prof
mkdir -p $P
timeout -k 10 300 python -u -m pytest tests/test_linear.py tests/test_forest.py -x -q --timeout 150 --timeout-method thread -m gpu -k "smo or svm or forest" > gpurun_out/p_tests.log 2>&1 &&
timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768 ws > gpurun_out/p_svm.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o svm8k -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_svm.py 8192 ws > $GRAFT_REPO_ROOT/gpurun_out/p_svmprof.log 2>&1
rc=$?
[ $rc -eq 0 ] && cd $GRAFT_REPO_ROOT && timeout -k 10 300 python -u benchmarks/bench_vs_reference.py --only svm --svm-rows 8192 > gpurun_out/p_vsref.log 2>&1 && timeout -k 10 300 python -u benchmarks/bench_vs_reference.py --only svm --svm-rows 32768 >> gpurun_out/p_vsref.log 2>&1
rc=$?
find $P -name "*kernel_trace.csv" -delete
find $P -name "*.db" -delete
exit $rc
