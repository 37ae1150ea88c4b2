# SVM solver, encoding and GBT checks on the box
set -o pipefail
P=$GRAFT_REPO_ROOT/gpurun_out/prof
mkdir -p $P
timeout -k 10 400 python -u -m pytest tests/test_linear.py tests/test_wide.py tests/test_encode_ops.py tests/test_tree.py -x -v --timeout 200 --timeout-method thread -m gpu -k "smo or svm or wide or huge or loo or gbt or node_histogram" > gpurun_out/s_tests.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/bench_svm.py 2048,8192,32768 ws > gpurun_out/s_svm.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/bench_models.py --only gbt > gpurun_out/s_gbt.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o svm2 -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_svm.py 8192 ws > $GRAFT_REPO_ROOT/gpurun_out/s_svmprof.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o gbt2 -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_models.py --only gbt > $GRAFT_REPO_ROOT/gpurun_out/s_gbtprof.log 2>&1
rc=$?
find $P -name "*kernel_trace.csv" -delete
find $P -name "*.db" -delete
exit $rc
