# GPU measurement batch (run on the box via gpurun): tests, benches, kernel-stat profiles (CSV only).
set -o pipefail
P=$GRAFT_REPO_ROOT/gpurun_out/prof
mkdir -p $P
timeout -k 10 300 python -u -m pytest tests/test_linear.py tests/test_forest.py tests/test_rnn.py tests/test_tree.py -x -v --timeout 200 --timeout-method thread -m gpu -k "smo or svm or forest_gpu or twenty or loss_curve or gbt" > gpurun_out/m_tests.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/bench_svm.py 2048,8192,32768 full,ws > gpurun_out/m_svm.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/bench_lstm.py --configs reference_ct,b8k_t16_h64 > gpurun_out/m_lstm.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o gbt -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_models.py --only gbt > $GRAFT_REPO_ROOT/gpurun_out/m_gbt.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o svm -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_svm.py 8192 ws > $GRAFT_REPO_ROOT/gpurun_out/m_svmprof.log 2>&1
rc=$?
find $P -name "*kernel_trace.csv" -delete
find $P -name "*.db" -delete
exit $rc
