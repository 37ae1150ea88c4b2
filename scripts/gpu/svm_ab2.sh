# rank merge + 16-wave update: tests, timings, A/B against the radix merge, kernel statistics
set -o pipefail
P=$GRAFT_REPO_ROOT/gpurun_out/prof
mkdir -p $P
timeout -k 10 300 python -u -m pytest tests/test_svm_ws.py tests/test_linear.py -x -q --timeout 150 --timeout-method thread -m gpu -k "smo or svm or rbf or native or select" > gpurun_out/ab2_tests.log 2>&1 &&
timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768 ws > gpurun_out/ab2_rank.log 2>&1 &&
AVMI_SMO_RANK_MERGE=0 timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768 ws > gpurun_out/ab2_radix.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o ab2 -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_svm.py 8192 ws > $GRAFT_REPO_ROOT/gpurun_out/ab2_prof.log 2>&1
rc=$?
find $P -name "*kernel_trace.csv" -delete
find $P -name "*.db" -delete
exit $rc
