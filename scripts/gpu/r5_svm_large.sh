# large-N SVM: the streaming selection tests, the implicit suite, and fit timings at 2^18 / 2^19 rows
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_svm_large.py tests/test_svm_implicit.py tests/test_svm_ws.py -x -v -s --timeout 300 --timeout-method thread -m gpu > gpurun_out/r5/svm_large_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u benchmarks/bench_svm_implicit.py --sizes 262144,524288 --d 16 --paths implicit --reps 1 --sklearn-sub 16384 > gpurun_out/r5/svm_large_bench.jsonl 2>&1 || exit $?
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5/prof_svm262k_v2 -o s262k -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_svm_implicit.py --sizes 262144 --d 16 --paths implicit --reps 1 > $GRAFT_REPO_ROOT/gpurun_out/r5/svm262k_prof_v2.log 2>&1
rc=$?
find $GRAFT_REPO_ROOT/gpurun_out/r5/prof_svm262k_v2 -name "*kernel_trace.csv" -delete
exit $rc
