# SVM top-k parts gated to N > 16384; per = 2 vs 4 at N = 32768
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest tests/test_svm_ws.py tests/test_svm_implicit.py tests/test_linear.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "svm or smo" > gpurun_out/r4_svm_topk2_tests.log 2>&1
step timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768 ws > gpurun_out/r4_svm_topk2.log 2>&1
AVMI_SMO_TOPK_PER=4 step timeout -k 10 200 python -u benchmarks/bench_svm.py 32768 ws >> gpurun_out/r4_svm_topk2.log 2>&1
AVMI_SMO_TOPK_PER=1 step timeout -k 10 200 python -u benchmarks/bench_svm.py 32768 ws >> gpurun_out/r4_svm_topk2.log 2>&1
P=$GRAFT_REPO_ROOT/gpurun_out/prof_svm2
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o svm -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_svm.py 8192,32768 ws > $GRAFT_REPO_ROOT/gpurun_out/r4_svmprof2.log 2>&1
rc=$?
find $P -name "*kernel_trace.csv" -delete
find $P -name "*.db" -delete
exit $rc
