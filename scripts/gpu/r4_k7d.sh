# repr formatter test, forest timings (3 reps), SVM rank merge A/B at N = 32768
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 300 python -u -m pytest tests/test_format_device.py tests/test_svm_ws.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_k7d_tests.log 2>&1
step timeout -k 10 300 python -u benchmarks/bench_models.py --only rf,rf_ref > gpurun_out/r4_k7d_bench.log 2>&1
step timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768 ws > gpurun_out/r4_svm_ab.log 2>&1
export AVMI_SMO_RANK_MERGE_MAX=512
step timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768 ws >> gpurun_out/r4_svm_ab.log 2>&1
step timeout -k 10 300 python -u -m pytest tests/test_svm_ws.py tests/test_svm_implicit.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_k7d_tests512.log 2>&1
