# top-k parts from 8193 rows: tests, timings
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest tests/test_svm_ws.py tests/test_svm_implicit.py tests/test_linear.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "svm or smo" > gpurun_out/r4_svm_mid2_tests.log 2>&1
step timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,12000,16384,32768 ws > gpurun_out/r4_svm_mid2.log 2>&1
step timeout -k 10 300 python -u benchmarks/bench_models.py --only svm >> gpurun_out/r4_svm_mid2.log 2>&1
