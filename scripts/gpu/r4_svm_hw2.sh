# top-k parts the default from 4097 rows: tests, sizes, reference comparison at 8192
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest tests/test_svm_ws.py tests/test_svm_implicit.py tests/test_linear.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "svm or smo or ovr" > gpurun_out/r4_svm_hw2_tests.log 2>&1
step timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,12000,16384,32768,8192 ws > gpurun_out/r4_svm_hw2.log 2>&1
step timeout -k 10 300 python -u benchmarks/bench_vs_reference.py --only svm --svm-rows 8192 >> gpurun_out/r4_svm_hw2.log 2>&1
step timeout -k 10 300 python -u benchmarks/bench_vs_reference.py --only svm --svm-rows 32768 >> gpurun_out/r4_svm_hw2.log 2>&1
