# top-k parts with HW = 4 keys per wave: tests, sizes, and 8192 with the top-k parts
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest tests/test_svm_ws.py tests/test_svm_implicit.py tests/test_linear.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "svm or smo" > gpurun_out/r4_svm_hw_tests.log 2>&1
O=gpurun_out/r4_svm_hw.log
step timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,12000,16384,32768,8192,12000,16384,32768 ws > $O 2>&1
echo "# top-k parts at 8192 (AVMI_SMO_TOPK_MIN_N=4097)" >> $O
AVMI_SMO_TOPK_MIN_N=4097 step timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,8192,8192 ws >> $O 2>&1
