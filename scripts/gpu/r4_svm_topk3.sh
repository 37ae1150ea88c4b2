# SVM top-k parts, one block per wave
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest tests/test_svm_ws.py tests/test_svm_implicit.py tests/test_linear.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "svm or smo" > gpurun_out/r4_svm_topk3_tests.log 2>&1
step timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768 ws > gpurun_out/r4_svm_topk3.log 2>&1
step timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768 ws >> gpurun_out/r4_svm_topk3.log 2>&1
step timeout -k 10 300 python -u benchmarks/bench_vs_reference.py --only svm --svm-rows 32768 > gpurun_out/r4_svm_vsref3.log 2>&1
step timeout -k 10 300 python -u benchmarks/bench_svm_implicit.py > gpurun_out/r4_svm_implicit3.log 2>&1
