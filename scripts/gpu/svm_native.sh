# working-set SMO: native host loop vs graph replay, correctness tests first
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_svm_ws.py tests/test_linear.py tests/test_forest.py -x -q --timeout 150 --timeout-method thread -m gpu -k "smo or svm or rbf or native" > gpurun_out/n_tests.log 2>&1 &&
timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768 ws > gpurun_out/n_svm.log 2>&1 &&
AVMI_SMO_LOOP=graph timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768 ws > gpurun_out/n_svm_graph.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/bench_vs_reference.py --only svm --svm-rows 8192 > gpurun_out/n_vsref.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/bench_vs_reference.py --only svm --svm-rows 32768 >> gpurun_out/n_vsref.log 2>&1
