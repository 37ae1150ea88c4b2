# working-set SMO: tests + sub-problem tolerance sweep
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_linear.py -x -q --timeout 150 --timeout-method thread -m gpu -k "smo or svm" > gpurun_out/w_tests.log 2>&1 &&
for t in 0.3 0.4; do
  AVMI_SMO_REL_TOL=$t timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768 ws > gpurun_out/w_svm_$t.log 2>&1 || exit $?
done
