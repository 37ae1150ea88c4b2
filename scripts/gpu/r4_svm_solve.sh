# branch-free SMO loop + merge fused into the gather: tests, per-iteration cost, fits (A/B)
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest tests/test_svm_ws.py tests/test_svm_implicit.py tests/test_linear.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "svm or smo" > gpurun_out/r4_svm_solve_tests.log 2>&1
step timeout -k 10 200 python -u benchmarks/bench_smo_solve.py > gpurun_out/r4_smo_solve_call.log 2>&1
step timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768,8192,32768 ws > gpurun_out/r4_svm_solve.log 2>&1
echo "# AVMI_SMO_FUSED_GATHER=0" >> gpurun_out/r4_svm_solve.log
AVMI_SMO_FUSED_GATHER=0 step timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768,8192,32768 ws >> gpurun_out/r4_svm_solve.log 2>&1
step timeout -k 10 300 python -u benchmarks/bench_vs_reference.py --only svm --svm-rows 8192 > gpurun_out/r4_svm_vsref_solve.log 2>&1
