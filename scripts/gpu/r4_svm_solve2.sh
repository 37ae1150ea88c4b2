# permlane-swap wave maxima in the SMO loop; N = 8192 sweep (rel_tol, top-k parts)
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest tests/test_svm_ws.py tests/test_svm_implicit.py tests/test_linear.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "svm or smo" > gpurun_out/r4_svm_solve2_tests.log 2>&1
step timeout -k 10 200 python -u benchmarks/bench_smo_solve.py > gpurun_out/r4_smo_solve_call2.log 2>&1
step timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768,8192,32768 ws > gpurun_out/r4_svm_solve2.log 2>&1
step bash scripts/gpu/r4_svm_sweep8k.sh
