# SVM kernel-row cache: tests and fit timings with / without the cache (d = 128, learnable problem)
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_svm_large.py -x -v -s --timeout 300 --timeout-method thread -m gpu -k cache > gpurun_out/r5/svm_cache_tests.log 2>&1 || exit $?
for c in 0 auto; do
  timeout -k 10 400 python -u benchmarks/bench_svm_implicit.py --sizes 16384,65536 --d 128 --gamma 0.01 --paths implicit --reps 2 --cache $c >> gpurun_out/r5/svm_cache_bench.jsonl 2>> gpurun_out/r5/svm_cache_bench.err || exit $?
done
