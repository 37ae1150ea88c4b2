# SVM kernel-row cache: tests and fit timings with / without the cache at D = 16 and 128
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_svm_large.py tests/test_svm_implicit.py -x -v -s --timeout 300 --timeout-method thread -m gpu > gpurun_out/r5/svm_cache_tests.log 2>&1 || exit $?
for c in 0 4096; do
  timeout -k 10 400 python -u benchmarks/bench_svm_implicit.py --sizes 65536,262144 --d 128 --paths implicit --reps 1 --cache $c >> gpurun_out/r5/svm_cache_bench.jsonl 2>> gpurun_out/r5/svm_cache_bench.err || exit $?
  timeout -k 10 400 python -u benchmarks/bench_svm_implicit.py --sizes 262144 --d 16 --paths implicit --reps 1 --cache $c >> gpurun_out/r5/svm_cache_bench.jsonl 2>> gpurun_out/r5/svm_cache_bench.err || exit $?
done
