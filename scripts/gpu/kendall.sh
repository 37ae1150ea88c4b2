# K26 Kendall merge-path inversion kernels: tests + kernel bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_stats_ops.py tests/test_analytics.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/kendall_tests.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/bench_r3_kernels.py ranks > gpurun_out/kendall_bench.log 2>&1
