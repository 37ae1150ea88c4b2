# mixed kNN rewrite + Kendall merge count: tests then the kernel benchmark sections
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_distance.py tests/test_stats_ops.py tests/test_jobs.py -x -q --timeout 150 --timeout-method thread -m gpu > gpurun_out/r3k2_tests.log 2>&1 &&
timeout -k 10 400 python -u benchmarks/bench_r3_kernels.py ranks,mixed_knn > gpurun_out/r3k2.log 2>&1
