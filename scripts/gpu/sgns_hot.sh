# SGNS with hot-row replicas: text tests + word2vec epoch benchmark
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_text.py tests/test_text_jobs.py -x -q --timeout 150 --timeout-method thread -m gpu > gpurun_out/sh_tests.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/bench_r3_kernels.py sgns > gpurun_out/sh_bench.log 2>&1
