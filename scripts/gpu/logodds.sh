set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_markov.py tests/test_jobs.py tests/test_world_sizes.py tests/test_pipelines.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/lo_tests.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/bench_more_kernels.py > gpurun_out/lo_bench.log 2>&1 &&
AVMI_LOGODDS_TILED=0 timeout -k 10 300 python -u benchmarks/bench_more_kernels.py > gpurun_out/lo_bench_off.log 2>&1
