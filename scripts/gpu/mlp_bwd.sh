# K27 fused backward: nn tests + MLP kernel bench + kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_nn.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mlpb_tests.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/bench_kernels.py --only mlp > gpurun_out/mlpb_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mbprof -o run --output-format csv -- python3 benchmarks/bench_kernels.py --only mlp > gpurun_out/mlpb_prof.log 2>&1
