set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mprof -o run --output-format csv -- python3 benchmarks/bench_kernels.py --only mlp > gpurun_out/mlp_prof.log 2>&1
