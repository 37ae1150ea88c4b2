set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/tprof -o run --output-format csv -- python3 benchmarks/bench_r3_kernels.py tfidf > gpurun_out/tfidf_prof.log 2>&1
