set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/tprof2 -o run --output-format csv -- python3 benchmarks/bench_ingest.py --formats tmc --jobs --reps 1 > gpurun_out/tmc_prof.log 2>&1
