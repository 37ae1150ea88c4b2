# rocprofv3 kernel + memory-copy trace of the K1 upload (one setting, 2 loads)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/uprof -o run --output-format csv -- python3 benchmarks/bench_upload.py --reps 1 --settings pread:16:2 > gpurun_out/upload_prof.log 2>&1
