# K1 LDS-staged parse: device CSV tests, upload bench, bench ingest, kernel trace of the loads
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_csv_device.py tests/test_records.py tests/test_native_jobs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/csvp_tests.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/bench_upload.py --settings pread:16:2,pread:16:1 --reps 3 > gpurun_out/csvp_upload.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cprof -o run --output-format csv -- python3 benchmarks/bench_upload.py --settings pread:16:2 --reps 1 > gpurun_out/csvp_prof.log 2>&1
