# ingest refresh after the upload changes: record tests, bench.py, text-layout tokenize + job rates
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_csv_device.py tests/test_records.py tests/test_native_jobs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ir_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/ir_bench.log 2>&1 &&
timeout -k 10 600 python -u benchmarks/bench_ingest.py --jobs --out gpurun_out/ir_ingest.jsonl > gpurun_out/ir_ingest.log 2>&1
