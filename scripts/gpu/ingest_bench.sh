# device CSV tests + 1-GPU bench (headline + ingest with first/warm loads)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_csv_device.py tests/test_records.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ingest_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/ingest_bench.log 2>&1
