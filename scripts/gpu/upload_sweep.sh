# K1 device-CSV upload sweep (pread / mmap x host threads) + device CSV tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_csv_device.py tests/test_records.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/upload_tests.log 2>&1 &&
timeout -k 10 400 python -u benchmarks/bench_upload.py --settings pread:8:1,pread:8:2,pread:16:1,pread:16:2,mmap:8:2 --out gpurun_out/upload_sweep.jsonl > gpurun_out/upload_sweep.log 2>&1
