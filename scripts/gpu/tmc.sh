set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_native_jobs.py tests/test_records.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tmc_tests.log 2>&1 &&
timeout -k 10 400 python -u benchmarks/bench_ingest.py --formats tmc,nen --jobs --out gpurun_out/tmc_jobs.jsonl > gpurun_out/tmc_jobs.log 2>&1
