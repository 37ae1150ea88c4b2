# round 4: the GPU tests touched by the native job I/O work (no -x: every failure in one call)
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_markov.py tests/test_native_predictors.py tests/test_csv_device.py tests/test_records.py tests/test_native_jobs.py tests/test_cli.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r4_subset.log 2>&1
