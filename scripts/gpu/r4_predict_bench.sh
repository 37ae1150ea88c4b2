# round 4: full GPU suite, then the prediction / sequence jobs end to end at 2^24 records
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gpu_tests.log 2>&1 &&
timeout -k 10 900 python -u benchmarks/bench_predict_jobs.py --records 16777216 --reps 2 --out gpurun_out/r4_predict_jobs.jsonl > gpurun_out/r4_predict_bench.log 2>&1
