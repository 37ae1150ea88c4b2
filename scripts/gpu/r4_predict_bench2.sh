set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_native_predictors.py tests/test_data_parallel_jobs.py tests/test_records.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_pred_tests2.log 2>&1 &&
timeout -k 10 900 python -u benchmarks/bench_predict_jobs.py --records 16777216 --reps 2 --out gpurun_out/r4_predict_jobs_v2.jsonl > gpurun_out/r4_predict_bench2.log 2>&1 &&
timeout -k 10 600 python -u benchmarks/profile_predict_jobs.py --jobs vit,nbp --top 25 > gpurun_out/r4_profile_predict2.log 2>&1
