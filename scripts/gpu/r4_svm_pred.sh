set -o pipefail
# run a GPU step; stop the script on anything but pass (0) / test failures (1)
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 600 python -u -m pytest tests/test_svm_implicit.py tests/test_svm_ws.py tests/test_linear.py tests/test_rnn.py tests/test_tree.py tests/test_forest.py tests/test_optimize.py tests/test_native_predictors.py tests/test_native_explore_jobs.py tests/test_format_device.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4_svm_tests.log 2>&1
step timeout -k 10 600 python -u -m pytest tests/test_data_parallel_jobs.py tests/test_records.py tests/test_distance.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r4_pred_tests2.log 2>&1
step timeout -k 10 600 python -u benchmarks/bench_models.py --only rf,rf_ref > gpurun_out/r4_rf_bench.log 2>&1
step timeout -k 10 900 python -u benchmarks/bench_predict_jobs.py --records 16777216 --jobs vit,mmc,pst,nbp,detr,mop,usb,hash,dummy,rs --reps 2 --out gpurun_out/r4_predict_jobs_v2.jsonl > gpurun_out/r4_predict_bench2.log 2>&1
step timeout -k 10 600 python -u benchmarks/profile_predict_jobs.py --jobs vit,nbp --top 25 > gpurun_out/r4_profile_predict2.log 2>&1
