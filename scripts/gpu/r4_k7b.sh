# reference-semantics forest with per-tree row ranges in node_hist
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest tests/test_tree.py tests/test_forest.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_k7b_tests.log 2>&1
step timeout -k 10 300 python -u benchmarks/bench_models.py --only rf,rf_ref > gpurun_out/r4_k7b_bench.log 2>&1
step timeout -k 10 300 python -u benchmarks/bench_models.py --only rf_ref >> gpurun_out/r4_k7b_bench.log 2>&1
step timeout -k 10 300 python -u -m pytest tests/test_format_device.py tests/test_native_predictors.py tests/test_native_explore_jobs.py tests/test_data_parallel_jobs.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_fmt_tests.log 2>&1
export AVMI_FORMAT_TIMING=1
step timeout -k 10 400 python -u benchmarks/bench_predict_jobs.py --records 16777216 --jobs vit,mmc,mop,usb,detr,nbp --reps 2 --out gpurun_out/r4_predict_mmc.jsonl > gpurun_out/r4_predict_mmc.log 2>&1
step timeout -k 10 600 python -u benchmarks/profile_predict_jobs.py --jobs mop,usb,pst,detr,hash --top 40 > gpurun_out/r4_profile_predict3.log 2>&1
