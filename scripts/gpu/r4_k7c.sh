# K7 forest host-side vectorisation, repr formatter test, predict jobs v5
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest tests/test_tree.py tests/test_forest.py tests/test_format_device.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_k7c_tests.log 2>&1
step timeout -k 10 300 python -u benchmarks/bench_models.py --only rf,rf_ref > gpurun_out/r4_k7c_bench.log 2>&1 && timeout -k 10 300 python -u benchmarks/bench_models.py --only rf_ref >> gpurun_out/r4_k7c_bench.log 2>&1
export AVMI_FORMAT_TIMING=1
step timeout -k 10 900 python -u benchmarks/bench_predict_jobs.py --records 16777216 --jobs vit,mmc,pst,nbp,detr,mop,usb,hash,dummy,rs --reps 2 --out gpurun_out/r4_predict_jobs_v5.jsonl > gpurun_out/r4_predict_bench5.log 2>&1
