# Round-4 measurements, part 4: re-test the last fixes, predict jobs v4 (fresh output files),
# reference-semantics forest vs binary forest.
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 600 python -u -m pytest tests/test_rnn.py tests/test_native_explore_jobs.py tests/test_tree.py tests/test_forest.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4_tests4.log 2>&1
step timeout -k 10 300 python -u benchmarks/bench_models.py --only rf,rf_ref > gpurun_out/r4_rf_bench4.log 2>&1
export AVMI_FORMAT_TIMING=1
step timeout -k 10 900 python -u benchmarks/bench_predict_jobs.py --records 16777216 --jobs vit,mmc,pst,nbp,detr,mop,usb,hash,dummy,rs --reps 2 --out gpurun_out/r4_predict_jobs_v4.jsonl > gpurun_out/r4_predict_bench4.log 2>&1
