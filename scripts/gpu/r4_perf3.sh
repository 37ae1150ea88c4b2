# Round-4 measurements, part 3: GPU tests of this round's fixes, K7 kernel profile, predict jobs with
# the device formatter (write-time breakdown; /tmp and /dev/shm outputs), then the perf2 set.
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
R=$GRAFT_REPO_ROOT
step timeout -k 10 600 python -u -m pytest tests/test_rnn.py tests/test_tree.py tests/test_distance.py tests/test_native_explore_jobs.py tests/test_native_predictors.py tests/test_format_device.py tests/test_data_parallel_jobs.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4_tests3.log 2>&1
export AVMI_FORMAT_TIMING=1
step timeout -k 10 900 python -u benchmarks/bench_predict_jobs.py --records 16777216 --jobs vit,nbp,detr,usb,hash --reps 2 --out gpurun_out/r4_predict_jobs_v3.jsonl > gpurun_out/r4_predict_bench3.log 2>&1
step timeout -k 10 900 python -u benchmarks/bench_predict_jobs.py --records 16777216 --jobs vit,nbp --reps 2 --dir /dev/shm --out gpurun_out/r4_predict_jobs_v3.jsonl >> gpurun_out/r4_predict_bench3.log 2>&1
unset AVMI_FORMAT_TIMING
cd /tmp && export TMPDIR=/tmp
P=$R/gpurun_out/prof_k7
step timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o k7 -- python3 $R/benchmarks/bench_models.py --only rf_ref > $R/gpurun_out/r4_k7_prof.log 2>&1
find $P -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/r4_k7_kernel_stats.csv \;
find $P -name "*kernel_trace.csv" -delete
cd $R
step bash scripts/gpu/r4_perf2.sh
