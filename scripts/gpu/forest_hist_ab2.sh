# forest histogram replicas: alternating A/B timings on one box
set -o pipefail
for r in 1 8 1 8 4 2; do
  AVMI_FOREST_HIST_REP=$r timeout -k 10 200 python -u benchmarks/bench_models.py --only rf > gpurun_out/fh2_$r.log 2>&1 || exit 1
  grep '"random_forest"' gpurun_out/fh2_$r.log | sed "s/^/rep=$r /" >> gpurun_out/fh2_all.log
done
