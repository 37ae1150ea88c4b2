# GBT gradient histogram replicas: tests, alternating A/B timings
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_tree.py tests/test_forest.py -x -q --timeout 150 --timeout-method thread -m gpu > gpurun_out/gh_tests.log 2>&1 || exit 1
for r in 1 4 1 4 2; do
  AVMI_GBT_HIST_REP=$r timeout -k 10 200 python -u benchmarks/bench_models.py --only gbt > gpurun_out/gh_$r.log 2>&1 || exit 1
  grep '^{' gpurun_out/gh_$r.log | sed "s/^/rep=$r /" >> gpurun_out/gh_all.log
done
