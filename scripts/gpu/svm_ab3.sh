# host-side loop variants (graph-captured block vs direct launches) x merge (rank vs radix), same box
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_svm_ws.py -x -q --timeout 150 --timeout-method thread -m gpu > gpurun_out/ab3_tests.log 2>&1 &&
for v in "1 1" "0 1" "1 0" "0 0"; do
  set -- $v
  AVMI_SMO_RUN_GRAPH=$1 AVMI_SMO_RANK_MERGE=$2 timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768,8192,32768 ws > gpurun_out/ab3_g$1_r$2.log 2>&1 || exit 1
done
