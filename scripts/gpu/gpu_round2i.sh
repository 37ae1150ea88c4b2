#!/bin/bash
# A/B of four kNN kernel builds (_C_v0..3.so), then the full GPU suite on v2
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1 2 3; do
  cp avenir_amd/_C_v$v.so avenir_amd/_C.so
  timeout -k 10 200 python -u -m pytest tests/test_distance.py -x -q -m gpu -k knn --timeout 120 --timeout-method thread > gpurun_out/r2i_t$v.log 2>&1
  echo "== v$v" >> gpurun_out/r2i_knn.log
  timeout -k 10 200 python -u benchmarks/bench_kernels.py --only knn >> gpurun_out/r2i_knn.log 2>&1
done
cp avenir_amd/_C_v2.so avenir_amd/_C.so
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2i_tests.log 2>&1
cat gpurun_out/r2i_knn.log; tail -3 gpurun_out/r2i_tests.log
