#!/bin/bash
# split-bf16 gemm_tn / knn: GPU tests of the touched kernels and their users, then the mode sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gemm.py tests/test_distance.py tests/test_native_predictors.py tests/test_rnn.py \
  > gpurun_out/r6_sbf16_gemm_knn_tests.log 2>&1 || { tail -30 gpurun_out/r6_sbf16_gemm_knn_tests.log; exit 1; }
tail -3 gpurun_out/r6_sbf16_gemm_knn_tests.log
timeout -k 10 400 python -u benchmarks/bench_sbf16_modes.py > gpurun_out/r6_sbf16_gemm_knn.jsonl 2> gpurun_out/r6_sbf16_bench.err || { tail -20 gpurun_out/r6_sbf16_bench.err; exit 1; }
cat gpurun_out/r6_sbf16_gemm_knn.jsonl
# K27 x6: the swizzled three-per-CU tile against the padded two-per-CU one
for swz in 1 0; do
  AVMI_F32_GEMM=bf16x6 AVMI_SBF16_SWZ=$swz timeout -k 10 300 python -u benchmarks/bench_gemm_shapes.py > gpurun_out/r6_gemm_x6_swz$swz.jsonl 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_nn.py tests/test_bert.py \
  > gpurun_out/r6_swz_nn_bert_tests.log 2>&1 || { tail -30 gpurun_out/r6_swz_nn_bert_tests.log; exit 1; }
tail -2 gpurun_out/r6_swz_nn_bert_tests.log
