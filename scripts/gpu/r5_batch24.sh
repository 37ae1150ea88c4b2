# round-5 batch 24: 128 x 128 tile for large outputs (A/B by AVMI_BIG_TILES)
set -o pipefail
mkdir -p gpurun_out/r5b24
export TMPDIR=/tmp
O=gpurun_out/r5b24
timeout -k 10 400 python -u -m pytest tests/test_gemm.py tests/test_nn.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
AVMI_BIG_TILES=1 timeout -k 10 200 python -u benchmarks/bench_gemm_shapes.py > $O/gemm1.jsonl 2> $O/g1.err || exit $?
AVMI_BIG_TILES=0 timeout -k 10 200 python -u benchmarks/bench_gemm_shapes.py > $O/gemm0.jsonl 2> $O/g0.err || exit $?
