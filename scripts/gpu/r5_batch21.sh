# round-5 batch 21: XCD-aware grouped tile order in the K27 tile (A/B by AVMI_XCD_TILES)
set -o pipefail
mkdir -p gpurun_out/r5b21
export TMPDIR=/tmp
O=gpurun_out/r5b21
timeout -k 10 400 python -u -m pytest tests/test_gemm.py tests/test_nn.py tests/test_rnn.py tests/test_bert.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
AVMI_XCD_TILES=0 timeout -k 10 200 python -u benchmarks/bench_gemm_shapes.py > $O/gemm_shapes_xcd0.jsonl 2> $O/g0.err || exit $?
AVMI_XCD_TILES=1 timeout -k 10 200 python -u benchmarks/bench_gemm_shapes.py > $O/gemm_shapes_xcd1.jsonl 2> $O/g1.err || exit $?
AVMI_XCD_TILES=0 timeout -k 10 200 python -u benchmarks/bench_gemm_shapes.py > $O/gemm_shapes_xcd0b.jsonl 2> $O/g0b.err || exit $?
