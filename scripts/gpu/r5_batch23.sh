# round-5 batch 23: one-shot split-K slices (A/B by AVMI_SPLITK_ONESHOT)
set -o pipefail
mkdir -p gpurun_out/r5b23
export TMPDIR=/tmp
O=gpurun_out/r5b23
timeout -k 10 400 python -u -m pytest tests/test_gemm.py tests/test_bert.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
AVMI_SPLITK_ONESHOT=1 timeout -k 10 200 python -u benchmarks/bench_gemm_shapes.py > $O/gemm1.jsonl 2> $O/g1.err || exit $?
AVMI_SPLITK_ONESHOT=0 timeout -k 10 200 python -u benchmarks/bench_gemm_shapes.py > $O/gemm0.jsonl 2> $O/g0.err || exit $?
AVMI_SPLITK_ONESHOT=1 timeout -k 10 300 python -u benchmarks/bench_bert.py > $O/bert1.jsonl 2> $O/b1.err || exit $?
AVMI_SPLITK_ONESHOT=0 timeout -k 10 300 python -u benchmarks/bench_bert.py > $O/bert0.jsonl 2> $O/b0.err || exit $?
