# full GPU suite + smoke + 1-GPU bench (round-end rehearsal)
set -o pipefail
mkdir -p gpurun_out/r5full
export TMPDIR=/tmp
O=gpurun_out/r5full
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
