# full GPU suite (round-end rehearsal, part 1)
set -o pipefail
mkdir -p gpurun_out/r5full
export TMPDIR=/tmp
O=gpurun_out/r5full
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || exit $?
