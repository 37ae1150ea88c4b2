# round-5 batch 35: numericalAttrDistrStats on the device
set -o pipefail
mkdir -p gpurun_out/r5b35
export TMPDIR=/tmp
O=gpurun_out/r5b35
timeout -k 10 300 python -u -m pytest tests/test_native_explore_jobs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/bench_explore_jobs_scale.py --rows 2097152 --device cuda nads > $O/jobs.jsonl 2> $O/jobs.err || exit $?
