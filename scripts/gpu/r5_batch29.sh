# round-5 batch 29: record-wise jobs GPU == CPU, all 18 jobs end to end at 2^21 records
set -o pipefail
mkdir -p gpurun_out/r5b29
export TMPDIR=/tmp
O=gpurun_out/r5b29
timeout -k 10 300 python -u -m pytest tests/test_native_explore_jobs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 900 python -u benchmarks/bench_explore_jobs_scale.py --rows 2097152 --device cuda > $O/jobs.jsonl 2> $O/jobs.err || exit $?
