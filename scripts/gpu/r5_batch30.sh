# round-5 batch 30: profiles of the slowest record-wise jobs (bag, loo, nads)
set -o pipefail
mkdir -p gpurun_out/r5b30
export TMPDIR=/tmp
O=gpurun_out/r5b30
timeout -k 10 300 python -u -m pytest tests/test_native_explore_jobs.py tests/test_resample.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for j in loo nads; do
  timeout -k 10 200 python -u scripts/diag/job_profile.py $j > $O/$j.log 2>&1 || exit $?
done
timeout -k 10 300 python -u benchmarks/bench_explore_jobs_scale.py --rows 2097152 --device cuda bag spc > $O/jobs.jsonl 2> $O/jobs.err || exit $?
