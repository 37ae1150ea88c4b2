# round-5 batch 28: the remaining scale jobs + profiles of the slow ones (loo, nuc)
set -o pipefail
mkdir -p gpurun_out/r5b28
export TMPDIR=/tmp
O=gpurun_out/r5b28
timeout -k 10 300 python -u -m pytest tests/test_native_explore_jobs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 600 python -u benchmarks/bench_explore_jobs_scale.py --rows 2097152 --device cuda loo nuc spc kmc bag nor pro tra uvc nads > $O/jobs.jsonl 2> $O/jobs.err || exit $?
timeout -k 10 200 python -u scripts/diag/job_profile.py nuc > $O/nuc.log 2>&1 || exit $?
