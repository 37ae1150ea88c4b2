# round-5 batch 27: exploration / encoding jobs end to end at 2^21 records
set -o pipefail
mkdir -p gpurun_out/r5b27
export TMPDIR=/tmp
O=gpurun_out/r5b27
timeout -k 10 900 python -u benchmarks/bench_explore_jobs_scale.py --rows 2097152 --device cuda > $O/jobs.jsonl 2> $O/jobs.err || exit $?
