# round-5 batch 31: keyed / data-parallel jobs end to end at 400 x their test sizes
set -o pipefail
mkdir -p gpurun_out/r5b31
export TMPDIR=/tmp
O=gpurun_out/r5b31
timeout -k 10 900 python -u benchmarks/bench_keyed_jobs_scale.py --scale 400 --device cuda > $O/jobs.jsonl 2> $O/jobs.err || exit $?
