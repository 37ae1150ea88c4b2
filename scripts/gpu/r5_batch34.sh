# round-5 batch 34: tabular counting jobs at 2^22 records
set -o pipefail
mkdir -p gpurun_out/r5b34
export TMPDIR=/tmp
O=gpurun_out/r5b34
timeout -k 10 600 python -u benchmarks/bench_tabular_jobs_scale.py --rows 4194304 --device cuda > $O/tab.jsonl 2> $O/tab.err || exit $?
