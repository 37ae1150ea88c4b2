# round-5 batch 33: text drivers on a 6,000-document corpus
set -o pipefail
mkdir -p gpurun_out/r5b33
export TMPDIR=/tmp
O=gpurun_out/r5b33
timeout -k 10 900 python -u benchmarks/bench_text_jobs_scale.py --per 2000 --device cuda > $O/text.jsonl 2> $O/text.err || exit $?
