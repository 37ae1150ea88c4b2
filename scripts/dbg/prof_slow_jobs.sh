#!/bin/bash
# host (cProfile) and kernel (rocprofv3) profiles of the slowest record-wise jobs
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_slow
mkdir -p $O
timeout -k 10 240 python -m cProfile -o $O/explore.prof benchmarks/bench_explore_jobs_scale.py --rows 2097152 nads loo > $O/explore.jsonl 2> $O/explore.err || exit 1
timeout -k 10 240 python -m cProfile -o $O/keyed.prof benchmarks/bench_keyed_jobs_scale.py kpp cgs gb > $O/keyed.jsonl 2> $O/keyed.err || exit 1
timeout -k 10 240 python -m cProfile -o $O/text.prof benchmarks/bench_text_jobs_scale.py semanticSearch_corpus > $O/text.jsonl 2> $O/text.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kt_explore -o run --output-format csv -- python3 benchmarks/bench_explore_jobs_scale.py --rows 2097152 nads loo > $O/kt_explore.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kt_keyed -o run --output-format csv -- python3 benchmarks/bench_keyed_jobs_scale.py kpp cgs gb > $O/kt_keyed.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kt_text -o run --output-format csv -- python3 benchmarks/bench_text_jobs_scale.py semanticSearch_corpus > $O/kt_text.log 2>&1 || exit 1
# keep only the per-kernel statistics (the full traces exceed the 64 MiB pull limit)
find $O -name "*kernel_trace.csv" -delete
find $O -name "*agent_info.csv" -delete
du -sh $O
