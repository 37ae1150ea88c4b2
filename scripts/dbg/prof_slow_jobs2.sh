#!/bin/bash
# warm-call host profiles (cProfile) + kernel statistics of the slowest record-wise jobs
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_slow2
mkdir -p $O
timeout -k 10 240 python scripts/dbg/warm_profile.py $O benchmarks/bench_explore_jobs_scale.py --rows 2097152 nads loo > $O/explore.jsonl 2> $O/explore.err || exit 1
timeout -k 10 240 python scripts/dbg/warm_profile.py $O benchmarks/bench_keyed_jobs_scale.py kpp cgs gb > $O/keyed.jsonl 2> $O/keyed.err || exit 1
timeout -k 10 240 python scripts/dbg/warm_profile.py $O benchmarks/bench_text_jobs_scale.py semanticSearch_corpus > $O/text.jsonl 2> $O/text.err || exit 1
# unprofiled rates
timeout -k 10 240 python benchmarks/bench_explore_jobs_scale.py --rows 2097152 nads loo > $O/explore_plain.jsonl 2>&1 || exit 1
timeout -k 10 240 python benchmarks/bench_keyed_jobs_scale.py kpp cgs gb smb rfb > $O/keyed_plain.jsonl 2>&1 || exit 1
timeout -k 10 240 python benchmarks/bench_text_jobs_scale.py semanticSearch_corpus > $O/text_plain.jsonl 2>&1 || exit 1
