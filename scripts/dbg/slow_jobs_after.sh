#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_slow3
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_native_explore_jobs.py tests/test_distance.py tests/test_text_jobs.py tests/test_data_parallel_jobs.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 240 python scripts/dbg/warm_profile.py $O benchmarks/bench_explore_jobs_scale.py --rows 2097152 nads loo > $O/explore.jsonl 2> $O/explore.err || exit 1
timeout -k 10 240 python scripts/dbg/warm_profile.py $O benchmarks/bench_keyed_jobs_scale.py kpp cgs > $O/keyed.jsonl 2> $O/keyed.err || exit 1
timeout -k 10 240 python benchmarks/bench_explore_jobs_scale.py --rows 2097152 nads loo > $O/explore_plain.jsonl 2>&1 || exit 1
timeout -k 10 240 python benchmarks/bench_keyed_jobs_scale.py kpp cgs > $O/keyed_plain.jsonl 2>&1 || exit 1
timeout -k 10 240 python benchmarks/bench_text_jobs_scale.py semanticSearch_corpus > $O/text_plain.jsonl 2>&1 || exit 1
