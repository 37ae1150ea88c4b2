#!/bin/bash
# the round-5 job sweeps re-run on the final round-6 tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_sweeps; mkdir -p $O
timeout -k 10 400 python -u benchmarks/bench_explore_jobs_scale.py > $O/explore.jsonl 2> $O/explore.err || { tail -20 $O/explore.err; exit 1; }
echo "explore: $(grep -c '^{' $O/explore.jsonl) jobs"
timeout -k 10 400 python -u benchmarks/bench_keyed_jobs_scale.py > $O/keyed.jsonl 2> $O/keyed.err || { tail -20 $O/keyed.err; exit 1; }
echo "keyed: $(grep -c '^{' $O/keyed.jsonl) jobs"
timeout -k 10 400 python -u benchmarks/bench_tabular_jobs_scale.py > $O/tabular.jsonl 2> $O/tabular.err || { tail -20 $O/tabular.err; exit 1; }
echo "tabular: $(grep -c '^{' $O/tabular.jsonl) jobs"
timeout -k 10 400 python -u benchmarks/bench_text_jobs_scale.py > $O/text.jsonl 2> $O/text.err || { tail -20 $O/text.err; exit 1; }
echo "text: $(grep -c '^{' $O/text.jsonl) jobs"
