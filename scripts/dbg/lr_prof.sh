#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/lrprof; mkdir -p $O
timeout -k 10 300 python scripts/dbg/warm_profile.py $O benchmarks/bench_tabular_jobs_scale.py > $O/tab.jsonl 2> $O/tab.err || { tail -20 $O/tab.err; exit 1; }
grep logistic $O/tab.jsonl | cut -c1-250
python -c "
import pstats
pstats.Stats('$O/warm_logisticRegression.prof').sort_stats('tottime').print_stats(14)
" > $O/lr_profile.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o t --output-format csv -- python3 benchmarks/bench_tabular_jobs_scale.py > $O/trace.log 2>&1 || exit 1
