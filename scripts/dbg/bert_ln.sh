#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_bert.py tests/test_text_jobs.py > gpurun_out/bert_ln_tests.log 2>&1 || { tail -30 gpurun_out/bert_ln_tests.log; exit 1; }
tail -1 gpurun_out/bert_ln_tests.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/bert1b -o trace --output-format csv -- python3 benchmarks/pmc_targets.py bert > gpurun_out/bert1b.log 2>&1 || exit 1
timeout -k 10 300 python -u benchmarks/bench_bert.py > gpurun_out/bert_ln.jsonl 2>&1 || exit 1
grep '"B"' gpurun_out/bert_ln.jsonl | cut -c1-200
