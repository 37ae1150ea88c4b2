#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm.py tests/test_bert.py > gpurun_out/bert_after_tests.log 2>&1 || { tail -30 gpurun_out/bert_after_tests.log; exit 1; }
tail -1 gpurun_out/bert_after_tests.log
for g in bf16x3 bf16x6; do
  AVMI_BERT_GEMM=$g timeout -k 10 300 python -u benchmarks/bench_bert.py > gpurun_out/bert_after_$g.jsonl 2>&1 || exit 1
  grep '"B"' gpurun_out/bert_after_$g.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('bert', '$g', d['B'], d['S'], round(d['ours_ms'], 3), round(d['transformers_ms'], 3), round(d['speedup'], 2), d['max_abs_diff'])"
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/bert32b -o trace --output-format csv -- python3 benchmarks/pmc_targets.py bert32 > gpurun_out/bert32b.log 2>&1 || exit 1
