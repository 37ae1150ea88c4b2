#!/bin/bash
# planes kernel: tests, then kernel-trace timing at BK 16 / 32 (x6, x3) and BK 16 ablations
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/k27bk; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cfg in "16 bf16x6 0 2" "16 bf16x6 3 2" "16 bf16x3 0 2" "16 bf16x3 3 2"; do
  set -- $cfg
  AVMI_PLANES_BK=$1 AVMI_F32_GEMM=$2 AVMI_PLANES_ABL=$3 AVMI_PLANES_NST=$4 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/bk$1_$2_a$3_n$4 -o trace --output-format csv -- python3 benchmarks/pmc_targets.py k27 > $O/bk$1_$2_a$3_n$4.log 2>&1 || exit 1
done
python3 scripts/pmc_summary.py $O | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print(d['target'], d['kernel'], round(d['mean_ms'] * 1000, 1), 'us')"
