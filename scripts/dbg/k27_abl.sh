#!/bin/bash
# planes kernel ablations (kernel trace): 0 full, 1 no MFMA, 2 no in-loop DMA
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/k27abl; mkdir -p $O
for a in 0 1 2; do
  AVMI_PLANES_ABL=$a AVMI_F32_GEMM=bf16x6 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/abl$a -o trace --output-format csv -- python3 benchmarks/pmc_targets.py k27 > $O/abl$a.log 2>&1 || exit 1
done
python3 scripts/pmc_summary.py $O | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print(d['target'], d['kernel'], round(d['mean_ms'] * 1000, 1), 'us')"
