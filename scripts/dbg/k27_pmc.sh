#!/bin/bash
# K27 at 4,096 x 3,072 x 768: kernel trace + SQ counter pass per arithmetic mode
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/k27pmc
mkdir -p $O
SQ="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
for m in ${K27_MODES:-bf16x6 bf16x3}; do
  AVMI_F32_GEMM=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$m -o trace --output-format csv -- python3 benchmarks/pmc_targets.py k27 > $O/$m.trace.log 2>&1 || exit 1
  AVMI_F32_GEMM=$m timeout -s KILL 90 rocprofv3 --pmc $SQ -d $O/$m -o sq --output-format csv -- python3 benchmarks/pmc_targets.py k27 > $O/$m.sq.log 2>&1 || exit 1
done
python3 scripts/pmc_summary.py $O > $O/summary.jsonl; cat $O/summary.jsonl
