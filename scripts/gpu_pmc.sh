#!/bin/bash
# Hardware-counter passes over the hot kernels (benchmarks/pmc_targets.py), one short program per
# target: a kernel-trace run for durations, then separate --pmc passes (SQ+GRBM, FETCH_SIZE,
# WRITE_SIZE) so no block exceeds its counter slots.  Summary: scripts/pmc_summary.py.
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=${PMC_OUT:-gpurun_out/pmc}
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
SQ=""
for c in SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES; do
  if grep -qw "$c" $O/counters.txt; then SQ="$SQ $c"; fi
done
echo "SQ pass counters:$SQ" | tee $O/sq_counters.txt
TARGETS=${PMC_TARGETS:-rowpack columns knn16 knn64 knn256 smo_ws forest}
for t in $TARGETS; do
  echo "== $t $(date +%T)"
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/$t -o trace --output-format csv -- python3 benchmarks/pmc_targets.py $t > $O/$t.trace.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $SQ GRBM_GUI_ACTIVE GRBM_COUNT -d $O/$t -o sq --output-format csv -- python3 benchmarks/pmc_targets.py $t > $O/$t.sq.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/$t -o fetch --output-format csv -- python3 benchmarks/pmc_targets.py $t > $O/$t.fetch.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $O/$t -o write --output-format csv -- python3 benchmarks/pmc_targets.py $t > $O/$t.write.log 2>&1
done
python3 scripts/pmc_summary.py $O > $O/summary.jsonl
cat $O/summary.jsonl
