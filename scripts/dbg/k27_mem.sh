#!/bin/bash
# planes kernel memory counters: HBM fetch bytes, L2 hit / miss (ABL0 and the in-loop tile)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/k27mem; mkdir -p $O
for p in 1 0; do
  AVMI_SBF16_PLANES=$p AVMI_F32_GEMM=bf16x6 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/p$p -o fetch --output-format csv -- python3 benchmarks/pmc_targets.py k27 > $O/p$p.f.log 2>&1 || exit 1
  AVMI_SBF16_PLANES=$p AVMI_F32_GEMM=bf16x6 timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/p$p -o tcc --output-format csv -- python3 benchmarks/pmc_targets.py k27 > $O/p$p.t.log 2>&1 || exit 1
  AVMI_SBF16_PLANES=$p AVMI_F32_GEMM=bf16x6 timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum -d $O/p$p -o ta --output-format csv -- python3 benchmarks/pmc_targets.py k27 > $O/p$p.ta.log 2>&1 || true
done
python3 scripts/pmc_summary.py $O | cut -c1-700
