#!/bin/bash
# k-means score kernel per arithmetic mode: kernel trace stats, then one PMC pass per mode
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for m in f32 bf16x3 bf16x6; do
  AVMI_KMEANS_MFMA=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_km2_$m -o km --output-format csv -- python3 benchmarks/pmc_targets.py kmeans > gpurun_out/r6_km2_$m.log 2>&1 || exit 1
done
for m in f32 bf16x6; do
  AVMI_KMEANS_MFMA=$m timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVES -d gpurun_out/r6_km_pmc_$m -o km --output-format csv -- python3 benchmarks/pmc_targets.py kmeans > gpurun_out/r6_km_pmc_$m.log 2>&1 || exit 1
done
