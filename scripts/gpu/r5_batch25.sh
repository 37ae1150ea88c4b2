# round-5 batch 25: counters for the final BERT kernels (attention, fused split-K LayerNorm, split-K tile)
set -o pipefail
mkdir -p gpurun_out/r5b25
export TMPDIR=/tmp
O=gpurun_out/r5b25
PMC_OUT=$O/pmc PMC_TARGETS="bert" timeout -k 10 600 bash scripts/gpu_pmc.sh > $O/pmc.log 2>&1 || exit $?
find $O/pmc -name "*kernel_trace.csv" -delete
find $O/pmc -name "*counter_collection.csv" -size +4M -delete
