# PMC counters (waves, VALU / SALU / LDS instructions, busy cycles) of the SMO kernels at N = 8192
set -o pipefail
P=$GRAFT_REPO_ROOT/gpurun_out/pmc
mkdir -p $P
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $P -o svm -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_svm.py 8192 ws > $GRAFT_REPO_ROOT/gpurun_out/pmc_run.log 2>&1
rc=$?
f=$(find $P -name "*counter_collection.csv" | head -1)
[ $rc -eq 0 ] && python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py "$f" > $GRAFT_REPO_ROOT/gpurun_out/svm_pmc.jsonl 2>&1
rc=$?
find $P -name "*.csv" -size +2M -delete
find $P -name "*.db" -delete
exit $rc
