# forest histogram: LDS replicas on / off — forest tests, RF timings, LDS conflict counters
set -o pipefail
P=$GRAFT_REPO_ROOT/gpurun_out/pmc
mkdir -p $P
timeout -k 10 300 python -u -m pytest tests/test_forest.py -x -q --timeout 150 --timeout-method thread -m gpu > gpurun_out/fh_tests.log 2>&1 &&
timeout -k 10 200 python -u benchmarks/bench_models.py --only rf > gpurun_out/fh_rep.log 2>&1 &&
AVMI_FOREST_HIST_REP=1 timeout -k 10 200 python -u benchmarks/bench_models.py --only rf > gpurun_out/fh_norep.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $P -o fh_rep -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_models.py --only rf > $GRAFT_REPO_ROOT/gpurun_out/fh_pmc1.log 2>&1 &&
AVMI_FOREST_HIST_REP=1 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $P -o fh_norep -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_models.py --only rf > $GRAFT_REPO_ROOT/gpurun_out/fh_pmc2.log 2>&1
rc=$?
for n in fh_rep fh_norep; do
  f=$(find $P -name "${n}*counter_collection.csv" | head -1)
  [ -n "$f" ] && python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py "$f" > $GRAFT_REPO_ROOT/gpurun_out/${n}_pmc.jsonl 2>&1
done
find $P -name "*.csv" -size +2M -delete
find $P -name "*.db" -delete
exit $rc
