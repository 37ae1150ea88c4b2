# PMC of the kernels added this session: fused MLP weight gradient (mlp bench) and TF-IDF (tfidf bench)
set -o pipefail
P=$GRAFT_REPO_ROOT/gpurun_out/pmc3
mkdir -p $P
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $P/mlp -o mlp -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_kernels.py --only mlp > $GRAFT_REPO_ROOT/gpurun_out/pmc3_mlp.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $P/tfidf -o tfidf -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_r3_kernels.py tfidf > $GRAFT_REPO_ROOT/gpurun_out/pmc3_tfidf.log 2>&1
rc=$?
for f in $(find $P -name "*counter_collection.csv"); do python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py "$f" >> $GRAFT_REPO_ROOT/gpurun_out/r3_new_kernels_pmc.jsonl; done
find $P -name "*.csv" -size +2M -delete
find $P -name "*.db" -delete
exit $rc
