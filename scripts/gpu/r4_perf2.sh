# Round-4 measurements: fused fp32 LSTM pairs, implicit-kernel SVM at production sizes, batched
# one-vs-rest waves (PMC).  Each GPU step under its own time limit; stop on a timeout / crash.
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
R=$GRAFT_REPO_ROOT
step timeout -k 10 500 python -u benchmarks/bench_lstm.py --steps 20 --warmup 3 > gpurun_out/r4_lstm.jsonl 2> gpurun_out/r4_lstm.err
step timeout -k 10 600 python -u benchmarks/bench_svm_implicit.py --sizes 8192,32768 --d 8 --paths dense,implicit --sklearn --out gpurun_out/r4_svm_implicit.jsonl > gpurun_out/r4_svm_implicit.log 2>&1
step timeout -k 10 600 python -u benchmarks/bench_svm_implicit.py --sizes 262144 --d 16 --paths implicit --reps 1 --out gpurun_out/r4_svm_implicit.jsonl >> gpurun_out/r4_svm_implicit.log 2>&1
step timeout -k 10 300 python -u benchmarks/bench_svm_ovr.py --n 8192 --classes 16 > gpurun_out/r4_svm_ovr.jsonl 2>&1
cd /tmp && export TMPDIR=/tmp
P=$R/gpurun_out/pmc_ovr
step timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $P -o ovr -- python3 $R/benchmarks/bench_svm_ovr.py --n 8192 --classes 16 --reps 1 > $R/gpurun_out/pmc_ovr.log 2>&1
for f in $(find $P -name "*counter_collection.csv"); do python3 $R/tools/pmc_summary.py "$f" >> $R/gpurun_out/r4_svm_ovr_pmc.jsonl; done
find $P -name "*counter_collection.csv" -delete
exit 0
