# does a preceding sklearn run slow the next GPU fit? (GBT / SVM in the full reference run)
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
O=gpurun_out/r4_vsref_order.log
: > $O
echo "# rf,gbt,svm" >> $O
step timeout -k 10 300 python -u benchmarks/bench_vs_reference.py --only rf,gbt,svm >> $O 2>&1
echo "# rf,gbt,svm OMP_WAIT_POLICY=PASSIVE" >> $O
OMP_WAIT_POLICY=PASSIVE step timeout -k 10 300 python -u benchmarks/bench_vs_reference.py --only rf,gbt,svm >> $O 2>&1
echo "# nb,gbt,svm" >> $O
step timeout -k 10 300 python -u benchmarks/bench_vs_reference.py --only nb,gbt,svm >> $O 2>&1
