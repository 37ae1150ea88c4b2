# SVM at 12 000 / 16 384 rows: radix parts (default up to 16 384) vs top-k parts
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
O=gpurun_out/r4_svm_mid.log
: > $O
echo "# radix (default)" >> $O
step timeout -k 10 200 python -u benchmarks/bench_svm.py 12000,16384,12000,16384 ws >> $O 2>&1
echo "# topk (AVMI_SMO_TOPK_MIN_N=8193)" >> $O
AVMI_SMO_TOPK_MIN_N=8193 step timeout -k 10 200 python -u benchmarks/bench_svm.py 12000,16384,12000,16384 ws >> $O 2>&1
