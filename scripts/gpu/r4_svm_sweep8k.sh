# N = 8192: rel_tol and top-k part A/B
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
O=gpurun_out/r4_svm_sweep8k.log
: > $O
for rt in 0.2 0.3 0.45; do
  echo "# rel_tol $rt radix" >> $O
  AVMI_SMO_REL_TOL=$rt step timeout -k 10 120 python -u benchmarks/bench_svm.py 8192,8192 ws >> $O 2>&1
done
for hp in 8 16; do
  echo "# topk hp $hp" >> $O
  AVMI_SMO_TOPK_MIN_N=4097 AVMI_SMO_TOPK_HP=$hp step timeout -k 10 120 python -u benchmarks/bench_svm.py 8192,8192 ws >> $O 2>&1
done
