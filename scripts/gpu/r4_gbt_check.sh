# GBT / SVM reference-comparison regressions: host profile of the GBT fit, the two benches alone
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 300 python -u benchmarks/profile_gbt.py --rows 65536 > gpurun_out/r4_profile_gbt.log 2>&1
step timeout -k 10 300 python -u benchmarks/bench_vs_reference.py --only gbt,svm > gpurun_out/r4_vsref_gbt_svm.log 2>&1
step timeout -k 10 300 python -u benchmarks/bench_models.py --only gbt > gpurun_out/r4_models_gbt.log 2>&1
