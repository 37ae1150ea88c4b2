# GBT whole-round graph: tests, fits alone and after the other reference benches
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest tests/test_tree.py tests/test_recovery.py tests/test_supervised.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_gbt_round_tests.log 2>&1
step timeout -k 10 300 python -u benchmarks/profile_gbt.py --rows 65536 > gpurun_out/r4_profile_gbt2.log 2>&1
step timeout -k 10 300 python -u benchmarks/bench_models.py --only gbt > gpurun_out/r4_models_gbt2.log 2>&1
step timeout -k 10 900 python -u benchmarks/bench_vs_reference.py > gpurun_out/r4_vs_reference_final3.jsonl 2> gpurun_out/r4_vs_reference_final3.err
