# closing reference comparison and model benches with the GC frozen before each bench
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
export AVMI_GBT_TIMING=1
step timeout -k 10 900 python -u benchmarks/bench_vs_reference.py > gpurun_out/r4_vs_reference_final4.jsonl 2> gpurun_out/r4_vs_reference_final4.err
step timeout -k 10 600 python -u benchmarks/bench_models.py > gpurun_out/r4_models_final4.jsonl 2> gpurun_out/r4_models_final4.err
