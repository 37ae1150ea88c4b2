# Round-4 closing measurements: every model bench, reference comparisons, prediction jobs
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 600 python -u benchmarks/bench_models.py > gpurun_out/r4_models_final.jsonl 2> gpurun_out/r4_models_final.err
step timeout -k 10 900 python -u benchmarks/bench_vs_reference.py > gpurun_out/r4_vs_reference_final.jsonl 2> gpurun_out/r4_vs_reference_final.err
