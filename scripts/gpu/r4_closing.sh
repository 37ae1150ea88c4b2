# Round-4 closing run: the whole GPU suite, smoke, the 1-GPU bench, then the model / reference benches
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_closing_gpu.log 2>&1
step timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r4_closing_smoke.log 2>&1
step timeout -k 10 300 python -u bench.py > gpurun_out/r4_closing_bench.log 2>&1
step timeout -k 10 600 python -u benchmarks/bench_models.py > gpurun_out/r4_models_final2.jsonl 2> gpurun_out/r4_models_final2.err
step timeout -k 10 900 python -u benchmarks/bench_vs_reference.py > gpurun_out/r4_vs_reference_final2.jsonl 2> gpurun_out/r4_vs_reference_final2.err
