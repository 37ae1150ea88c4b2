# Round-4 whole GPU suite (no -x: every failure listed), smoke, 1-GPU bench.
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_full_gpu.log 2>&1
step timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r4_full_smoke.log 2>&1
step timeout -k 10 300 python -u bench.py > gpurun_out/r4_full_bench.log 2>&1
