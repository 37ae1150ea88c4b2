# whole GPU test suite + smoke + 1-GPU bench
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/full_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/full_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/full_bench.log 2>&1
