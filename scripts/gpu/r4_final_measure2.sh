# graph capture without the allocator flush: tests, then the closing model / reference benches
set -o pipefail
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 600 python -u -m pytest tests/test_tree.py tests/test_linear.py tests/test_svm_ws.py tests/test_rnn.py tests/test_nn.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_graph_tests.log 2>&1
step timeout -k 10 600 python -u benchmarks/bench_models.py > gpurun_out/r4_models_final2.jsonl 2> gpurun_out/r4_models_final2.err
step timeout -k 10 900 python -u benchmarks/bench_vs_reference.py > gpurun_out/r4_vs_reference_final2.jsonl 2> gpurun_out/r4_vs_reference_final2.err
