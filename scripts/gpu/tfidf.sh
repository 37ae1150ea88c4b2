# K28 TF-IDF: LDS document-frequency kernel + fused idf rows; tests and the kernel bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_text.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tfidf_tests.log 2>&1 &&
timeout -k 10 300 python -u benchmarks/bench_r3_kernels.py tfidf > gpurun_out/tfidf_bench.log 2>&1
