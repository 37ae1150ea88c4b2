# working-set SMO: graph-captured vs eager outer steps
set -o pipefail
timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768 ws > gpurun_out/g_svm_graph.log 2>&1 &&
AVMI_SMO_GRAPH=0 timeout -k 10 200 python -u benchmarks/bench_svm.py 8192,32768 ws > gpurun_out/g_svm_eager.log 2>&1
