# round-5 batch 16: counters for the round-5 kernels (gemm_tn, transformer epilogues, streaming SMO select), BERT bench
set -o pipefail
mkdir -p gpurun_out/r5b16
export TMPDIR=/tmp
O=gpurun_out/r5b16
timeout -k 10 300 python -u benchmarks/bench_bert.py > $O/bert_bench.jsonl 2> $O/bert_bench.err || exit $?
PMC_OUT=$O/pmc PMC_TARGETS="gemm_tn bert svm_select" timeout -k 10 900 bash scripts/gpu_pmc.sh > $O/pmc.log 2>&1 || exit $?
find $O/pmc -name "*kernel_trace.csv" -delete
find $O/pmc -name "*counter_collection.csv" -size +4M -delete
