#!/bin/bash
# round-6 re-measure of the model benches on the final kernels (fp32 GEMMs now split-bf16 x6 by default)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_models; mkdir -p $O
timeout -k 10 400 python -u benchmarks/bench_lstm.py --impls fused,fused_graph,miopen,miopen_graph > $O/lstm.jsonl 2> $O/lstm.err || { tail -20 $O/lstm.err; exit 1; }
cat $O/lstm.jsonl
timeout -k 10 500 python -u benchmarks/bench_vs_reference.py --only nb,kmeans,logit,svm,knn,lstm > $O/vsref.jsonl 2> $O/vsref.err || { tail -20 $O/vsref.err; exit 1; }
cut -c1-260 $O/vsref.jsonl
