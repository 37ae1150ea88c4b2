# round-5 batch 11: gemm_tn with fewer slices + unrolled slice sum
set -o pipefail
mkdir -p gpurun_out/r5b11
export TMPDIR=/tmp
O=gpurun_out/r5b11
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for g in mfma blas; do
  AVMI_LSTM_GEMM=$g timeout -k 10 300 python -u benchmarks/bench_lstm.py --configs reference_ct --impls fused,fused_graph,miopen,miopen_graph --steps 50 >> $O/lstm_ab.jsonl 2>> $O/lstm.err || exit $?
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_lstm -o l -- python3 $R/benchmarks/bench_lstm.py --configs reference_ct --impls fused --steps 20 > $R/$O/prof_lstm.log 2>&1 || exit $?
find $R/$O/prof_* -name "*kernel_trace.csv" -delete
