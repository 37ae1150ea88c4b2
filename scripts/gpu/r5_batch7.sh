# round-5 batch 7: recordSimilarity host profile; LSTM GEMMs on the f32-MFMA tile kernel vs hipBLASLt
set -o pipefail
mkdir -p gpurun_out/r5b7
export TMPDIR=/tmp
O=gpurun_out/r5b7
timeout -k 10 300 python -u scripts/gpu/rs_profile.py > $O/rs_profile.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_rnn.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/rnn_tests.log 2>&1 || exit $?
for g in mfma blas; do
  AVMI_LSTM_GEMM=$g timeout -k 10 300 python -u benchmarks/bench_lstm.py --configs reference_ct --impls fused,fused_graph --steps 50 >> $O/lstm_gemm_ab.jsonl 2>> $O/lstm.err || exit $?
done
timeout -k 10 300 python -u benchmarks/bench_lstm.py --configs reference_ct --impls miopen,miopen_graph --steps 50 >> $O/lstm_gemm_ab.jsonl 2>> $O/lstm.err || exit $?
