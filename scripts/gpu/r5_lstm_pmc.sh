# fp32 LSTM trace at the reference shape + the round-4 kernels' counter passes
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_rnn.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5/rnn_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u benchmarks/bench_lstm.py --configs reference_ct --impls fused,fused_graph,miopen,miopen_graph --steps 30 > gpurun_out/r5/lstm_bench.jsonl 2> gpurun_out/r5/lstm_bench.err || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5/prof_lstm_fused -o l -- python3 $R/benchmarks/bench_lstm.py --configs reference_ct --impls fused --steps 20 > $R/gpurun_out/r5/prof_lstm_fused.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5/prof_lstm_miopen -o l -- python3 $R/benchmarks/bench_lstm.py --configs reference_ct --impls miopen --steps 20 > $R/gpurun_out/r5/prof_lstm_miopen.log 2>&1 || exit $?
find $R/gpurun_out/r5/prof_lstm_* -name "*kernel_trace.csv" -delete
cd $R
PMC_OUT=gpurun_out/r5/pmc_r4k PMC_TARGETS="fmt pairs split lstm" timeout -k 10 900 bash scripts/gpu_pmc.sh > gpurun_out/r5/pmc_r4k.log 2>&1
