# round-end rehearsal, part 2: smoke, 1-GPU bench, BERT bench
set -o pipefail
mkdir -p gpurun_out/r5full
export TMPDIR=/tmp
O=gpurun_out/r5full
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python -u benchmarks/bench_bert.py > $O/bert_bench.jsonl 2> $O/bert_bench.err || exit $?
timeout -k 10 400 python -u benchmarks/bench_lstm.py --impls fused,fused_graph,miopen,miopen_graph > $O/lstm.jsonl 2> $O/lstm.err || exit $?
