# round-5: every reference-vs-ours comparison on one box (sklearn / torch-CPU on 16 host threads)
set -o pipefail
mkdir -p gpurun_out/r5vs
export TMPDIR=/tmp
timeout -k 10 1000 python -u benchmarks/bench_vs_reference.py > gpurun_out/r5vs/vs_reference.jsonl 2> gpurun_out/r5vs/vs_reference.err || exit $?
