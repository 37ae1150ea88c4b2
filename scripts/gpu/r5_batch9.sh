# round-5 batch 9: recordSimilarity device formatting; k-means NBUF=2 default
set -o pipefail
mkdir -p gpurun_out/r5b9
export TMPDIR=/tmp
O=gpurun_out/r5b9
timeout -k 10 400 python -u -m pytest tests/test_data_parallel_jobs.py tests/test_distance.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/gpu/rs_profile.py > $O/rs_profile.txt 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/bench_predict_jobs.py --jobs rs --reps 3 > $O/rs_bench.jsonl 2> $O/rs_bench.err || exit $?
timeout -k 10 600 python -u benchmarks/bench_vs_reference.py --only kmeans > $O/kmeans_vsref.log 2>&1 || exit $?
