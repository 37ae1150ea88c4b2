# kernel-trace stats of the implicit-kernel SVM at N = 262,144 x 16
set -o pipefail
P=$GRAFT_REPO_ROOT/gpurun_out/r5/prof_svm262k
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $GRAFT_REPO_ROOT/benchmarks/bench_svm_implicit.py --sizes 262144 --d 16 --paths implicit --reps 1 > $GRAFT_REPO_ROOT/gpurun_out/r5/svm262k.jsonl 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o s262k -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_svm_implicit.py --sizes 262144 --d 16 --paths implicit --reps 1 > $GRAFT_REPO_ROOT/gpurun_out/r5/svm262k_prof.log 2>&1
rc=$?
find $P -name "*kernel_trace.csv" -delete
find $P -name "*.db" -delete
exit $rc
