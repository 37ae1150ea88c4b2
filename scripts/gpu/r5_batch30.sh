# round-5 batch 30: profiles of the slowest record-wise jobs (bag, loo, nads)
set -o pipefail
mkdir -p gpurun_out/r5b30
export TMPDIR=/tmp
O=gpurun_out/r5b30
for j in bag loo nads; do
  timeout -k 10 200 python -u scripts/diag/job_profile.py $j > $O/$j.log 2>&1 || exit $?
done
