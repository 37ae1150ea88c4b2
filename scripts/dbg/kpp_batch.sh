#!/bin/bash
# batched k-means++ seeding: GPU tests of the k-means users, the keyed-job sweep (kpp + bandits), warm profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_kpp
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread -m gpu tests/test_distance.py tests/test_data_parallel_jobs.py tests/test_world_sizes.py tests/test_recovery.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 240 python benchmarks/bench_keyed_jobs_scale.py kpp gb smb rfb > $O/keyed_plain.jsonl 2>&1 || { tail -20 $O/keyed_plain.jsonl; exit 1; }
cat $O/keyed_plain.jsonl
timeout -k 10 240 python scripts/dbg/warm_profile.py $O benchmarks/bench_keyed_jobs_scale.py kpp gb > $O/keyed.jsonl 2> $O/keyed.err || exit 1
python -c "
import pstats, glob
for f in sorted(glob.glob('$O/warm_*.prof')):
    print('=====', f)
    pstats.Stats(f).sort_stats('tottime').print_stats(8)
" > $O/profiles.txt 2>&1
