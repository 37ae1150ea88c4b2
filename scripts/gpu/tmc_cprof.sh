set -o pipefail
mkdir -p gpurun_out
CUDA_LAUNCH_BLOCKING=1 timeout -k 10 400 python -u -c "
import cProfile, pstats, sys
sys.argv = ['bench_ingest.py', '--formats', 'tmc', '--jobs', '--reps', '1']
sys.path.insert(0, 'benchmarks')
import runpy
cProfile.run(\"runpy.run_path('benchmarks/bench_ingest.py', run_name='__main__')\", 'gpurun_out/tmc.prof')
p = pstats.Stats('gpurun_out/tmc.prof'); p.sort_stats('tottime').print_stats(25)
" > gpurun_out/tmc_cprof.log 2>&1
