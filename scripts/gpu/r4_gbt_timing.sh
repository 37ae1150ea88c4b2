# GBT fit phases inside the full reference run (AVMI_GBT_TIMING=1)
set -o pipefail
export AVMI_GBT_TIMING=1
timeout -k 10 900 python -u benchmarks/bench_vs_reference.py --only nb,rf,gbt,svm > gpurun_out/r4_vsref_timing.jsonl 2> gpurun_out/r4_vsref_timing.err
