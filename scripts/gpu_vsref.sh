#!/bin/bash
# avenir_amd (GPU) vs the reference's CPU library implementations on identical data.
set -eo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u benchmarks/bench_vs_reference.py ${VSREF_ARGS:-} 2>&1 | tee gpurun_out/vsref.log
