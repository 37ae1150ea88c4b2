#!/bin/bash
# the GPU suite in the two non-default fp32 GEMM modes (default x6 is the round-end run)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
for m in bf16x3 f32; do
  AVMI_F32_GEMM=$m timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/suite_$m.log 2>&1 \
    || { tail -40 gpurun_out/suite_$m.log; exit 1; }
  echo "$m: $(tail -1 gpurun_out/suite_$m.log)"
done
