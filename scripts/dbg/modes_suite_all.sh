#!/bin/bash
# the GPU suite in the two non-default fp32 GEMM modes, every failure listed (no -x)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
for m in bf16x3 f32; do
  AVMI_F32_GEMM=$m timeout -k 10 700 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/suite_$m.log 2>&1
  echo "$m rc=$?: $(tail -1 gpurun_out/suite_$m.log)"
  grep "^FAILED\|^ERROR" gpurun_out/suite_$m.log | cut -c1-160
done
