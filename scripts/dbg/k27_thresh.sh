#!/bin/bash
# planes path everywhere (min tiles 1) vs never, per mode: where does it pay?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_bert.py > gpurun_out/k27t_tests.log 2>&1 || { tail -30 gpurun_out/k27t_tests.log; exit 1; }
tail -1 gpurun_out/k27t_tests.log
for m in bf16x6 bf16x3; do for p in 1 0; do
  AVMI_F32_GEMM=$m AVMI_SBF16_PLANES=$p AVMI_PLANES_MIN_TILES=1 timeout -k 10 300 python -u benchmarks/bench_gemm_shapes.py > gpurun_out/k27t_${m}_p$p.jsonl 2>&1 || exit 1
done; done
python3 - <<'PY'
import json
for m in ("bf16x6", "bf16x3"):
    rows = {}
    for p in (1, 0):
        for l in open(f"gpurun_out/k27t_{m}_p{p}.jsonl"):
            if l.startswith("{"):
                d = json.loads(l)
                if d.get("op") == "linear_act_fwd" and d["M"] >= 1024:
                    t = -(-d["M"] // 128) * -(-d["N"] // 128)
                    rows.setdefault((d["M"], d["N"], d["K"], t), {})[p] = (round(d["us"], 1), d["us_cached_w"] and round(d["us_cached_w"], 1), round(d["torch_us"], 1))
    for k, v in rows.items(): print(m, k, "planes", v.get(1), "inloop", v.get(0))
PY
