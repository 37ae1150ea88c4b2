#!/bin/bash
# K27 pre-split planes path: GPU tests, then the shape sweep with the path on / off (x6, x3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm.py tests/test_bert.py tests/test_nn.py tests/test_nn_graphs.py tests/test_rnn.py \
  > gpurun_out/k27_planes_tests.log 2>&1 || { tail -30 gpurun_out/k27_planes_tests.log; exit 1; }
tail -1 gpurun_out/k27_planes_tests.log
for m in bf16x6 bf16x3; do for p in 1 0; do
  AVMI_F32_GEMM=$m AVMI_SBF16_PLANES=$p timeout -k 10 300 python -u benchmarks/bench_gemm_shapes.py > gpurun_out/k27_planes_${m}_p$p.jsonl 2>&1 || exit 1
done; done
python3 - <<'PY'
import json
for m in ("bf16x6", "bf16x3"):
    rows = {}
    for p in (1, 0):
        for l in open(f"gpurun_out/k27_planes_{m}_p{p}.jsonl"):
            if l.startswith("{"):
                d = json.loads(l)
                if d.get("op") == "linear_act_fwd" and d["M"] * d["N"] >= 1 << 21:
                    rows.setdefault((d["M"], d["N"], d["K"]), {})[p] = (round(d["us"], 1), d["us_cached_w"] and round(d["us_cached_w"], 1), round(d["torch_us"], 1), d.get("err_fp64"))
    for k, v in rows.items(): print(m, k, "planes", v.get(1), "inloop", v.get(0))
PY
for g in bf16x3 bf16x6; do for p in 1 0; do
  AVMI_BERT_GEMM=$g AVMI_SBF16_PLANES=$p timeout -k 10 300 python -u benchmarks/bench_bert.py > gpurun_out/k27_bert_${g}_p$p.jsonl 2>&1 || exit 1
  grep '"B"' gpurun_out/k27_bert_${g}_p$p.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('bert', '$g', 'planes=$p', d['B'], d['S'], round(d['ours_ms'], 3), round(d['transformers_ms'], 3), round(d['speedup'], 2), d['max_abs_diff'])"
done; done
