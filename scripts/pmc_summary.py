#!/usr/bin/env python3
"""Summarise scripts/gpu_pmc.sh output: one JSON line per (target, hand-written kernel) with the
mean duration (kernel-trace run), mean counters per dispatch (pmc runs) and derived roofline
numbers.  FETCH_SIZE on gfx950 reports half the bytes of a wide coalesced stream
(MI355X_MICROARCH.md), so both the raw and the doubled read estimate are given."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

OURS = re.compile(r"\(anonymous namespace\)::(\w+)|^(\w+_kernel)\b")


def kname(s):
    m = OURS.search(s)
    return (m.group(1) or m.group(2)) if m else None


def main(root):
    for tdir in sorted(d for d in glob.glob(os.path.join(root, "*")) if os.path.isdir(d)):
        target = os.path.basename(tdir)
        dur = defaultdict(list)
        for f in glob.glob(os.path.join(tdir, "**", "trace_kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = kname(r["Kernel_Name"])
                if k:
                    dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9)
        ctr = defaultdict(lambda: defaultdict(float))
        nd = defaultdict(lambda: defaultdict(set))
        for f in glob.glob(os.path.join(tdir, "**", "*_counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = kname(r["Kernel_Name"])
                if not k:
                    continue
                c = r["Counter_Name"]
                ctr[k][c] += float(r["Counter_Value"])
                nd[k][c].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
        for k in sorted(set(dur) | set(ctr), key=lambda x: -sum(dur.get(x, [0]))):
            d = dur.get(k, [])
            t = sum(d) / len(d) if d else None
            per = {c: v / max(1, len(nd[k][c])) for c, v in ctr[k].items()}
            out = {"target": target, "kernel": k, "dispatches": len(d), "mean_ms": t * 1e3 if t else None,
                   "counters_per_dispatch": per}
            der = {}
            if t and "FETCH_SIZE" in per:
                der["fetch_GBps_raw"] = per["FETCH_SIZE"] * 1024 / t / 1e9
                der["fetch_GBps_x2"] = 2 * der["fetch_GBps_raw"]
            if t and "WRITE_SIZE" in per:
                der["write_GBps"] = per["WRITE_SIZE"] * 1024 / t / 1e9
            if per.get("SQ_WAVES"):
                der["valu_insts_per_wave"] = per.get("SQ_INSTS_VALU", 0) / per["SQ_WAVES"]
            if per.get("SQ_WAVE_CYCLES"):
                der["valu_active_frac_of_wave_cycles"] = per.get("SQ_ACTIVE_INST_VALU", 0) / per["SQ_WAVE_CYCLES"]
            if per.get("SQ_INSTS_LDS"):
                der["lds_bank_conflict_cycles_per_lds_inst"] = per.get("SQ_LDS_BANK_CONFLICT", 0) / per["SQ_INSTS_LDS"]
            if t and per.get("GRBM_GUI_ACTIVE"):
                der["effective_clock_GHz"] = per["GRBM_GUI_ACTIVE"] / 8 / t / 1e9
                # SQ_ACTIVE_INST_VALU counts quad-cycles summed over waves: x4 / (1024 SIMDs x the
                # kernel's cycles per XCD) = fraction of SIMD cycles issuing VALU (1.0 = issue-bound)
                der["valu_busy_per_simd"] = per.get("SQ_ACTIVE_INST_VALU", 0) * 4 / (1024 * per["GRBM_GUI_ACTIVE"] / 8)
            if t and per.get("SQ_VALU_MFMA_BUSY_CYCLES") and per.get("GRBM_GUI_ACTIVE"):
                # MFMA busy cycles summed over 1024 SIMDs vs the kernel's active cycles per XCD
                der["mfma_busy_frac"] = per["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * per["GRBM_GUI_ACTIVE"] / 8)
            hits, miss = per.get("TCC_HIT_sum"), per.get("TCC_MISS_sum")
            if hits is not None and miss is not None and hits + miss > 0:
                der["l2_hit_rate"] = hits / (hits + miss)
            out["derived"] = der
            print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
