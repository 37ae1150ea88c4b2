#!/usr/bin/env python3
"""Per-kernel means of rocprofv3 --pmc counters (counter_collection.csv): one JSON line per kernel
name with the dispatch count and the mean of every collected counter per dispatch."""
import csv
import json
import sys
from collections import defaultdict


def main(path, top=12):
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r.get("Kernel_Name", "?")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    rows = []
    for k, c in acc.items():
        n = max(1, len(disp[k]))
        rows.append({"kernel": k[:90], "dispatches": n, **{name: v / n for name, v in sorted(c.items())}})
    rows.sort(key=lambda d: -d["dispatches"] * d.get("GRBM_GUI_ACTIVE", 1.0))
    for d in rows[:top]:
        print(json.dumps(d))


if __name__ == "__main__":
    main(sys.argv[1])
