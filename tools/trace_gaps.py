#!/usr/bin/env python3
"""Kernel-timeline gap analysis of a rocprofv3 --kernel-trace csv: busy vs idle time of the GPU
between the first and last kernel whose name contains ``--from`` (default: the whole trace),
the distribution of inter-kernel gaps and the largest gaps with the kernels around them."""
import argparse
import csv
import statistics
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--from", dest="start", default="")
    ap.add_argument("--skip", type=int, default=0, help="skip this many matches of --from first")
    ap.add_argument("--to", dest="end", default="", help="stop at the last kernel containing this")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    if a.start:
        idx = [k for k, e in enumerate(ev) if a.start in e[2]]
        if len(idx) <= a.skip:
            sys.exit("no kernel matches")
        ev = ev[idx[a.skip]:]
    if a.end:
        idx = [k for k, e in enumerate(ev) if a.end in e[2]]
        if idx:
            ev = ev[:idx[-1] + 1]
    span = ev[-1][1] - ev[0][0]
    busy = sum(e[1] - e[0] for e in ev)
    gaps = [(ev[k + 1][0] - ev[k][1], ev[k][2][:50], ev[k + 1][2][:50]) for k in range(len(ev) - 1)]
    g = [x[0] for x in gaps]
    print(f"kernels {len(ev)}  span {span / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  idle {(span - busy) / 1e6:.3f} ms")
    if g:
        q = statistics.quantiles(g, n=20)
        print(f"gap us: median {statistics.median(g) / 1e3:.2f}  p5 {q[0] / 1e3:.2f}  p95 {q[-1] / 1e3:.2f}  "
              f"max {max(g) / 1e3:.1f}")
        by = {}
        for gg, _, y in gaps:
            t = by.setdefault(y, [0, 0])
            t[0] += gg
            t[1] += 1
        print("idle before each kernel (total ms, count, mean us):")
        for y, (tot, n) in sorted(by.items(), key=lambda kv: -kv[1][0])[:8]:
            print(f"  {tot / 1e6:8.3f} {n:6d} {tot / n / 1e3:7.2f}  {y}")
        for gg, x, y in sorted(gaps, reverse=True)[:12]:
            print(f"  {gg / 1e3:9.1f} us  {x}  ->  {y}")


if __name__ == "__main__":
    main()
