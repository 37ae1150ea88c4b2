"""Command-line entry point: one sub-command per reference job / driver operation.

    python -m avenir_amd <job> --input IN --output OUT [--config CONF] [--app APP] [--schema SCHEMA]
                         [-D key=value ...]

Reference drivers: the Hadoop jobs run as ``<main class> -Dconf.path=<props> in out`` and the
Spark jobs as ``<object> in out <hocon>`` (``getCommandLineArgs(args, 3)``, e.g.
S/util/LinearMapper.scala:40-99); the shell drivers in R/*.sh chain them (detr, rafo,
knn, conv, carm, fit, hica, ovsa, caen, dvg, ks, str/sup, opt, wc); the Python drivers take
``mode config`` (P/app/rfd.py, svmd.py, gb.py).  Here every job runs in-process on the device.
Launched under ``torchrun`` (one process per GPU), each rank reads its shard of the input, the
reductions are RCCL collectives, map-side jobs write one ``part-NNNNN`` per rank into a directory
output (or gather to rank 0 for a single-file output) and reducing jobs write from rank 0
(jobs/common.py).  Outputs keep the reference's line formats where one exists.
"""
from __future__ import annotations

import argparse
import sys

from .jobs import JOBS  # noqa: F401  (registers every job)


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="avenir_amd", description=__doc__.split("\n\n")[0])
    ap.add_argument("job", nargs="?", help="job name (see --list)")
    ap.add_argument("rest", nargs="*", help="positional arguments of an app driver verb (e.g. ctrace simu 1000 y)")
    ap.add_argument("--list", action="store_true")
    ap.add_argument("--input", "-i")
    ap.add_argument("--output", "-o")
    ap.add_argument("--config", "-c")
    ap.add_argument("--app", help="HOCON block name")
    ap.add_argument("--schema")
    ap.add_argument("--model")
    ap.add_argument("--train")
    ap.add_argument("--domain")
    ap.add_argument("--device")
    ap.add_argument("--kind")
    ap.add_argument("--mode")
    ap.add_argument("--name")
    ap.add_argument("--port", type=int, default=5000)
    ap.add_argument("--k")
    ap.add_argument("--gen-args", help="comma-separated generator arguments (genData)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("-D", "--define", action="append", default=[], metavar="KEY=VALUE",
                    help="config override (Hadoop -D), repeatable")
    return ap


def main(argv: list[str] | None = None) -> int:
    args = build_parser().parse_intermixed_args(argv)
    if args.list or not args.job:
        for n, (_, h) in sorted(JOBS.items()):
            print(f"{n:36s} {h}")
        return 0
    if args.job not in JOBS:
        print(f"unknown job {args.job}; use --list", file=sys.stderr)
        return 2
    JOBS[args.job][0](args)
    return 0


if __name__ == "__main__":
    from . import freeze_startup_objects
    freeze_startup_objects()
    sys.exit(main())
