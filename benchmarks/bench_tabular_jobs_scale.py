#!/usr/bin/env python3
"""End-to-end (file -> output file) time of the tabular counting jobs (tests/test_gpu_jobs.py's
commands: bayesianDistribution, cramerCorrelation, mutualInformation) on a churn-schema CSV of
``--rows`` records (data/synth.write_churn_native), warm process.  One JSON line per job."""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time
from pathlib import Path

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from avenir_amd.cli import main  # noqa: E402
from avenir_amd.data import synth  # noqa: E402


def main_(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 22)
    ap.add_argument("--device", default="cuda")
    args = ap.parse_args(argv)
    tmp = Path(tempfile.mkdtemp(prefix="avmi_tab_scale_"))
    try:
        data, schema = tmp / "churn.csv", tmp / "churn.json"
        synth.write_churn(tmp / "small.csv", 10, seed=3, schema_path=schema)
        nbytes = synth.write_churn_native(str(data), args.rows, seed=3)
        sj = json.loads(schema.read_text())
        ords = [f["ordinal"] for f in sj["fields"] if f.get("feature") and f.get("dataType") == "categorical"][:3]
        props = tmp / "p.properties"
        props.write_text(f"crc.feature.schema.file.path={schema}\ncrc.source.attributes={ords[0]}\n"
                         f"crc.dest.attributes={','.join(map(str, ords[1:]))}\n")
        jobs = {"bayesianDistribution": ["--schema", str(schema)], "cramerCorrelation": ["-c", str(props)],
                "mutualInformation": ["--schema", str(schema)]}
        # the model builders on the call-hangup schema (tests/test_cli.py's configurations)
        hdata, hschema = tmp / "hangup.csv", tmp / "hangup.json"
        hdata.write_text("\n".join(synth.call_hangup_lines(args.rows // 4, seed=2)) + "\n")
        hschema.write_text(json.dumps(synth.CALL_HANGUP_SCHEMA))
        tcfg = tmp / "detr.properties"
        tcfg.write_text("dtb.split.algorithm=giniIndex\ndtb.path.stopping.strategy=maxDepth\ndtb.max.depth.limit=2\n"
                        "dtb.num.trees=3\n")
        lcfg = tmp / "lr.properties"
        lcfg.write_text("lor.iteration.limit=5\nlor.positive.class.value=T\n")
        for job, cfg in (("decisionTree", tcfg), ("randomForest", tcfg), ("logisticRegression", lcfg)):
            times = []
            for rep in range(2):
                t0 = time.perf_counter()
                assert main([job, "-i", str(hdata), "-o", str(tmp / f"{job}{rep}"), "-c", str(cfg), "--schema",
                             str(hschema), "--device", args.device]) == 0
                times.append(time.perf_counter() - t0)
            print(json.dumps({"bench": "tabular_job_scale", "job": job, "rows": args.rows // 4,
                              "file_bytes": os.path.getsize(hdata), "cold_s": times[0], "warm_s": times[1],
                              "rows_per_s": (args.rows // 4) / times[1]}), flush=True)
        for job, extra in jobs.items():
            times = []
            for rep in range(2):
                t0 = time.perf_counter()
                assert main([job, "-i", str(data), "-o", str(tmp / f"{job}{rep}.txt"), "--device", args.device]
                            + extra) == 0
                times.append(time.perf_counter() - t0)
            print(json.dumps({"bench": "tabular_job_scale", "job": job, "rows": args.rows, "file_bytes": nbytes,
                              "cold_s": times[0], "warm_s": times[1], "rows_per_s": args.rows / times[1]}), flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(main_())
