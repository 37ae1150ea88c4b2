"""End-to-end (file -> output file) timings of the prediction / sequence jobs that moved onto
native input and output in round 4: viterbiStatePredictor,
markovModelClassifier, probabilisticSuffixTreeGenerator (K5), bayesianPredictor, decisionTree
level mode, modelPredictor.  Each job runs in-process on ``--records`` records (default 2^24) of a
synthetic file of its reference layout; models are trained once beforehand (untimed); the best
of ``--reps`` runs is reported as records/s, one JSON line per job.

    python benchmarks/bench_predict_jobs.py [--records N] [--jobs vit,mmc,...] [--out file]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from avenir_amd.cli import main as cli  # noqa: E402
from avenir_amd.data import synth  # noqa: E402
from avenir_amd.data import synth_text as S  # noqa: E402


def _run(args):
    assert cli([str(a) for a in args]) == 0


def _props(d, name, text):
    p = os.path.join(d, name)
    with open(p, "w") as fh:
        fh.write(text)
    return p


def setup(job: str, d: str, n: int, dev: str):
    """(argv without -o, input path) for ``job``; trains its model (untimed)."""
    if job == "vit":
        tagged = os.path.join(d, "tagged.txt")
        S.tagged_sequences(tagged, min(n, 1 << 20), seed=3)
        cfg = _props(d, "hmm.properties", "hmmb.model.states=S,T,U\nhmmb.model.observations=a,b,c,d\n"
                                          "hmmb.skip.field.count=1\nhmmb.trans.prob.scale=1000\n")
        model = os.path.join(d, "hmm.txt")
        _run(["hiddenMarkovModelBuilder", "-i", tagged, "-o", model, "-c", cfg, "--device", dev])
        data = os.path.join(d, "obs.txt")
        S.observation_sequences(data, n, seed=4)
        return ["viterbiStatePredictor", "-i", data, "--model", model, "-c",
                _props(d, "vit.properties", "vsp.skip.field.count=1\n")], data
    if job in ("mmc", "pst"):
        data = os.path.join(d, "seq.txt")
        if not os.path.exists(data):
            S.state_sequences(data, n, seed=5)
        if job == "pst":
            return ["probabilisticSuffixTreeGenerator", "-i", data, "-c",
                    _props(d, "pst.properties", "pstg.skip.field.count=1\npstg.class.label.field.ord=1\n"
                                                "pstg.max.seq.length=5\n")], data
        cfg = _props(d, "mmc.properties", "mst.model.states=" + ",".join(S.STATES) + "\nmst.skip.field.count=2\n"
                     "mst.class.label.field.ord=1\nmst.class.labels=T,F\nmmc.class.labels=T,F\n"
                     "mmc.skip.field.count=2\nmmc.validation.mode=true\nmmc.class.label.field.ord=1\n")
        model = os.path.join(d, "mm.txt")
        _run(["markovStateTransitionModel", "-i", data, "-o", model, "-c", cfg, "--device", dev])
        return ["markovModelClassifier", "-i", data, "--model", model, "-c", cfg], data
    data, schema = os.path.join(d, "churn.csv"), os.path.join(d, "churn.json")
    if not os.path.exists(data):
        synth.write_churn_native(data, n, seed=6)
        with open(schema, "w") as fh:
            json.dump(synth.CHURN_SCHEMA, fh)
    if job == "nbp":
        model = os.path.join(d, "nb.txt")
        _run(["bayesianDistribution", "-i", data, "-o", model, "--schema", schema, "--device", dev])
        return ["bayesianPredictor", "-i", data, "--schema", schema, "--model", model], data
    if job == "detr":
        return ["decisionTree", "-i", data, "--schema", schema, "-c",
                _props(d, "detr.properties", "dtb.split.algorithm=giniIndex\ndtb.path.stopping.strategy=maxDepth\n"
                       f"dtb.max.depth.limit=3\ndtb.decision.file.path.out={os.path.join(d, 'dp.json')}\n")], data
    if job == "mop":
        forest = os.path.join(d, "forest")
        cfg = _props(d, "mop.properties", f"dtb.feature.schema.file.path={schema}\ndtb.split.algorithm=giniIndex\n"
                     "dtb.path.stopping.strategy=maxDepth\ndtb.max.depth.limit=4\ndtb.num.trees=5\n"
                     f"mop.model.dir.path={forest}\nmop.output.mode=withActualClassAttr\nmop.rec.id.ordinal=0\n"
                     "mop.rec.class.attr.ordinal=6\n")
        _run(["randomForest", "-i", data, "-o", forest, "-c", cfg, "--device", dev])
        return ["modelPredictor", "-i", data, "-c", cfg], data
    if job == "usb":
        return ["underSamplingBalancer", "-i", data, "-c", _props(d, "usb.properties", "usb.class.attr.ord=6\n")], data
    if job in ("hash", "dummy"):
        block = ("categoricalFeatureHashingEncoding { cat.fieldOrdinals = [1,2,3]\n encoding.size = 8 }\n"
                 if job == "hash" else "binaryDummyVariableGenerator { cat.field.ordinals = [1,4] }\n")
        return [block.split()[0], "-i", data, "-c", _props(d, f"{job}.conf", block)], data
    raise SystemExit(f"unknown job {job}")


def setup_fcb(d: str, n: int):
    """featureCondProbJoiner on ``n`` distance pairs (``trainId,testId,dist,trainCls,testCls``;
    4,096 training records x n / 4,096 test records) plus a 4,096-line posterior file."""
    import numpy as np
    ntr = 4096
    nte = max(1, n // ntr)
    rng = np.random.default_rng(7)
    pdir = os.path.join(d, "fcb_in")
    os.makedirs(pdir, exist_ok=True)
    cls = ["pass", "fail"]
    with open(os.path.join(pdir, "prDistr-00000"), "w") as fh:
        for t in range(ntr):
            p = rng.random()
            fh.write(f"T{t},{rng.random():.4f},pass,{p:.6f},fail,{1 - p:.6f},{cls[t % 2]}\n")
    head = [f"T{t}," for t in range(ntr)]
    tail = [f",{cls[t % 2]}," for t in range(ntr)]
    with open(os.path.join(pdir, "part-00000"), "w") as fh:
        for q in range(nte):
            dist = rng.integers(0, 100000, ntr).tolist()
            qs = f"Q{q},"
            qc = cls[q % 2] + "\n"
            fh.write("".join(h + qs + str(v) + tl + qc for h, v, tl in zip(head, dist, tail)))
    cfg = _props(d, "fcb.properties", "fcb.feature.cond.prob.split.prefix=prDistr\n")
    return ["featureCondProbJoiner", "-i", pdir, "-c", cfg], os.path.join(pdir, "part-00000")


def setup_rs(d: str, n: int):
    """recordSimilarity on ``n`` records x 8 uniform dims: the all-pairs ring
    with a distance threshold that keeps ~1e-4 of the pairs."""
    import numpy as np
    data = os.path.join(d, f"rs_{n}.csv")
    rng = np.random.default_rng(3)
    X = rng.random((n, 8))
    with open(data, "w") as fh:
        for i in range(0, n, 65536):
            blk = X[i:i + 65536]
            fh.write("\n".join(f"r{i + j}," + ",".join(f"{v:.5f}" for v in row) for j, row in enumerate(blk)) + "\n")
    cfg = _props(d, "rs.properties", "resi.attr.ordinals=1,2,3,4,5,6,7,8\nresi.id.ordinal=0\n"
                                     "resi.distance.scale=1000\nresi.dist.threshold=100\n")
    return ["recordSimilarity", "-i", data, "-c", cfg], data


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 24)
    ap.add_argument("--jobs", default="vit,mmc,pst,nbp,detr,mop")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--rs-records", type=int, default=1 << 17)
    ap.add_argument("--dir", default=None, help="directory of the input / output files (default: a temp dir)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    d = tempfile.mkdtemp(prefix="avmi_pred_", dir=args.dir)
    for job in args.jobs.split(","):
        n_rec = args.rs_records if job == "rs" else args.records
        if job == "rs":
            argv, data = setup_rs(d, n_rec)
        elif job == "fcb":
            argv, data = setup_fcb(d, n_rec)
        else:
            argv, data = setup(job, d, args.records, dev)
        best = None
        for rep in range(args.reps):
            # a fresh output path per run (a job writes a new output; re-using one would time the
            # truncation of the previous run's file)
            out = os.path.join(d, f"{job}.{rep}.out")
            if dev == "cuda":
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            _run(argv + ["-o", out, "--device", dev])
            if dev == "cuda":
                torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
            if rep + 1 < args.reps:
                import shutil
                shutil.rmtree(out, ignore_errors=True) if os.path.isdir(out) else os.remove(out)
        files = [out] if os.path.isfile(out) else [os.path.join(out, f) for f in sorted(os.listdir(out))]
        n_out = 0
        for fn in files:
            with open(fn, "rb") as fh:
                n_out += sum(1 for _ in fh)
        rec = {"bench": "predict_job", "job": argv[0], "records": n_rec, "device": dev, "dir": os.path.dirname(d),
               "bytes": os.path.getsize(data), "seconds": round(best, 4), "records_per_s": n_rec / best,
               "output_lines": n_out}
        if job == "rs":
            rec["pairs_per_s"] = n_rec * (n_rec - 1) / 2 / best
        print(json.dumps(rec), flush=True)
        for fn in files:
            os.remove(fn)
        if args.out:
            with open(args.out, "a") as fh:
                fh.write(json.dumps(rec) + "\n")
    import shutil
    shutil.rmtree(d, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
