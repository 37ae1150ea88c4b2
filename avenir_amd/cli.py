"""Command-line entry point: one sub-command per reference job / driver operation.

    python -m avenir_amd <job> --input IN --output OUT [--config CONF] [--app APP] [--schema SCHEMA] ...

Reference drivers: the Hadoop / Spark jobs are launched as ``<main class> input output config``
(``getCommandLineArgs(args, 3)``, e.g. S/util/LinearMapper.scala:40-99) and chained by the shell
drivers in R/*.sh (§2.27 of the survey: detr, rafo, knn, conv, carm, fit, hica, ovsa, caen, dvg,
ks, str/sup, opt, wc); the Python drivers take ``mode config`` (P/app/rfd.py, svmd.py, gb.py).
Here every job runs in-process on the device; with ``torchrun`` each rank reads its shard of the
input and the collectives are RCCL (``--gpus N`` wraps the job in torch.distributed.run).
Outputs keep the reference's line formats where one exists.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path
from typing import Callable

import torch

JOBS: dict[str, tuple[Callable, str]] = {}


def job(name: str, help_: str):
    def deco(fn):
        JOBS[name] = (fn, help_)
        return fn
    return deco


def _device(args):
    if args.device:
        return torch.device(args.device)
    return torch.device("cuda" if torch.cuda.is_available() else "cpu")


def _cfg(args, prefix: str = ""):
    from .utils.config import JobConfig
    if not args.config:
        return JobConfig({}, prefix)
    return JobConfig.from_file(args.config, prefix, args.app)


def _schema(args, cfg=None):
    from .utils.schema import FeatureSchema
    path = args.schema or (cfg.get_str("feature.schema.file.path", None) if cfg is not None else None)
    if not path:
        raise SystemExit("a feature schema is required (--schema or feature.schema.file.path)")
    return FeatureSchema.from_json(Path(path))


def _write(args, lines):
    out = Path(args.output)
    if out.suffix == "" and not out.exists():
        out.mkdir(parents=True, exist_ok=True)
    target = out / "part-00000" if out.is_dir() else out
    target.write_text("\n".join(lines) + ("\n" if lines else ""))
    return target


def _lines(path: str) -> list[str]:
    p = Path(path)
    files = sorted(f for f in p.iterdir() if f.is_file() and not f.name.startswith(".")) if p.is_dir() else [p]
    out = []
    for f in files:
        out += [l for l in f.read_text().splitlines() if l.strip()]
    return out


def _table(args, cfg, raw_numeric: bool = False):
    from .data.table import load_csv
    from .parallel.comm import get_comm
    comm = get_comm()
    return load_csv(args.input, _schema(args, cfg), cfg.field_delim_in, rank=comm.rank, world=comm.world,
                    device=_device(args), keep_lines=True, raw_numeric=raw_numeric)


# ================================================================================================
# Bayesian / trees / kNN / linear
# ================================================================================================
@job("bayesianDistribution", "naive Bayes training (BayesianDistribution): CSV -> model lines")
def _nb_train(args):
    from .models.bayes import NaiveBayes
    cfg = _cfg(args, "bad.")
    t = _table(args, cfg)
    nb = NaiveBayes(t.schema).fit(t)
    _write(args, nb.model_lines(cfg.field_delim_out))


@job("bayesianPredictor", "naive Bayes prediction (BayesianPredictor): CSV + --model -> record,class,prob")
def _nb_predict(args):
    from .models.bayes import NaiveBayes
    cfg = _cfg(args, "bap.")
    t = _table(args, cfg)
    nb = NaiveBayes.load_model(args.model or cfg.get_str("bayesian.model.file.path"), t.schema)
    r = nb.predict(t)
    vals = t.class_field.cardinality if t.class_field else None
    d = cfg.field_delim_out
    pred = r.pred.cpu().tolist()
    prob = r.prob.max(1).values.cpu().tolist() if r.prob is not None else [1.0] * len(pred)
    lines = [f"{t.lines[i]}{d}{vals[p] if vals else p}{d}{prob[i]:.3f}" for i, p in enumerate(pred)]
    _write(args, lines)
    if r.confusion is not None:
        print(json.dumps({"confusion": r.confusion.cpu().tolist()}))


@job("decisionTree", "decision tree (DecisionTreeBuilder, dtb.* keys) -> decision path JSON")
def _dec_tree(args):
    from .models.tree import DecisionTreeBuilder, TreeParams
    cfg = _cfg(args, "dtb.")
    t = _table(args, cfg, raw_numeric=True)
    tree = DecisionTreeBuilder(t.schema, TreeParams.from_config(cfg)).fit(t)
    Path(args.output).write_text(json.dumps(tree.to_decision_paths(t.n), indent=1))


@job("randomForest", "random forest of decision trees (rafo driver) -> one JSON per tree")
def _rafo(args):
    from .models.tree import RandomForest, TreeParams
    cfg = _cfg(args, "dtb.")
    t = _table(args, cfg, raw_numeric=True)
    p = TreeParams.from_config(cfg)
    p.sub_sampling = cfg.get_str("sub.sampling.strategy", "withReplace")
    rf = RandomForest(t.schema, cfg.get_int("num.trees", 10), p, cfg.get_str("max.features", "sqrt")).fit(t)
    out = Path(args.output)
    out.mkdir(parents=True, exist_ok=True)
    for i, tr in enumerate(rf.trees):
        (out / f"tree_{i}.json").write_text(json.dumps(tr.to_decision_paths(t.n)))


@job("knnClassifier", "kNN classification (NearestNeighbor, nen.* keys): --input test --train train CSV")
def _knn(args):
    from .data.table import load_csv
    from .models.knn import NearestNeighbor
    cfg = _cfg(args, "nen.")
    schema = _schema(args, cfg)
    dev = _device(args)
    tr = load_csv(args.train, schema, cfg.field_delim_in, device=dev, raw_numeric=True)
    te = load_csv(args.input, schema, cfg.field_delim_in, device=dev, keep_lines=True, raw_numeric=True)
    Xtr, Xte = tr.dense_features(one_hot=True), te.dense_features(one_hot=True)
    lo, hi = Xtr.min(0).values, Xtr.max(0).values
    scale = (hi - lo).clamp_min(1e-12)
    nn = NearestNeighbor.from_config(cfg).fit((Xtr - lo) / scale, tr.labels[: tr.n].long(), tr.n_classes)
    res = nn.predict((Xte - lo) / scale)
    vals = te.class_field.cardinality
    d = cfg.field_delim_out
    _write(args, [f"{te.lines[i]}{d}{vals[p]}" for i, p in enumerate(res.pred.cpu().tolist())])


@job("logisticRegression", "logistic regression (LogisticRegressionJob): CSV -> coefficient lines per iteration")
def _logit(args):
    from .models.linear import LogisticRegression
    cfg = _cfg(args, "lor.")
    t = _table(args, cfg, raw_numeric=True)
    X = t.dense_features()
    m = LogisticRegression(solver=cfg.get_str("solver", "newton"), max_iter=cfg.get_int("iteration.limit", 10),
                           criteria=cfg.get_str("convergence.criteria", "iterLimit"),
                           threshold=cfg.get_float("convergence.threshold", 5.0))
    pos = cfg.get_str("positive.class.value", None)
    vals = t.class_field.cardinality
    y = (t.labels[: t.n].long() == (vals.index(pos) if pos in vals else 1)).float()
    m.fit(X, y)
    _write(args, m.coefficient_lines(cfg.field_delim_out))


# ================================================================================================
# exploration / encoding / sampling
# ================================================================================================
@job("mutualInformation", "mutual information feature scores (MutualInformation, mut.* keys)")
def _mi(args):
    from .models.explore import MutualInformation
    cfg = _cfg(args, "mut.")
    t = _table(args, cfg)
    mi = MutualInformation()
    mi.fit(t)
    alg = cfg.get_str("mutual.info.score.algorithms", "mutual.info.maximization").split(",")
    lines = []
    fns = {"mutual.info.maximization": mi.mim, "mutual.info.selection": mi.mifs, "joint.mutual.info": mi.jmi,
           "double.input.symmetrical.relevance": mi.disr, "min.redundancy.max.relevance": mi.mrmr}
    for a in alg:
        if a in fns:
            lines.append(a)
            lines += [f"{f},{s:.6f}" for f, s in fns[a]()]
    _write(args, lines)


@job("categoricalClassAffinity", "class affinity of categorical values (CategoricalClassAffinity)")
def _caff(args):
    from .models.explore import class_affinity
    cfg = _cfg(args, "cca.")
    t = _table(args, cfg)
    res = class_affinity(t, cfg.get_str("affinity.strategy", "oddsRatio"))
    lines = []
    for ordinal, vals in (res.items() if isinstance(res, dict) else []):
        for v, s in (vals.items() if isinstance(vals, dict) else []):
            lines.append(f"{ordinal},{v},{s:.6f}")
    _write(args, lines)


@job("categoricalContinuousEncoding", "supervised ratio / weight-of-evidence encoding (hica driver)")
def _hica(args):
    from .models.explore import supervised_encoding
    cfg = _cfg(args, "cce.")
    t = _table(args, cfg)
    enc = supervised_encoding(t, cfg.get_str("encoding.strategy", "supervisedRatio"),
                              cfg.get_int("output.scale", 1000))
    _write(args, [f"{o},{v},{s}" for o, m in enc.items() for v, s in m.items()])


@job("frequentItemsApriori", "Apriori frequent item sets (fit driver): one transaction per line")
def _apriori(args):
    from .models.association import Apriori
    cfg = _cfg(args, "fia.")
    d = cfg.field_delim_in
    skip = cfg.get_int("skip.field.count", 1)
    tx = [l.split(d)[skip:] for l in _lines(args.input)]
    ap = Apriori(cfg.get_float("support.threshold", 0.1), cfg.get_int("max.item.set.length", 4))
    fi = ap.fit_transactions(tx, device=_device(args))
    lines = []
    for k in range(1, ap.max_len + 1):
        for names, sup in fi.as_names(k):
            lines.append(cfg.field_delim_out.join(names) + f"{cfg.field_delim_out}{sup:.6f}")
    _write(args, lines)


@job("classBasedOverSampler", "SMOTE over-sampling of the minority class (ovsa driver)")
def _smote(args):
    from .models.sampling import smote
    cfg = _cfg(args, "cbos.")
    t = _table(args, cfg, raw_numeric=True)
    X = t.dense_features()
    y = t.labels[: t.n].long()
    minority = int(torch.bincount(y).argmin())
    n_new = int((y != minority).sum() - (y == minority).sum())
    Xn, _ = smote(X, y, minority, max(n_new, 0), cfg.get_int("neighbor.count", 5))
    vals = t.class_field.cardinality
    d = cfg.field_delim_out
    _write(args, [d.join(f"{v:.4f}" for v in row) + f"{d}{vals[minority]}" for row in Xn.cpu().tolist()])


@job("kolmogorovSmirnovModelDrift", "KS drift between reference and current numeric distributions")
def _ks(args):
    from .models.explore import kolmogorov_smirnov_drift, numeric_histogram
    cfg = _cfg(args, "ksd.")
    d = cfg.field_delim_in
    col = cfg.get_int("attr.ordinal", 0)
    ref = torch.tensor([float(l.split(d)[col]) for l in _lines(args.train)], dtype=torch.float64)
    cur = torch.tensor([float(l.split(d)[col]) for l in _lines(args.input)], dtype=torch.float64)
    bw = cfg.get_float("bin.width", float((ref.max() - ref.min()) / 50 or 1))
    lo = float(min(ref.min(), cur.min()))
    nb = int((float(max(ref.max(), cur.max())) - lo) / bw) + 1
    stat, crit, drift = kolmogorov_smirnov_drift(numeric_histogram(ref, bw, lo, nb), numeric_histogram(cur, bw, lo, nb))
    _write(args, [f"{col},{stat:.6f},{crit:.6f},{drift}"])


# ================================================================================================
# sequences / Markov
# ================================================================================================
@job("markovStateTransitionModel", "Markov transition probabilities per class (conv driver)")
def _markov(args):
    from .models.markov import MarkovStateTransitionModel
    cfg = _cfg(args, "mst.")
    d = cfg.field_delim_in
    states = cfg.get_str("model.states").split(",")
    skip = cfg.get_int("skip.field.count", 1)
    cls_ord = cfg.get_int("class.label.field.ordinal", -1)
    rows = [l.split(d) for l in _lines(args.input)]
    seqs = [r[skip:] if cls_ord < 0 else [v for i, v in enumerate(r) if i >= skip and i != cls_ord] for r in rows]
    m = MarkovStateTransitionModel(states, cfg.get_int("trans.prob.scale", 1000))
    enc = m.encode(seqs)
    labels = None
    if cls_ord >= 0:
        cl = sorted({r[cls_ord] for r in rows})
        m.class_labels = cl
        labels = torch.tensor([cl.index(r[cls_ord]) for r in rows])
    m.fit(enc, labels)
    _write(args, m.model_lines(cfg.field_delim_out))


@job("viterbiStatePredictor", "HMM state sequence per observation sequence (J/markov/ViterbiStatePredictor.java); --model <HMM lines>")
def _viterbi(args):
    """Rows ``id,obs,obs,...`` -> ``id,state,state,...`` (a token outside the model's observations
    ends the sequence).  vsp.skip.field.count (default 1) leading fields are copied through."""
    from .models.markov import HiddenMarkovModel, ViterbiDecoder
    cfg = _cfg(args, "vsp.")
    d = cfg.field_delim_in
    skip = cfg.get_int("skip.field.count", 1)
    hmm = HiddenMarkovModel.from_lines(_lines(args.model), d)
    rows = [l.split(d) for l in _lines(args.input)]
    oi = {o: i for i, o in enumerate(hmm.observations)}
    obs = torch.full((len(rows), max([len(r) - skip for r in rows] + [1])), -1, dtype=torch.int16)
    for r, row in enumerate(rows):
        for j, tok in enumerate(row[skip:]):
            obs[r, j] = oi.get(tok, -1)
    paths = ViterbiDecoder(hmm).decode_labels(obs.to(_device(args)))
    _write(args, [d.join(row[:skip] + p) for row, p in zip(rows, paths)])


@job("genData", "tutorial fixture generator: --name <P/app script> --gen-args a,b,c [--seed s] (data/fixtures.py)")
def _gen_data(args):
    from .data.fixtures import FIXTURES

    def num(v):
        for t in (int, float):
            try:
                return t(v)
            except ValueError:
                pass
        return v
    if args.name not in FIXTURES:
        raise SystemExit(f"unknown fixture {args.name}; one of {', '.join(sorted(FIXTURES))}")
    gargs = [num(v) for v in args.gen_args.split(",")] if args.gen_args else []
    out = FIXTURES[args.name](*gargs, seed=args.seed)
    lines = out[0] if isinstance(out, tuple) else out
    if args.output:
        _write(args, lines)
    else:
        sys.stdout.write("\n".join(lines) + "\n")


@job("wordCount", "word count sanity job")
def _wc(args):
    from collections import Counter
    c = Counter(w for l in _lines(args.input) for w in l.split())
    _write(args, [f"{w},{n}" for w, n in sorted(c.items())])


# ================================================================================================
# optimisation / clustering / bandits
# ================================================================================================
@job("simulatedAnnealing", "SA over a task-schedule domain (R/opt.conf block simulatedAnnealing)")
def _sa(args):
    from .optimize import SimulatedAnnealing, TaskScheduleSearch
    args.app = args.app or "simulatedAnnealing"
    cfg = _cfg(args)
    dom_file = args.domain or cfg.get_str("domain.callback.config.file")
    if not Path(dom_file).exists() and args.config:
        dom_file = str(Path(args.config).parent / dom_file)
    d = TaskScheduleSearch.from_json(dom_file, _device(args))
    r = SimulatedAnnealing.from_config(d, cfg).run()
    o = cfg.get_str("field.delim.out", ",")
    lines = [f"{d.format_solution(s)}{o}{c:.6f}" for s, c in zip(r.solutions.tolist(), r.costs.tolist())]
    lines.sort(key=lambda l: float(l.rsplit(o, 1)[1]))
    _write(args, lines)
    print(json.dumps({"best_cost": r.best_cost, **r.stats}))


@job("kmeansCluster", "k-means over numeric columns; --k list of cluster counts; knuckle-point k")
def _kmeans(args):
    from .models.cluster import KMeans
    cfg = _cfg(args, "kmc.")
    d = cfg.field_delim_in
    cols = [int(c) for c in cfg.get_str("attr.ordinals", "0").split(",")]
    X = torch.tensor([[float(l.split(d)[c]) for c in cols] for l in _lines(args.input)], device=_device(args))
    ks = [int(k) for k in (args.k or cfg.get_str("num.clusters", "3")).split(",")]
    km = KMeans(ks, n_init=cfg.get_int("num.init.groups", 3), max_iter=cfg.get_int("max.iterations", 100)).fit(X)
    lines = []
    for k in ks:
        run = km.best[k]
        lines += [f"{k},{i}," + ",".join(f"{v:.4f}" for v in c) for i, c in enumerate(run.centroids.cpu().tolist())]
        lines.append(f"{k},sse,{run.sse:.4f}")
    if len(ks) > 2:
        lines.append(f"knuckle,{km.knuckle_k()}")
    _write(args, lines)


@job("multiArmBandit", "batch bandit per group (MultiArmBandit Spark job): rewards in, actions out")
def _mab(args):
    from .models.bandit import BanditBank
    cfg = _cfg(args)
    d = cfg.get_str("field.delim.in", ",")
    actions = cfg.get_str("action.list").split(",")
    rows = [l.split(d) for l in _lines(args.input)]           # group, action, reward
    groups = sorted({r[0] for r in rows})
    bank = BanditBank(cfg.get_str("learner.type", "upperConfidenceBoundOne"), actions, len(groups),
                      {k: v for k, v in cfg.values.items()}, device=_device(args))
    if rows:
        gi = torch.tensor([groups.index(r[0]) for r in rows])
        ai = torch.tensor([actions.index(r[1]) for r in rows])
        rw = torch.tensor([float(r[2]) for r in rows])
        bank.set_rewards(gi, ai, rw)
    acts = bank.next_actions().cpu()
    _write(args, [f"{g}," + ",".join(actions[a] for a in acts[i].tolist()) for i, g in enumerate(groups)])


# ================================================================================================
# python-side drivers and services
# ================================================================================================
@job("classifier", "config-driven classifier: --kind rf|gbt|svm|lr --mode train|trainValidate|validate|...")
def _classifier(args):
    from .models import supervised as SV
    cls = {"rf": SV.RandomForest, "gbt": SV.GradientBoostedTrees, "svm": SV.SupportVectorMachine,
           "lr": SV.LogisticRegressionDiscriminant}[args.kind]
    c = cls(args.config, device=args.device)
    mode = args.mode or c.getMode()
    res = {"training": c.train, "train": c.train, "trainValidate": c.trainValidate,
           "trainValidateSearch": c.trainValidateSearch, "validate": c.validate, "predict": c.predict,
           "predictProb": c.predictProb, "autoTrain": c.autoTrain}[mode]()
    if isinstance(res, torch.Tensor):
        res = res.cpu().tolist()
    print(json.dumps(res, default=str))


@job("serve", "REST prediction service: --kind rf|gbt|svm|lr --config props --port P [--name rf]")
def _serve(args):
    from .serve import PredictionServer, classifier_factory
    srv = PredictionServer()
    srv.register_lazy(args.name or args.kind, classifier_factory(args.kind, args.config))
    print(f"serving /{args.name or args.kind}/predict on 127.0.0.1:{args.port}", flush=True)
    srv.serve(args.port)


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="avenir_amd", description=__doc__.split("\n\n")[0])
    ap.add_argument("job", nargs="?", help="job name (see --list)")
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
    args = ap.parse_args(argv)
    if args.list or not args.job:
        for n, (_, h) in sorted(JOBS.items()):
            print(f"{n:32s} {h}")
        return 0
    if args.job not in JOBS:
        print(f"unknown job {args.job}; use --list", file=sys.stderr)
        return 2
    JOBS[args.job][0](args)
    return 0


if __name__ == "__main__":
    sys.exit(main())
