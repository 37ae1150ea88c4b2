"""Core jobs: Naive Bayes, trees, kNN, logistic regression, MI, encodings, Apriori, SMOTE, KS,
Markov, Viterbi, fixtures, SA, k-means, bandits, classifier / serving drivers.

Reference drivers: R/detr.sh, R/rafo.sh, R/knn.sh, R/carm.sh, R/hica.sh, R/fit.sh, R/ovsa.sh,
R/ks.sh, R/conv.sh, R/opt.sh, R/wc.sh and the P/app classifier drivers.
"""
from __future__ import annotations

import json
import math
import sys
from pathlib import Path

import numpy as np
import torch

from .. import _native
from .common import JobContext, job


# ================================================================================================
# Bayesian / trees / kNN / linear
# ================================================================================================
@job("bayesianDistribution", "naive Bayes training (J/bayesian/BayesianDistribution.java): CSV -> model lines")
def nb_train(args):
    """``bad.tabular.input=false`` selects the text mode (``mapText``, :186-195): every line is
    ``text<delim>class`` and the word tokens are the bins of one text feature (ordinal 1)."""
    from ..models.bayes import NaiveBayes
    ctx = JobContext(args, "bad.")
    if not ctx.get_bool("tabular.input", True):
        from ..models.bayes import TextNaiveBayesModel
        co, to = ctx.get_int("class.field.ordinal", 1), ctx.get_int("text.field.ordinal", 0)
        m = TextNaiveBayesModel.fit_native(ctx, co, to) or TextNaiveBayesModel.fit_lines(ctx.lines(), ctx.split, ctx,
                                                                                          co, to)
        ctx.emit_root(m.model_lines(ctx.delim_out))
        return
    t = ctx.table()
    nb = NaiveBayes(t.schema).fit(t)
    ctx.emit_root(nb.model_lines(ctx.delim_out))


@job("bayesianPredictor", "naive Bayes prediction (J/bayesian/BayesianPredictor.java): CSV + model -> record,class,prob")
def nb_predict(args):
    """Output modes: ``record,predClass,prob`` (default), or with ``bap.output.feature.prob.only``
    ``id,featurePriorProb,cls0,p0,cls1,p1,...,actualClass`` (:271-285; the stage that feeds the
    class-conditioned kNN of R/knn.sh)."""
    from ..models.bayes import NaiveBayes
    ctx = JobContext(args, "bap.")
    if not ctx.get_bool("tabular.input", True):
        from ..models.bayes import TextNaiveBayesModel
        m = TextNaiveBayesModel.load(ctx.path("bayesian.model.file.path", "model"), ctx.split)
        to = ctx.get_int("text.field.ordinal", 0)
        got = TextNaiveBayesModel.word_tokens(ctx, ctx.get_int("class.field.ordinal", 1), to)
        if got is not None:
            # native: word ids of the shard's documents -> the model vocabulary (dictionary level),
            # one bag-of-words GEMM, output from the raw line bytes
            line, wid, uniq, _, fields = got
            mi = {w: i for i, w in enumerate(m.vocab)}
            lut = torch.tensor([mi.get(w, -1) for w in uniq] or [-1], dtype=torch.long)
            mw = lut[wid] if wid.numel() else wid
            k = mw >= 0
            pred, prob = m.predict_bow(line[k], mw[k], fields.n_lines)
            spans = fields.line_spans()
            ctx.emit_columns([spans.column("r", delims=ctx.native_delim()), ("s", m.classes, pred.cpu()),
                              ("i", torch.round(100 * prob.cpu()).long())], fields.n_lines)
            return
        rows = ctx.rows()
        pred, prob = m.predict([r[to] for r in rows])
        d = ctx.delim_out
        ctx.emit([f"{d.join(r)}{d}{m.classes[p]}{d}{int(round(100 * q))}" for r, p, q in zip(rows, pred, prob)])
        return
    from ..data.records import format_lines
    t = ctx.table()
    nb = NaiveBayes.load_model(ctx.path("bayesian.model.file.path", "model"), t.schema)
    vals = t.class_field.cardinality if t.class_field else None
    d = ctx.delim_out
    lit = _single_delim(ctx)
    if ctx.get_bool("output.feature.prob.only", False):
        # id,featurePriorProb,cls0,p0,cls1,p1,...,actualClass: columns straight from the device
        # results and the raw line bytes (the id field), one native formatting pass
        fp, post = nb.feature_probs(t)
        idf = t.schema.id_field
        cols = [t.lines.column("rf", idf.ordinal if idf is not None else 0, lit if idf is not None else ",")]
        cols.append(("f", fp.double().cpu(), -1))
        pc = post.double().cpu()
        for c, v in enumerate(nb.class_values):
            cols += [("c", v), ("f", pc[:, c].contiguous(), -1)]
        lab = t.labels[: t.n].int().cpu() if t.labels is not None else torch.full((t.n,), -1, dtype=torch.int32)
        cols.append(("s", list(vals or []), lab))
        ctx.emit_columns(cols, t.n)
        return
    r = nb.predict(t)
    prob = r.prob.max(1).values if r.prob is not None else torch.ones(t.n, device=r.pred.device)
    pred = r.pred.int()          # device tensors: the device formatter writes the rows (format.hip)
    cols = [t.lines.column("r"), ("s", list(vals), pred) if vals else ("i", pred.long()),
            ("f", prob.double(), 3)]
    ctx.emit_columns(cols, t.n)
    if r.confusion is not None:
        conf = r.confusion.clone()
        ctx.all_reduce(conf)
        ctx.report({"confusion": conf.cpu().tolist()})


def _single_delim(ctx) -> str:
    """The one-character literal input delimiter (raw-line field extraction), else ','."""
    from ..data.table import _literal
    lit = _literal(ctx.delim_in)
    return lit if lit is not None and len(lit) == 1 else ","


@job("decisionTree", "decision tree (J/tree/DecisionTreeBuilder.java, dtb.* keys) -> decision path JSON")
def dec_tree(args):
    """Whole tree in one call (decision-path JSON to ``--output``), or — with
    ``dtb.decision.file.path.out`` — ONE LEVEL per call like the reference's MR iteration
    (R/detr.sh decTree / mvDecFiles, :713-725): the current paths are read from
    ``dtb.decision.file.path.in`` (absent = root), the tree is grown one level deeper and written to
    ``decision.file.path.out``; the records, each prefixed by the predicates of its path
    (``dtb.dec.path.delim``), go to ``--output``.  Each level's JSON is the resume point."""
    from ..models.tree import DecisionPathModel, DecisionTreeBuilder, TreeParams
    ctx = JobContext(args, "dtb.")
    t = ctx.table(raw_numeric=True)
    p = TreeParams.from_config(ctx.cfg)
    n = torch.tensor([t.n])
    ctx.all_reduce(n)
    out_path = ctx.get_str("decision.file.path.out", None)
    if not out_path:
        tree = DecisionTreeBuilder(t.schema, p, comm=ctx.comm).fit(t)
        ctx.emit_json(tree.to_decision_paths(int(n)))
        return
    in_path = ctx.get_str("decision.file.path.in", None)
    depth = 0
    if in_path and Path(in_path).exists():
        prev = json.loads(Path(in_path).read_text())
        depth = max((len(dp["predicates"]) - 1 for dp in prev["decisionPaths"]), default=0)
    limit = p.max_depth if p.stopping == "maxDepth" else 10 ** 6
    level = min(depth + 1, limit)
    p.stopping, p.max_depth = "maxDepth", level
    tree = DecisionTreeBuilder(t.schema, p, comm=ctx.comm).fit(t)
    js = tree.to_decision_paths(int(n))
    ctx.check()
    if ctx.is_root:
        Path(out_path).parent.mkdir(parents=True, exist_ok=True)
        Path(out_path).write_text(json.dumps(js, indent=1))
    grown = max((len(dp["predicates"]) - 1 for dp in js["decisionPaths"]), default=0)
    # every record prefixed by the predicates of the path it takes: the paths are evaluated
    # column-wise on the table's device, the lines formatted natively from their byte spans
    from ..data.records import format_lines
    from ..models.tree import TableColumns
    _, first = DecisionPathModel(js).predict_proba_cols(TableColumns(t))
    pd = ctx.get_str("dec.path.delim", ";")
    paths = [pd.join(pr["predicateStr"] for pr in dp["predicates"]) for dp in js["decisionPaths"]] + ["$root"]
    first = torch.where(first >= 0, first, torch.full_like(first, len(paths) - 1)).int()
    ctx.emit_columns([("s", paths, first), t.lines.column("r")], t.n)
    ctx.report({"level": grown, "done": grown <= depth or grown >= limit})


@job("randomForest", "random forest of decision trees (R/rafo.sh) -> one JSON per tree")
def rafo(args):
    from ..models.tree import RandomForest, TreeParams
    ctx = JobContext(args, "dtb.")
    t = ctx.table(raw_numeric=True)
    p = TreeParams.from_config(ctx.cfg)
    p.sub_sampling = ctx.get_str("sub.sampling.strategy", "withReplace")
    rf = RandomForest(t.schema, ctx.get_int("num.trees", 10), p, ctx.get_str("max.features", "sqrt")).fit(t)
    if ctx.is_root:
        ctx.check()
        out = Path(args.output)
        out.mkdir(parents=True, exist_ok=True)
        for i, tr in enumerate(rf.trees):
            (out / f"tree_{i}.json").write_text(json.dumps(tr.to_decision_paths(t.n)))


@job("knnClassifier", "kNN classification with the fused distance+top-k kernel: --input test --train train CSV")
def knn(args):
    """Both sets are sharded over ranks; the training shards circulate around the ring
    (``distributed_knn``) so every rank classifies only its own query shard.  Distance: euclidean
    over min-max scaled numeric attributes + one-hot categorical attributes.  With categorical /
    bucketed attributes present (and at most 32 numeric + 32 categorical columns, k <= 32) the
    one-hot matrix is never built: ``mixed_knn_kernel`` adds a mismatch weight of 2 per differing
    category (1 against a missing value) — the one-hot squared distance — to the numeric terms."""
    from ..models.knn import NearestNeighbor
    from ..ops.distance import mixed_knn_max_dims
    ctx = JobContext(args, "nen.")
    schema = ctx.schema()
    tr = ctx.table(raw_numeric=True, path=args.train, schema=schema)
    te = ctx.table(raw_numeric=True, schema=schema)
    nn = NearestNeighbor.from_config(ctx.cfg)
    mx = mixed_knn_max_dims()
    mixed = (bool(tr.binned_fields) and len(tr.numeric_fields) <= mx and len(tr.binned_fields) <= mx
             and nn.k <= 32 and nn.metric == "euclidean")
    if mixed:
        Xtr, Xte = _numeric_block(tr), _numeric_block(te)
        Ctr, Cte = _category_codes(tr), _category_codes(te)
    else:
        Xtr, Xte = tr.dense_features(one_hot=True), te.dense_features(one_hot=True)
    lo, hi = Xtr.min(0).values if tr.n else Xtr.new_full((Xtr.shape[1],), math.inf), \
        Xtr.max(0).values if tr.n else Xtr.new_full((Xtr.shape[1],), -math.inf)
    if ctx.comm.is_distributed:
        ctx.comm.all_reduce(lo, "min")
        ctx.comm.all_reduce(hi, "max")
    scale = (hi - lo).clamp_min(1e-12)
    y = tr.labels[: tr.n].long()
    if mixed:
        wc = torch.full((Ctr.shape[1],), 2.0, device=Xtr.device)
        nn.fit_mixed((Xtr - lo) / scale, Ctr, wc, y, tr.n_classes, index_base=tr.row_offset)
        res = nn.predict((Xte - lo) / scale, q_base=te.row_offset, Qc=Cte)
    else:
        nn.fit((Xtr - lo) / scale, y, tr.n_classes, index_base=tr.row_offset)
        res = nn.predict((Xte - lo) / scale, q_base=te.row_offset)
    vals = te.class_field.cardinality
    ctx.emit_columns([te.lines.column("r"), ("s", list(vals), res.pred.int())], te.n)


def _numeric_block(t) -> torch.Tensor:
    """[n, Dn] float32 numeric attributes of ``t`` in schema order."""
    if not t.numeric_fields:
        return torch.zeros((t.n, 0), device=t.device)
    o = sorted(range(len(t.numeric_fields)), key=lambda i: t.numeric_fields[i].ordinal)
    return t.numeric[o, : t.n].T.float().contiguous()


def _category_codes(t) -> torch.Tensor:
    """[n, Dc] int32 codes of the binned attributes (categorical and bucketed), -1 = missing."""
    o = sorted(range(len(t.binned_fields)), key=lambda i: t.binned_fields[i].ordinal)
    nb = torch.tensor([t.binned_fields[i].num_bins for i in o], device=t.device).view(1, -1)
    c = t.codes[o, : t.n].T.long()
    return torch.where(c < nb, c, torch.full_like(c, -1)).int().contiguous()


@job("logisticRegression", "logistic regression (J/regress/LogisticRegressionJob.java): CSV -> coefficient lines per iteration")
def logit(args):
    from ..models.linear import LogisticRegression
    ctx = JobContext(args, "lor.")
    t = ctx.table(raw_numeric=True)
    X = t.dense_features()
    m = LogisticRegression(solver=ctx.get_str("solver", "newton"), max_iter=ctx.get_int("iteration.limit", 10),
                           criteria=ctx.get_str("convergence.criteria", "iterLimit"),
                           threshold=ctx.get_float("convergence.threshold", 5.0))
    pos = ctx.get_str("positive.class.value", None)
    vals = t.class_field.cardinality
    y = (t.labels[: t.n].long() == (vals.index(pos) if pos in vals else 1)).float()
    m.fit(X, y)
    ctx.emit_root(m.coefficient_lines(ctx.delim_out))


# ================================================================================================
# exploration / encoding / sampling
# ================================================================================================
@job("mutualInformation", "mutual information feature scores (J/explore/MutualInformation.java, mut.* keys)")
def mi(args):
    """One class histogram + all pair histograms (K2/K3), one all-reduce; the scores of
    ``mut.mutual.info.score.algorithms``; with ``mut.feature.class.cond.dstr.sep.output`` the
    feature class-conditional distribution is written to
    ``mut.feature.class.distr.output.file.path`` (the input of categoricalClassAffinity, R/carm.sh)."""
    from ..models.explore import MutualInformation
    ctx = JobContext(args, "mut.")
    t = ctx.table()
    m = MutualInformation(comm=ctx.comm)
    m.fit(t)
    alg = ctx.get_str("mutual.info.score.algorithms", "mutual.info.maximization").split(",")
    lines = []
    fns = {"mutual.info.maximization": m.mim, "mutual.info.selection": m.mifs, "joint.mutual.info": m.jmi,
           "double.input.symmetrical.relevance": m.disr, "min.redundancy.max.relevance": m.mrmr}
    for a in alg:
        if a in fns:
            lines.append(a)
            lines += [f"{f},{s:.6f}" for f, s in fns[a]()]
    ctx.emit_root(lines)
    if ctx.get_bool("feature.class.cond.dstr.sep.output", False):
        ctx.emit_root(m.class_conditional_lines(t, ctx.delim_out), ctx.get_str("feature.class.distr.output.file.path"))


@job("categoricalClassAffinity", "class affinity of categorical values (J/explore/CategoricalClassAffinity.java, cca.*)")
def caff(args):
    """Input: the feature class-conditional distribution file of mutualInformation
    (``featOrd,classVal,featVal,prob``, R/carm.sh), or — with a schema — the raw records (the
    distribution is then computed here by the K2 class histogram).  For each strategy of
    ``cca.affinity.strategy`` (oddsRatio, distrDiff, minRisk, klDiff): an ``algorithm: <s>`` line,
    then ``featOrd,value,score`` per feature sorted by descending score (:189-258)."""
    ctx = JobContext(args, "cca.")
    strategies = ctx.get_list("affinity.strategy", "oddsRatio")
    pos = ctx.get_str("pos.class.attr.value", None) or ctx.get_str("positive.class.value", None)
    d = ctx.delim_out
    has_schema = bool(getattr(args, "schema", None) or ctx.has("feature.schema.file.path"))
    lines = []
    if has_schema:
        from ..models.explore import class_affinity
        t = ctx.table()
        pc = t.class_field.cardinality.index(pos) if pos in (t.class_field.cardinality or []) else 0
        for sname in strategies:
            res = class_affinity(t, sname, pos_class=pc, comm=ctx.comm)
            lines.append(f"algorithm: {sname}")
            lines += [f"{o}{d}{v}{d}{s!r}" for o, vals in res.items() for v, s in vals]
        ctx.emit_root(lines)
        return
    pos_d, neg_d = {}, {}
    feats = []
    for r in ctx.rows(shard=False):
        if len(r) < 4:
            continue
        o = int(r[0])
        if o not in feats:
            feats.append(o)
        (pos_d if r[1] == pos else neg_d).setdefault(o, {})[r[2]] = float(r[3])
    for sname in strategies:
        lines.append(f"algorithm: {sname}")
        for o in feats:
            pdist, ndist = pos_d.get(o, {}), neg_d.get(o, {})
            vals = list(pdist)
            p = torch.tensor([pdist[v] for v in vals], dtype=torch.float64)
            q = torch.tensor([ndist.get(v, 0.0) for v in vals], dtype=torch.float64)
            if sname == "oddsRatio":
                sc = (p / (1 - p)) / (q / (1 - q))
            elif sname == "distrDiff":
                sc = p - q
            elif sname == "minRisk":
                sc = p * (1 - q)
            elif sname == "klDiff":
                sc = p * torch.log(p / q)
            else:
                raise SystemExit(f"unknown affinity strategy {sname}")
            order = sorted(range(len(vals)), key=lambda i: -float(sc[i]) if not math.isnan(float(sc[i])) else math.inf)
            lines += [f"{o}{d}{vals[i]}{d}{float(sc[i])!r}" for i in order]
    ctx.emit_root(lines)


@job("categoricalContinuousEncoding", "supervised ratio / weight-of-evidence encoding (R/hica.sh, J/explore/CategoricalContinuousEncoding.java)")
def hica(args):
    """Reference keys ``coe.cat.attribute.ordinals``, ``coe.class.attr.ordinal``,
    ``coe.pos.class.attr.value``, ``coe.encoding.strategy``, ``coe.output.scale`` (schema-less; the
    dictionaries of the categorical fields are discovered, any cardinality — uint16 codes above 255
    values), or a feature schema.  Output ``attr,value,encodedInt`` (:204-230)."""
    from ..models.explore import supervised_encoding
    ctx = JobContext(args, "coe.")
    if ctx.has("cat.attribute.ordinals"):
        schema = ctx.adhoc_schema(ctx.get_int_list("cat.attribute.ordinals"), ctx.get_int("class.attr.ordinal"))
        t = ctx.table(schema=schema)
    else:
        ctx.cfg.prefix = "cce."
        t = ctx.table()
    pos = ctx.get_str("pos.class.attr.value", None)
    vals = t.class_field.cardinality
    pc = vals.index(pos) if pos in vals else 1
    enc = supervised_encoding(t, ctx.get_str("encoding.strategy", "supervisedRatio"), ctx.get_int("output.scale", 1000),
                              pos_class=pc, comm=ctx.comm)
    d = ctx.delim_out
    ctx.emit_root([f"{o}{d}{v}{d}{int(s)}" for o, m in enc.items() for v, s in m.items()])


@job("frequentItemsApriori", "Apriori frequent item sets (R/fit.sh): one transaction per line")
def apriori(args):
    from ..data.table import _literal
    from ..models.association import Apriori
    ctx = JobContext(args, "fia.")
    skip = ctx.get_int("skip.field.count", 1)
    ap = Apriori(ctx.get_float("support.threshold", 0.1), ctx.get_int("max.item.set.length", 4), comm=ctx.comm)
    lit = _literal(ctx.delim_in)
    if lit is not None and len(lit) == 1:
        # native transaction ingest: this rank's byte range -> (transaction, item) pairs -> device bit rows
        fi = ap.fit_records(ctx.records(modes="x" * skip), skip)
    else:
        rows = ctx.rows()
        fi = ap.fit_transactions([r[skip:] for r in rows], device=ctx.device)
    d = ctx.delim_out
    lines = [d.join(names) + f"{d}{sup:.6f}" for k in range(1, ap.max_len + 1) for names, sup in fi.as_names(k)]
    ctx.emit_root(lines)


@job("classBasedOverSampler", "SMOTE over-sampling of the minority class (R/ovsa.sh, J/explore/ClassBasedOverSampler.java)")
def smote(args):
    """Two input forms.  With ``cbos.rec.len`` (the reference): every line is a minority record
    followed by its same-class neighbours (topMatchesByClass compact output), each ``rec.len``
    fields; ``cbos.over.sampling.multiplier`` synthetic records per line interpolate the numeric
    fields of the record and a neighbour picked uniformly or exponentially
    (``cbos.neighbor.sampling.distr``) and take categorical values from either (:125-200) — all
    lines of the shard at once as ``[n, M, rec.len]`` tensors.  Without it: the neighbourhoods are
    computed here by the fused kNN kernel over the schema's features."""
    from ..models.sampling import smote as _smote
    ctx = JobContext(args, "cbos.")
    if ctx.has("rec.len"):
        return _smote_from_neighbors(ctx)
    t = ctx.table(raw_numeric=True)
    X = t.dense_features()
    y = t.labels[: t.n].long()
    cnt = torch.bincount(y, minlength=t.n_classes).double()
    ctx.all_reduce(cnt)                                       # global class counts
    present = torch.nonzero(cnt > 0).view(-1)
    minority = int(present[cnt[present].argmin()])
    n_new = int(cnt.sum() - 2 * cnt[minority])                # majority total - minority
    Xn, _ = _smote(X, y, minority, max(n_new, 0), ctx.get_int("neighbor.count", 5),
                   seed=ctx.get_int("random.seed", 0), comm=ctx.comm)
    vals = t.class_field.cardinality
    d = ctx.delim_out
    ctx.emit([d.join(f"{v:.4f}" for v in row) + f"{d}{vals[minority]}" for row in Xn.cpu().tolist()])


def _smote_from_neighbors(ctx: JobContext) -> None:
    """ClassBasedOverSampler.map (:125-200) on topMatchesByClass compact lines: record + up to M
    neighbour records of ``rec.len`` fields.  Every line's ``over.sampling.multiplier`` synthetic
    records come from the K25 SMOTE kernel (Philox draws keyed by the GLOBAL line index and copy:
    neighbour pick uniform / exponential, gap, categorical coin), so the output does not depend on
    the world size; the id field shuffles the two ids' characters with a generator seeded by the
    same key."""
    from ..ops import resample_ops as RS
    L = ctx.get_int("rec.len")
    mult = ctx.get_int("over.sampling.multiplier")
    distr = ctx.get_str("neighbor.sampling.distr", "uniform")
    prec = ctx.get_int("output.precision", 3)
    schema = ctx.schema("feature.schema.file.path")
    seed = ctx.get_int("random.seed", 0)
    rec = ctx.try_records(tail_mode="n", numeric=True)
    if rec is not None:
        _smote_native(ctx, rec, L, mult, distr, prec, schema, seed)
        return
    all_rows = ctx.rows()
    base = ctx.line_base(len(all_rows))
    keep_i = [i for i, r in enumerate(all_rows) if len(r) >= 2 * L]
    rows = [all_rows[i] for i in keep_i]
    if not rows:
        ctx.emit([])
        return
    M = max((len(r) - L) // L for r in rows)
    n = len(rows)
    fields = {f.ordinal: f for f in schema.fields}
    num_cols = [i for i in range(L) if i in fields and fields[i].feature and fields[i].is_numeric]
    nnb = torch.tensor([(len(r) - L) // L for r in rows], dtype=torch.int32)
    src = torch.tensor([[float(r[i]) for i in num_cols] for r in rows], dtype=torch.float32).view(n, len(num_cols))
    nb = torch.zeros((n, M, len(num_cols)), dtype=torch.float32)
    for a, r in enumerate(rows):
        for m in range((len(r) - L) // L):
            nb[a, m] = torch.tensor([float(r[L + m * L + i]) for i in num_cols], dtype=torch.float32)
    # categorical coin: source codes 0, neighbour codes 1 -> the kernel's choice per synthetic record
    Cs = torch.zeros((n, 1), dtype=torch.int32)
    Cn = torch.ones((n, M, 1), dtype=torch.int32)
    gidx = torch.tensor([base + i for i in keep_i], dtype=torch.long)
    dev = ctx.device
    outs = []
    # the kernel keys draws by (gbase + r) * mult + j with contiguous r: run per contiguous run of lines
    runs, start = [], 0
    for a in range(1, n + 1):
        if a == n or int(gidx[a]) != int(gidx[a - 1]) + 1:
            runs.append((start, a))
            start = a
    newX, newC, pick = [], [], []
    for a0, a1 in runs:
        x, c, pk = RS.smote_rows(src[a0:a1].to(dev), nb[a0:a1].to(dev), nnb[a0:a1].to(dev), Cs[a0:a1].to(dev),
                                 Cn[a0:a1].to(dev), mult, int(gidx[a0]), seed, distr == "exponential",
                                 ctx.get_float("exp.distr.mean", 1.0))
        newX.append(x.cpu())
        newC.append(c.cpu())
        pick.append(pk.cpu())
    newX, newC, pick = torch.cat(newX), torch.cat(newC), torch.cat(pick)
    d = ctx.delim_out
    for a, r in enumerate(rows):
        for j in range(mult):
            o = a * mult + j
            pj = max(int(pick[o]), 0)
            nrec = r[L + pj * L: L + pj * L + L]
            rec = list(r[:L])
            for i in range(L):
                f = fields.get(i)
                if f is None:
                    continue
                if f.id:
                    rec[i] = _scramble(r[i] + nrec[i], (seed * 1000003 + int(gidx[a])) * 131 + j)[: len(r[i])]
                elif f.feature and f.is_categorical:
                    rec[i] = r[i] if int(newC[o, 0]) == 0 else nrec[i]
            for c, i in enumerate(num_cols):
                v = float(newX[o, c])
                rec[i] = str(int(v)) if fields[i].is_integer else f"{v:.{prec}f}"
            outs.append(d.join(rec))
    ctx.emit(outs)


_M64 = (1 << 64) - 1


def _scramble(s: str, key: int) -> str:
    """The id scramble of ``smote_lines`` (bindings.cpp): Fisher-Yates over the bytes driven by a
    splitmix64 stream seeded with ``key`` (mod 2^64)."""
    b = bytearray(s.encode())
    x = key & _M64
    for k in range(len(b) - 1, 0, -1):
        x = (x + 0x9E3779B97F4A7C15) & _M64
        z = x
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
        z ^= z >> 31
        r = z % (k + 1)
        b[k], b[r] = b[r], b[k]
    return b.decode(errors="replace")


def _smote_native(ctx, rec, L, mult, distr, prec, schema, seed):
    """classBasedOverSampler on a native token table (every field parsed as a number): source and
    neighbour feature values are gathers from the token array, the K25 kernel draws the synthetic
    values, and ``smote_lines`` assembles the output records from the raw line bytes."""
    from .. import _native
    from ..data.lines import LineSpans
    from ..ops import resample_ops as RS
    dev = ctx.device
    lens = rec.lens()
    keep = lens >= 2 * L
    ki = torch.nonzero(keep).view(-1)
    n = int(ki.numel())
    if n == 0:
        ctx.emit([])
        return
    fields = {f.ordinal: f for f in schema.fields}
    num_cols = [i for i in range(L) if i in fields and fields[i].feature and fields[i].is_numeric]
    kinds = []
    for i in range(L):
        f = fields.get(i)
        if f is None or not (f.id or f.feature):
            kinds.append(0)
        elif f.id:
            kinds.append(1)
        elif i in num_cols:
            kinds.append(2 if f.is_integer else 3)
        elif f.is_categorical:
            kinds.append(4)
        else:
            kinds.append(0)
    base = rec.off[:-1][ki]
    nnb = ((lens[ki] - L) // L).to(torch.int32)
    M = int(nnb.max())
    nums = rec.nums
    cols = torch.tensor(num_cols, dtype=torch.long, device=base.device)
    src = nums[base.view(-1, 1) + cols.view(1, -1)].float()
    mm = torch.arange(M, device=base.device)
    pos = base.view(-1, 1, 1) + L + (mm * L).view(1, -1, 1) + cols.view(1, 1, -1)
    valid = (mm.view(1, -1) < nnb.view(-1, 1).long()).unsqueeze(2)
    nb = torch.where(valid, nums[torch.where(valid, pos, base.view(-1, 1, 1))].float(), torch.zeros((), device=base.device))
    Cs = torch.zeros((n, 1), dtype=torch.int32, device=base.device)
    Cn = torch.ones((n, M, 1), dtype=torch.int32, device=base.device)
    gidx = (rec.line_base + ki).long().cpu()
    # the kernel keys draws by (gbase + r) * mult + j with contiguous r: one launch per run of
    # consecutive kept lines
    brk = torch.nonzero(gidx[1:] != gidx[:-1] + 1).view(-1) + 1
    bounds = [0] + brk.tolist() + [n]
    newX, newC, pick = [], [], []
    for a0, a1 in zip(bounds[:-1], bounds[1:]):
        x, c, pk = RS.smote_rows(src[a0:a1].to(dev), nb[a0:a1].to(dev), nnb[a0:a1].to(dev), Cs[a0:a1].to(dev),
                                 Cn[a0:a1].to(dev), mult, int(gidx[a0]), seed, distr == "exponential",
                                 ctx.get_float("exp.distr.mean", 1.0))
        newX.append(x.cpu())
        newC.append(c.cpu())
        pick.append(pk.cpu())
    newX, newC, pick = torch.cat(newX), torch.cat(newC), torch.cat(pick)
    spans = rec.line_spans().select(ki.cpu())
    _, addr, ln = spans.spans()
    numcol = [num_cols.index(i) if i in num_cols else -1 for i in range(L)]
    buf, off = _native.C().smote_lines(addr, ln, L, torch.tensor(kinds, dtype=torch.int32),
                                       torch.tensor(numcol, dtype=torch.int32), newX.float(),
                                       newC[:, 0].int().contiguous(), pick.long(), gidx, mult, seed, prec,
                                       ctx.native_delim(), ctx.delim_out, 16)
    out = LineSpans.from_packed(buf, off)
    ctx.emit_columns([out.column("r")], len(out))


@job("kolmogorovSmirnovModelDrift", "KS drift between reference and current distributions (S/explore/KolmogorovSmirnovModelDrift.scala)")
def ks(args):
    from ..models.explore import kolmogorov_smirnov_drift, numeric_histogram
    ctx = JobContext(args, "ksd.")
    if not getattr(args, "train", None):
        from .pipeline_stages import ks_from_distr
        return ks_from_distr(ctx)
    col = ctx.get_int("attr.ordinal", 0)
    ref = ctx.numeric_matrix([col], path=args.train, shard=False)[0][:, 0].cpu()
    cur = ctx.numeric_matrix([col], shard=False)[0][:, 0].cpu()
    bw = ctx.get_float("bin.width", float((ref.max() - ref.min()) / 50 or 1))
    lo = float(min(ref.min(), cur.min()))
    nb = int((float(max(ref.max(), cur.max())) - lo) / bw) + 1
    stat, crit, drift = kolmogorov_smirnov_drift(numeric_histogram(ref, bw, lo, nb), numeric_histogram(cur, bw, lo, nb))
    ctx.emit_root([f"{col},{stat:.6f},{crit:.6f},{drift}"])


# ================================================================================================
# sequences / Markov
# ================================================================================================
@job("markovStateTransitionModel", "Markov transition probabilities per class (R/conv.sh, J/markov/MarkovStateTransitionModel.java)")
def markov(args):
    """Compact rows ``id,[class],s1,s2,...`` (MR and Spark compact format), or the Spark long format
    (``mst.input.format=long``: ``id,seq,state`` rows grouped by id and ordered by seq,
    S/sequence/MarkovStateTransitionModel.scala:202-225).

    Compact rows go through the native record path (J/markov/MarkovStateTransitionModel.java:116-133
    splits and looks up every token in its mapper): this rank's byte range is tokenized once (on
    the GPU when there is one), states and class labels are dictionary lookups on the device, the
    sequences a padded [N, L] state matrix for the K4 bigram kernel, and the [C, S, S] counts are
    all-reduced once."""
    from ..data.table import _literal
    ctx = JobContext(args, "mst.")
    lit = _literal(ctx.delim_in)
    if ctx.get_str("input.format", "compact") == "long" or lit is None or len(lit) != 1:
        return _markov_rows(ctx)
    from ..models.markov import MarkovStateTransitionModel
    states = ctx.get_list("model.states", None) or ctx.get_list("state.list")
    skip = ctx.get_int("skip.field.count", 1)
    cls_ord = ctx.get_int("class.label.field.ord", ctx.get_int("class.label.field.ordinal", -1))
    modes = "".join("d" if i == cls_ord else "x" for i in range(max(skip, cls_ord + 1)))
    rec = ctx.records(modes=modes)
    st = rec.map_codes(rec.codes, states)
    seqs, _ = rec.padded(st, start=skip, drop=(cls_ord,) if cls_ord >= 0 else ())
    m = MarkovStateTransitionModel(states, scale=ctx.get_int("trans.prob.scale", 1000), comm=ctx.comm)
    labels = None
    if cls_ord >= 0:
        lc = rec.field(cls_ord)
        present = torch.unique(lc[lc >= 0]).tolist()
        cl = ctx.get_list("class.labels", None) or ctx.union(rec.vocab[c] for c in present)
        if len(cl) > 254:
            raise SystemExit("markovStateTransitionModel: at most 254 class labels")
        m.class_labels = cl
        labels = rec.map_codes(lc, cl)
        labels = torch.where(labels >= 0, labels, torch.full_like(labels, 255)).to(torch.uint8)
    m.fit(seqs, labels)
    ctx.emit_root(m.model_lines(ctx.delim_out))


def _markov_rows(ctx: JobContext):
    """Long-format input (and regex delimiters): the row-list path."""
    from ..models.markov import MarkovStateTransitionModel
    states = ctx.get_list("model.states", None) or ctx.get_list("state.list")
    skip = ctx.get_int("skip.field.count", 1)
    cls_ord = ctx.get_int("class.label.field.ord", ctx.get_int("class.label.field.ordinal", -1))
    if ctx.get_str("input.format", "compact") == "long":
        from collections import defaultdict
        id_ord, seq_ord, st_ord = (ctx.get_int("id.field.ordinal", 0), ctx.get_int("seq.field.ordinal", 1),
                                   ctx.get_int("state.field.ordinal", 2))
        g = defaultdict(list)
        for r in ctx.rows(shard=False):
            g[r[id_ord]].append((float(r[seq_ord]), r[st_ord]))
        rows = [[k] + [s for _, s in sorted(v)] for k, v in sorted(g.items())]
        if ctx.comm.is_distributed:
            from ..data.table import shard_range
            a, b = shard_range(len(rows), ctx.comm.rank, ctx.comm.world)
            rows = rows[a:b]
        skip, cls_ord = 1, -1
    else:
        rows = ctx.rows()
    seqs = [r[skip:] if cls_ord < 0 else [v for i, v in enumerate(r) if i >= skip and i != cls_ord] for r in rows]
    m = MarkovStateTransitionModel(states, scale=ctx.get_int("trans.prob.scale", 1000), comm=ctx.comm)
    enc = m.encode(seqs)
    labels = None
    if cls_ord >= 0:
        cl = ctx.get_list("class.labels", None) or ctx.union(r[cls_ord] for r in rows)
        m.class_labels = cl
        labels = torch.tensor([cl.index(r[cls_ord]) for r in rows])
    m.fit(enc, labels)
    ctx.emit_root(m.model_lines(ctx.delim_out))


@job("viterbiStatePredictor", "HMM state sequence per observation sequence (J/markov/ViterbiStatePredictor.java); --model <HMM lines>")
def viterbi(args):
    """Rows ``id,obs,obs,...`` -> ``id,state,state,...``: ``vsp.id.field.ordinal`` (default 0) is
    written first, the observations start after ``vsp.skip.field.count`` (default 1) fields; with
    ``vsp.output.state.only=false`` each token is ``obs<sub.field.delim>state``.  The model file is
    always split on ',' (:94-142).  A token outside the model's observations ends the sequence."""
    from ..models.markov import HiddenMarkovModel, ViterbiDecoder
    ctx = JobContext(args, "vsp.")
    skip = ctx.get_int("skip.field.count", 1)
    id_ord = ctx.get_int("id.field.ordinal", 0)
    state_only = ctx.get_bool("output.state.only", True)
    sub = ctx.get_str("sub.field.delim", ":")
    hmm = HiddenMarkovModel.from_lines(ctx.all_lines(ctx.path("hmm.model.path", "model")), ",")
    from ..data.table import _literal
    lit = _literal(ctx.delim_in)
    if lit is None or len(lit) != 1:
        return _viterbi_rows(ctx, hmm, skip, id_ord, state_only, sub)
    from ..data.records import format_lines
    # native path: this rank's byte range tokenized once (observation tokens by dictionary), the
    # padded [N, L] observation matrix built on the device, the K-Viterbi kernel, and the output
    # formatted from the decoded state ids and the raw id field — no per-token Python
    rec = ctx.records(modes="x" * skip)
    obs, _ = rec.padded(rec.map_codes(rec.codes, hmm.observations), start=skip, min_len=1)
    path, _ = ViterbiDecoder(hmm).decode(obs.to(ctx.device))
    ok = path >= 0
    cnt = ok.sum(1).long()
    off = torch.cat([cnt.new_zeros(1), torch.cumsum(cnt, 0)])
    S = len(hmm.states)
    if state_only:
        table, idx = hmm.states, path[ok]
    else:   # obs<sub>state tokens: one table entry per (observation, state) pair
        table = [f"{o}{sub}{st}" for o in hmm.observations for st in hmm.states]
        idx = obs.to(path.device).long()[ok] * S + path[ok]
    cols = [rec.line_spans().column("rf", id_ord, lit), ("l", table, idx.int(), off)]
    ctx.emit_columns(cols, rec.n_lines)


def _viterbi_rows(ctx, hmm, skip, id_ord, state_only, sub):
    """Regex delimiters: the split-row path."""
    from ..models.markov import ViterbiDecoder
    rows = ctx.rows()
    oi = {o: i for i, o in enumerate(hmm.observations)}
    L = max([len(r) - skip for r in rows] + [1])
    obs = torch.tensor([[oi.get(t, -1) for t in r[skip:]] + [-1] * (L - len(r[skip:])) for r in rows],
                       dtype=torch.int16).view(len(rows), L)
    paths = ViterbiDecoder(hmm).decode_labels(obs.to(ctx.device))
    d = ctx.delim_out
    out = []
    for row, p in zip(rows, paths):
        toks = p if state_only else [f"{o}{sub}{s}" for o, s in zip(row[skip:], p)]
        out.append(d.join([row[id_ord]] + toks))
    ctx.emit(out)


@job("genData", "tutorial fixture generator: --name <P/app script> --gen-args a,b,c [--seed s] (data/fixtures.py)")
def gen_data(args):
    from ..data.fixtures import FIXTURES

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
        JobContext(args).emit_root(lines)
    else:
        sys.stdout.write("\n".join(lines) + "\n")


@job("wordCount", "word count (J/text/WordCounter.java, S/sanity/WordCount.scala)")
def wc(args):
    from collections import Counter
    ctx = JobContext(args)
    if _native.host() is not None:
        # native: whitespace tokens of this rank's byte range as dictionary codes (merged over ranks,
        # so the count vector is global after one all-reduce); only distinct words reach Python
        rec = ctx.records(delims=" \t\r\v\f", tail_mode="d")
        V = len(rec.vocab)
        cnt = torch.bincount(rec.codes[rec.codes >= 0].long(), minlength=V)[:V] if V else torch.zeros(0, dtype=torch.long)
        ctx.all_reduce(cnt)
        ch = cnt.cpu().tolist()
        ctx.emit_root([f"{w},{ch[i]}" for w, i in sorted((w, i) for i, w in enumerate(rec.vocab) if w and ch[i])])
        return
    c = ctx.sum_counts(Counter(w for l in ctx.lines() for w in l.split()))
    ctx.emit_root([f"{w},{n}" for w, n in sorted(c.items())])


# ================================================================================================
# optimisation / clustering / bandits
# ================================================================================================
@job("simulatedAnnealing", "SA over a task-schedule domain (R/opt.conf block simulatedAnnealing)")
def sa(args):
    from ..optimize import SimulatedAnnealing, TaskScheduleSearch
    ctx = JobContext(args, app="simulatedAnnealing")
    dom_file = ctx.path("domain.callback.config.file", "domain")
    d = TaskScheduleSearch.from_json(dom_file, ctx.device)
    r = SimulatedAnnealing.from_config(d, ctx.cfg).run()
    o = ctx.get_str("field.delim.out", ",")
    lines = [f"{d.format_solution(s)}{o}{c:.6f}" for s, c in zip(r.solutions.tolist(), r.costs.tolist())]
    lines.sort(key=lambda l: float(l.rsplit(o, 1)[1]))
    ctx.emit_root(lines)
    ctx.report({"best_cost": r.best_cost, **r.stats})


@job("kmeansCluster", "k-means over numeric columns (S/cluster/KmeansCluster.scala); --k list; knuckle-point k")
def kmeans(args):
    from ..models.cluster import KMeans
    ctx = JobContext(args, "kmc.")
    cols = ctx.get_int_list("attr.ordinals", "0")
    X = ctx.numeric_matrix(cols, dtype=torch.float32)[0]
    ks = [int(k) for k in (args.k or ctx.get_str("num.clusters", "3")).split(",")]
    km = KMeans(ks, n_init=ctx.get_int("num.init.groups", 3), max_iter=ctx.get_int("max.iterations", 100)).fit(X)
    lines = []
    for k in ks:
        run = km.best[k]
        lines += [f"{k},{i}," + ",".join(f"{v:.4f}" for v in c) for i, c in enumerate(run.centroids.cpu().tolist())]
        lines.append(f"{k},sse,{run.sse:.4f}")
    if len(ks) > 2:
        lines.append(f"knuckle,{km.knuckle_k()}")
    ctx.emit_root(lines)


@job("multiArmBandit", "batch bandit per group (S/reinforce/MultiArmBandit.scala): rewards in, actions out")
def mab(args):
    """Rows ``group,action,reward``; per group (string order) the learner's next action(s), output
    ``group,action..``.  Native path: each rank reads its byte range and sends every reward row to
    the rank owning its group (one all-to-all, input order kept); the bank spans ALL groups on
    every rank, so the selection's Philox streams are keyed by the global group index and the
    output does not depend on the world size; each rank writes its block of groups."""
    from ..data.table import _literal
    from ..models.bandit import BanditBank
    ctx = JobContext(args, app="multiArmBandit")
    actions = ctx.get_list("action.list")
    lit = _literal(ctx.delim_in)
    if lit is None or len(lit) != 1:
        rows = ctx.rows(shard=False)                # group, action, reward
        groups = sorted({r[0] for r in rows})
        bank = BanditBank(ctx.get_str("learner.type", "upperConfidenceBoundOne"), actions, len(groups),
                          dict(ctx.cfg.values), device=ctx.device)
        if rows:
            gi = {g: i for i, g in enumerate(groups)}
            bank.set_rewards(torch.tensor([gi[r[0]] for r in rows]), torch.tensor([actions.index(r[1]) for r in rows]),
                             torch.tensor([float(r[2]) for r in rows]))
        acts = bank.next_actions().cpu()
        from ..data.table import shard_range
        a, b = shard_range(len(groups), ctx.comm.rank, ctx.comm.world) if ctx.comm.is_distributed else (0, len(groups))
        ctx.emit([f"{g}," + ",".join(actions[x] for x in acts[i].tolist()) for i, g in enumerate(groups) if a <= i < b])
        return
    from ..data.records import format_lines, owner_of, shuffle, sorted_keys
    from ..data.table import shard_range
    comm = ctx.comm
    rec = ctx.records(modes="ddn", tail_mode="x", numeric=True)
    g_code = rec.field(0)
    act = rec.map_codes(rec.field(1), actions).long()
    if bool((act < 0).any()):
        raise SystemExit("multiArmBandit: an action outside action.list")
    keys, pos = sorted_keys(rec, g_code, comm)
    G = keys.numel()
    gp = pos[g_code.long()]
    owner = owner_of(gp, G, comm.world) if comm.is_distributed else torch.zeros_like(gp)
    gp, act, rw = shuffle(comm, owner, [gp, act, rec.field(2, numeric=True)])
    bank = BanditBank(ctx.get_str("learner.type", "upperConfidenceBoundOne"), actions, G, dict(ctx.cfg.values),
                      device=ctx.device)
    if gp.numel():
        bank.set_rewards(gp, act, rw)
    acts = bank.next_actions().cpu()
    a, b = shard_range(G, comm.rank, comm.world) if comm.is_distributed else (0, G)
    nb = acts.shape[1]
    cols = [("s", rec.vocab, keys[a:b].int().cpu()),
            ("l", list(actions), acts[a:b].reshape(-1).int(), torch.arange(0, (b - a) * nb + 1, nb, dtype=torch.long))]
    ctx.emit_columns(cols, b - a)


# ================================================================================================
# python-side drivers and services
# ================================================================================================
@job("classifier", "config-driven classifier (P/supv drivers): --kind rf|gbt|svm|lr --mode train|trainValidate|validate|...")
def classifier(args):
    from ..models import supervised as SV
    cls = {"rf": SV.RandomForest, "gbt": SV.GradientBoostedTrees, "svm": SV.SupportVectorMachine,
           "lr": SV.LogisticRegressionDiscriminant}[args.kind]
    c = cls(args.config, device=args.device)
    mode = args.mode or c.getMode()
    if mode == "explain":
        return _classifier_explain(c, args)
    res = {"training": c.train, "train": c.train, "trainValidate": c.trainValidate,
           "trainValidateSearch": c.trainValidateSearch, "validate": c.validate, "predict": c.predict,
           "predictProb": c.predictProb, "autoTrain": c.autoTrain}[mode]()
    if isinstance(res, torch.Tensor):
        res = res.cpu().tolist()
    print(json.dumps(res, default=str))


def _classifier_explain(clf, args):
    """``intrd.py explain <clf> <clfConf> <limeConf> <record>`` (P/app/intrd.py:69-89): a LIME
    surrogate (analytics/interpret.LimeTabular) around the record, built from the classifier's
    training features, with the LimeInterpreter keys of P/mlextra/interpret.py:38-56
    (``inter.feature.names``, ``inter.kernel.width``, ``data.cat.values`` -> categorical columns,
    ``inter.random.state``, ``explain.num.features``, ``explain.num.samples``); prints the top
    features and their weights as lime's ``as_list()``."""
    from ..analytics.interpret import LimeTabular
    from ..utils.config import read_properties
    rest = list(getattr(args, "rest", None) or [])
    if len(rest) < 2:
        raise SystemExit("usage: classifier --mode explain --kind K -c clf.props <lime.props> <record>")
    lc = read_properties(rest[0])
    get = lambda k, d=None: (d if lc.get(k, "_").strip() in ("_", "") else lc[k].strip())
    names = get("inter.feature.names").split(",")
    cats = [int(it.split(":")[0]) for it in get("data.cat.values", "").split(",") if it] \
        if get("data.cat.values") else []
    X, _ = clf.prepTrainingData()
    rec = np.array([float(v) for v in rest[1].split(",")], dtype=np.float32)
    clf._ensure_model()
    kw = get("inter.kernel.width")
    lime = LimeTabular(torch.tensor(X), names, kernel_width=float(kw) if kw else None, categorical=cats,
                       seed=int(get("inter.random.state", "100")))
    pf = lambda P: torch.as_tensor(np.asarray(clf.model.predict_proba(P.cpu().numpy())), dtype=torch.float32)
    exp = lime.explain(torch.tensor(rec), pf, label=1, num_samples=int(get("explain.num.samples", "5000")),
                       num_features=int(get("explain.num.features", "10")))
    print("model explanation")
    for name, w in exp["explanation"]:
        print(str((name, w)))


@job("autoSupervisedLearning", "TPE search over classifiers and their hyper-parameters (P/app/autosupv.py): "
     "--gen-args maxEvals,clf:config[:prob],...", aliases=("autosupv",))
def auto_supervised_learning(args):
    """``autosupv.py maxEvals rf:rf.properties[:p] gbt:gbt.properties[:p] ...``: each classifier's
    ``train.search.params`` defines its branch of the space; TPE minimises ``trainValidate()``.
    Prints the best assignment (hyperopt form: label -> index / value) and its loss."""
    from ..models import supervised as SV
    from ..optimize.tpe import auto_supervised
    items = [v for v in (args.gen_args or "").split(",") if v]
    if len(items) < 2:
        raise SystemExit("autoSupervisedLearning needs --gen-args maxEvals,clf:config[:prob],...")
    max_evals = int(items[0])
    kinds = {"rf": SV.RandomForest, "gbt": SV.GradientBoostedTrees, "svm": SV.SupportVectorMachine,
             "lr": SV.LogisticRegressionDiscriminant}
    clfs, probs = {}, []
    for it in items[1:]:
        parts = it.split(":")
        if parts[0] not in kinds:
            raise ValueError("unsupported classifier")
        clfs[parts[0]] = kinds[parts[0]](parts[1], device=args.device)
        if len(parts) == 3:
            probs.append(float(parts[2]))
    from ..parallel.comm import get_comm
    comm = get_comm()
    # under torchrun every rank trains one proposal of each TPE batch on its own GPU
    best, loss, t = auto_supervised(clfs, max_evals, probs or None, seed=args.seed or 0, comm=comm)
    if comm.rank == 0:
        print(json.dumps({"best": best, "loss": loss, "evals": len(t.trials)}, default=str))


@job("serve", "REST prediction service (P/app/rfsvc.py etc.): --kind rf|gbt|svm|lr --config props --port P [--name rf]")
def serve(args):
    from ..serve import PredictionServer, classifier_factory
    srv = PredictionServer()
    srv.register_lazy(args.name or args.kind, classifier_factory(args.kind, args.config))
    print(f"serving /{args.name or args.kind}/predict on 127.0.0.1:{args.port}", flush=True)
    srv.serve(args.port)
