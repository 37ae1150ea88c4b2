"""Association, clustering, nearest-neighbour pipeline, model-prediction, batch-bandit, similarity
and population-optimiser jobs (J/association, J/cluster, J/knn, J/model, J/tree/DataPartitioner,
J/reinforce batch bandits, S/similarity, S/cluster/KMeansPlusPlusCluster, S/optimize)."""
from __future__ import annotations

import itertools
import json
import math
import os
from collections import defaultdict
from pathlib import Path

import torch

from .. import _native
from .common import JobContext, field_modes, fmt, job


# ================================================================================================
# association rules
# ================================================================================================
@job("associationRuleMiner", "rules antecedent -> consequent from frequent item sets (J/association/AssociationRuleMiner.java, arm.*)")
def rule_miner(args):
    """Input: frequent item-set lines ``item,...,support`` (frequentItemsApriori output, all
    lengths).  Every proper subset (size <= ``arm.max.ante.size``) of a set is an antecedent;
    confidence = support(set) / support(antecedent); lines ``a,b -> c`` when above
    ``arm.conf.threshold`` (:111-196)."""
    from ..models.association import FrequentItemsets, association_rules
    ctx = JobContext(args, "arm.")
    max_ante = ctx.get_int("max.ante.size", 3)
    thr = ctx.get_float("conf.threshold")
    sup = {}
    for r in ctx.rows(shard=False):
        sup[tuple(r[:-1])] = float(r[-1])
    # the sets as item-id rows (ids in name order; every row sorted) with float supports: the
    # antecedent joins and confidences run on the device (models/association.association_rules)
    names = sorted({x for s_ in sup for x in s_})
    nid = {v: i for i, v in enumerate(names)}
    by_len: dict[int, list] = {}
    for s_, v in sup.items():
        by_len.setdefault(len(s_), []).append((sorted(nid[x] for x in s_), v))
    dev = ctx.device
    sets, sups = {}, {}
    for k, lst in by_len.items():
        lst.sort()
        sets[k] = torch.tensor([e[0] for e in lst], dtype=torch.long, device=dev)
        sups[k] = torch.tensor([e[1] for e in lst], dtype=torch.float64, device=dev)
    fi = FrequentItemsets(names, None, 1, sets, sups)
    rules = association_rules(fi, thr, min_len=2, max_ante=max_ante)
    # the reference's order: sets in name order, antecedent size, combination
    keyed = []
    for ante, cons, _, _ in rules:
        full = tuple(sorted(ante + cons))
        pos = tuple(full.index(x) for x in ante)
        keyed.append(((full, len(ante), pos), ",".join(ante) + " -> " + ",".join(cons)))
    keyed.sort(key=lambda e: e[0])
    ctx.emit_root([line for _, line in keyed])


@job("infrequentItemMarker", "replace items outside the frequent 1-item sets by a marker (J/association/InfrequentItemMarker.java, iim.*)")
def infrequent_marker(args):
    ctx = JobContext(args, "iim.")
    skip = ctx.get_int("skip.field.count", 1)
    marker = ctx.get_str("infreq.item.marker", "*")
    freq = set()
    for r in ctx.rows(ctx.path("item.set.file.path", "model"), shard=False):
        if len(r) == 2 or ctx.get_int("item.set.length", 1) == 1:
            freq.add(r[0])
    rec = ctx.try_records(modes="x" * skip, tail_mode="d")
    if rec is not None:
        # native: the item tokens stay dictionary codes; the marker substitution is one table over
        # the dictionary, the output a CSR string list behind the raw leading fields
        tab = [v if v in freq else marker for v in rec.vocab]
        spans, dl = rec.line_spans(), ctx.native_delim()
        idx, cnt = rec.padded(start=skip, dtype=torch.int32)
        off = torch.cat([torch.zeros(1, dtype=torch.long, device=cnt.device), torch.cumsum(cnt, 0)])
        flat = idx[torch.arange(idx.shape[1], device=idx.device).view(1, -1) < cnt.view(-1, 1)]
        ctx.emit_columns([spans.column("rf", j, dl) for j in range(skip)]
                         + [("l", tab, flat.cpu(), off.cpu())], rec.n_lines)
        return
    d = ctx.delim_out
    ctx.emit([d.join(r[:skip] + [x if x in freq else marker for x in r[skip:]]) for r in ctx.rows()])


# ================================================================================================
# clustering
# ================================================================================================
@job("entityDistanceStore", "build the memory-mapped entity-distance store from pair distances (J/util/EntityDistanceMapFileAccessor.java)")
def distance_store(args):
    """Input either ``entity,e1:d1,e2:d2,...`` lines or ``e1,e2,dist`` pair lines
    (``eds.pair.input=true``, e.g. sameTypeSimilarity / recordSimilarity output)."""
    from ..utils.distance_store import EntityDistanceStore
    ctx = JobContext(args, "eds.")
    if ctx.get_bool("pair.input", False) and ctx.native_delim() is not None:
        rec = ctx.records(shard=False, modes="ddn", tail_mode="x", numeric=True)
        EntityDistanceStore.write_codes(rec.field(0), rec.field(1), rec.field(2, numeric=True), rec.vocab, args.output)
        return
    lines = ctx.all_lines()
    if ctx.get_bool("pair.input", False):
        rows = [ctx.split(l) for l in lines]
        EntityDistanceStore.write_pairs([r[0] for r in rows], [r[1] for r in rows], [float(r[2]) for r in rows],
                                        args.output)
    else:
        EntityDistanceStore.write_text(lines, args.output, ctx.delim_in if len(ctx.delim_in) == 1 else ",",
                                       ctx.get_str("sub.field.delim", ":"))


@job("agglomerativeGraphical", "greedy edge-weighted clustering over a persisted distance store (J/cluster/AgglomerativeGraphical.java, agg.*)")
def agglomerative(args):
    """Entities (first field of each input line) join the cluster with the best new average edge
    weight above ``agg.min.av.edge.weight.threshold`` (``agg.distance.scale`` turns distances into
    similarities); the store is ``agg.distance.store.path`` (entityDistanceStore output).  Output:
    ``clusterIndex,member,...,avgEdgeWeight``."""
    from ..utils.distance_store import EntityDistanceStore, agglomerative_graphical
    ctx = JobContext(args, "agg.")
    store = EntityDistanceStore(ctx.path("distance.store.path", "model"))
    ents = [r[0] for r in ctx.rows(shard=False)]
    scale = ctx.get_float("distance.scale", None)
    cl = agglomerative_graphical(store, ents, ctx.get_float("min.av.edge.weight.threshold"), scale)
    d = ctx.delim_out
    ctx.emit_root([d.join([str(i)] + m + [repr(w)]) for i, (m, w) in enumerate(cl)])


@job("kMeansPlusPlusCluster", "k-means++ per key group and per k, knuckle-point k (S/cluster/KMeansPlusPlusCluster.scala)")
def kmeanspp(args):
    """Records ``key..,x1..xD`` grouped by ``id.fieldOrdinals``; for every group and every k of
    ``num.clusters`` a D^2-seeded k-means (``num.clustGroup`` restarts, ``num.iter`` Lloyd steps) runs
    batched on the device; output per group: ``key..,k,sse`` lines and ``key..,knuckle,k``; the
    centroids go to ``cluster.outputPath`` as ``key..,k,i,c..``.  Native path: each rank reads its
    byte range and sends every record to the rank owning its group (one all-to-all; groups in
    string order cut into contiguous blocks), which fits its groups."""
    from ..data.table import _literal
    from ..models.cluster import KMeans
    ctx = JobContext(args, app="kMeansPlusPlusCluster")
    kords = ctx.get_int_list("id.fieldOrdinals", []) if ctx.get_str("id.fieldOrdinals", "") else []
    ks = ctx.get_int_list("num.clusters")
    prec = ctx.get_int("output.precision", 3)
    attrs = ctx.get_int_list("attr.ordinals", None)
    lit = _literal(ctx.delim_in)
    groups = _kmeanspp_groups_native(ctx, kords, attrs) if lit is not None and len(lit) == 1 else \
        _kmeanspp_groups_rows(ctx, kords, attrs)
    d = ctx.delim_out
    out, cents = [], []
    local = _LocalComm()
    Xs = [X.to(ctx.device) for _, X in groups]
    models = [KMeans([c for c in ks if c <= X.shape[0]], n_init=ctx.get_int("num.clustGroup", 10),
                     max_iter=ctx.get_int("num.iter", 10), init="k-means++", comm=local) for X in Xs]
    inits = KMeans.init_many(models, Xs)        # every group's seeding in one batched pass
    for (k, _), X, km, C0 in zip(groups, Xs, models, inits):
        kk = km.ks
        km.fit(X, init_centroids=C0)
        for c in kk:
            run = km.best[c]
            out.append(d.join(list(k) + [str(c), fmt(run.sse, prec)]))
            cents += [d.join(list(k) + [str(c), str(i)] + [fmt(v, prec) for v in cc])
                      for i, cc in enumerate(run.centroids.cpu().tolist())]
        if len(kk) > 2:
            out.append(d.join(list(k) + ["knuckle", str(km.knuckle_k())]))
    ctx.emit(out)
    cp = ctx.get_str("cluster.outputPath", None)
    if cp:
        ctx.emit(cents, cp)


def _kmeanspp_groups_native(ctx, kords, attrs):
    """This rank's groups [(key strings, X float32 [n, D])] in key order, records in input order."""
    from ..data.records import owner_of, shuffle, sorted_key_tuples
    from ..data.table import shard_range
    comm = ctx.comm
    top = max(list(kords) + list(attrs or []) + [0]) + 1
    if attrs:
        modes = "".join("d" if i in kords else ("n" if i in attrs else "x") for i in range(top))
        rec = ctx.records(modes=modes, tail_mode="x", numeric=True)
        cols = list(attrs)
    else:   # every non-key field is a coordinate (all lines as wide as the first one)
        modes = "".join("d" if i in kords else "n" for i in range(top))
        rec = ctx.records(modes=modes, tail_mode="n", numeric=True)
        w = torch.tensor([rec.width() if rec.n_lines else 0], dtype=torch.long)
        if comm.is_distributed:
            comm.all_reduce(w, "max")
        cols = [i for i in range(int(w)) if i not in kords]
    kpos, G, ktab = sorted_key_tuples(rec, [rec.field(o) for o in kords], comm)
    owner = owner_of(kpos, G, comm.world) if comm.is_distributed else torch.zeros_like(kpos)
    sh = shuffle(comm, owner, [kpos] + [rec.field(c, numeric=True) for c in cols])
    kp = sh[0].cpu()
    X = torch.stack(sh[1:], 1).float().cpu() if cols else torch.zeros((kp.numel(), 0))
    a, b = shard_range(G, comm.rank, comm.world) if comm.is_distributed else (0, G)
    o = torch.argsort(kp, stable=True)
    kp, X = kp[o], X[o]
    cnt = torch.bincount(kp - a, minlength=b - a).tolist() if b > a else []
    out, s = [], 0
    for g, c in enumerate(cnt):
        key = tuple(rec.vocab[int(x)] for x in ktab[a + g].tolist())
        out.append((key, X[s:s + c]))
        s += c
    return out


def _kmeanspp_groups_rows(ctx, kords, attrs):
    """Regex delimiters: the split-row path."""
    groups = defaultdict(list)
    for r in ctx.rows(shard=False):
        cols = attrs or [i for i in range(len(r)) if i not in kords]
        groups[tuple(r[o] for o in kords)].append([float(r[c]) for c in cols])
    keys = sorted(groups)
    if ctx.comm.is_distributed:
        from ..data.table import shard_range
        a, b = shard_range(len(keys), ctx.comm.rank, ctx.comm.world)
        keys = keys[a:b]
    return [(k, torch.tensor(groups[k], dtype=torch.float32)) for k in keys]


class _LocalComm:
    """Single-process view: per-key models are independent (no cross-rank reduction)."""
    world, rank, is_distributed, is_root = 1, 0, False, True

    def all_reduce(self, t, op="sum"):
        return t

    def all_reduce_coalesced(self, ts, op="sum"):
        return None

    def barrier(self):
        return None


# ================================================================================================
# nearest-neighbour pipeline (R/knn.sh)
# ================================================================================================
@job("sameTypeSimilarity", "mixed-type all-pairs distances between a training and a test set (sifarish SameTypeSimilarity, R/knn.sh computeDistance)")
def same_type_similarity(args):
    """Both sets (``--train`` and ``--input``; or one input with ``sts.base.set.split.prefix``
    file-name prefixes) are encoded with the schema's mixed-type distance (numeric range-scaled,
    categorical mismatch, field weights) into a euclidean embedding, and the distances of every
    (train, test) pair are one device GEMM per block.  Output (``sts.output.id.first``):
    ``trainId,testId,dist*scale,trainClass,testClass`` — the layout the NearestNeighbor mapper
    and FeatureCondProbJoiner read (J/knn/NearestNeighbor.java:130-183).  ``sts.top.match.count``
    keeps only the k nearest train records per test record (fused distance + top-k kernel)."""
    from ..ops.distance import encode_mixed, knn, knn_mixed, pairwise, split_mixed
    ctx = JobContext(args, "sts.")
    schema = ctx.schema("same.schema.file.path")
    if args.train:
        tr_path, te_path = args.train, args.input
    else:
        from .common import input_files
        pref = ctx.get_str("base.set.split.prefix", "tr")
        files = input_files(args.input)
        tr_path = ",".join(str(f) for f in files if f.name.startswith(pref))
        te_path = ",".join(str(f) for f in files if not f.name.startswith(pref))
    # both sets are row-sharded; the training shards travel the ring (top-k) or are all-gathered
    # once (all pairs); output columns come from the raw line bytes of both sets
    tr = ctx.table(path=tr_path, schema=schema, raw_numeric=True)
    te = ctx.table(path=te_path, schema=schema, raw_numeric=True)
    comm = ctx.comm
    ranges = {}
    for j, f in enumerate(tr.numeric_fields):
        x = torch.cat([tr.numeric[j, : tr.n], te.numeric[j, : te.n].to(tr.numeric.device)])
        x = torch.nan_to_num(x)
        lo = x.min().view(1) if x.numel() else torch.full((1,), math.inf, device=x.device)
        hi = x.max().view(1) if x.numel() else torch.full((1,), -math.inf, device=x.device)
        if comm.is_distributed:
            comm.all_reduce(lo, "min")
            comm.all_reduce(hi, "max")
        ranges[f.ordinal] = (float(f.min) if f.min is not None else float(lo), float(f.max) if f.max is not None else float(hi))
    nf = max(1, len(tr.numeric_fields) + len(tr.binned_fields))
    topk = ctx.get_int("top.match.count", 0)
    onehot = sum(f.num_bins for f in tr.binned_fields if f.is_categorical)
    # wide categoricals: the column-wise mixed kernel instead of a one-hot embedding (GPU top-k)
    use_mixed = (0 < topk <= 32 and tr.device.type == "cuda" and onehot > 64
                 and len(tr.numeric_fields) + len(tr.binned_fields) <= 32)
    scale = ctx.get_float("distance.scale", 1000.0)
    idf = schema.id_field
    dl = ctx.native_delim() or ","
    cls_vals = list(te.class_field.cardinality) if te.class_field is not None else []
    lab = lambda t: (t.labels[: t.n].long().cpu() if t.labels is not None else torch.full((t.n,), -1, dtype=torch.long))
    # training rows' identity (line bytes + class codes) on every rank: one packed all-gather
    from ..data.lines import LineSpans
    tr_spans = _as_spans(tr)
    tr_lab = lab(tr)
    if comm.is_distributed:
        buf, off = tr_spans.pack()
        g_len = comm.all_gather_v(off[1:] - off[:-1])
        tr_spans = LineSpans.from_packed(comm.all_gather_v(buf),
                                         torch.cat([torch.zeros(1, dtype=torch.long), torch.cumsum(g_len, 0)]))
        tr_lab = comm.all_gather_v(tr_lab)
    te_spans, te_lab = _as_spans(te), lab(te)
    tr_base = tr.row_offset

    def pair_columns(it, iq, dist):
        """Output columns of pairs (global train row ``it``, local test row ``iq``)."""
        tid = tr_spans.select(it).column("rf", idf.ordinal, dl) if idf is not None else ("i", it)
        qid = te_spans.select(iq).column("rf", idf.ordinal, dl) if idf is not None else ("i", iq + te.row_offset)
        return [tid, qid, ("i", dist), ("s", cls_vals, tr_lab[it]), ("s", cls_vals, te_lab[iq])]

    if topk > 0:
        from ..ops.distance import distributed_knn, distributed_knn_mixed
        if use_mixed:
            An, Ac, wc = split_mixed(tr, ranges=ranges)
            Bn, Bc, _ = split_mixed(te, ranges=ranges)
            dist, idx = distributed_knn_mixed(Bn, Bc, An, Ac, wc, topk, comm, r_base=tr_base)
        else:
            A, B = encode_mixed(tr, ranges=ranges), encode_mixed(te, ranges=ranges)
            dist, idx = distributed_knn(B, A, topk, comm, "euclidean", r_base=tr_base)
        dist = (dist / math.sqrt(nf) * scale).round().long().cpu()
        idx = idx.cpu()
        ok = idx >= 0
        iq = torch.arange(idx.shape[0]).view(-1, 1).expand_as(idx)[ok]
        ctx.emit_columns(pair_columns(idx[ok], iq, dist[ok]), int(ok.sum()))
        return
    from ..data.records import format_lines
    A, B = encode_mixed(tr, ranges=ranges), encode_mixed(te, ranges=ranges)
    if comm.is_distributed:
        A = comm.all_gather_v(A.contiguous())
    ntr = A.shape[0]
    parts = []
    step = max(1, (1 << 22) // max(ntr, 1))
    for s0 in range(0, te.n, step):
        D = (pairwise(B[s0:s0 + step], A) / math.sqrt(nf) * scale).round().long().cpu()
        nq = D.shape[0]
        it = torch.arange(ntr).repeat(nq)
        iq = torch.arange(s0, s0 + nq).repeat_interleave(ntr)
        parts.append(format_lines(pair_columns(it, iq, D.reshape(-1)), nq * ntr, ctx.delim_out))
    ctx.emit_text(b"".join(parts))


def _as_spans(t):
    """A table's kept input lines as byte spans (data/lines.LineSpans)."""
    from ..data.lines import LineSpans
    if isinstance(t.lines, LineSpans):
        return t.lines
    return LineSpans.from_strings(list(t.lines or [""] * t.n))


@job("featureCondProbJoiner", "join NB feature posteriors of training records onto distance pairs (J/knn/FeatureCondProbJoiner.java, fcb.*)")
def cond_prob_joiner(args):
    """Input: the distance pairs and the ``bayesianPredictor`` prob-only files (file name prefix
    ``fcb.feature.cond.prob.split.prefix``).  Output per pair:
    ``testId,testClass,trainId,distance,trainClass,trainClassPostProb`` (:153-178)."""
    from .common import input_files
    ctx = JobContext(args, "fcb.")
    pref = ctx.get_str("feature.cond.prob.split.prefix", "condProb")
    files = input_files(args.input)
    if args.model:
        files += input_files(args.model)
    prob_files = [f for f in files if f.name.startswith(pref)]
    pair_files = [f for f in files if not f.name.startswith(pref)]
    if ctx.native_delim() is not None and prob_files and pair_files:
        return _cond_prob_joiner_native(ctx, prob_files, pair_files)
    sp = ctx.split
    post = {}
    for f in prob_files:
        for l in f.read_text().splitlines():
            if not l.strip():
                continue
            p = sp(l)
            cls = p[-1]
            for i in range(2, len(p) - 1, 2):
                if p[i] == cls:
                    post[p[0]] = (cls, p[i + 1])
                    break
    d = ctx.delim_out
    lines = [l for f in pair_files for l in f.read_text().splitlines() if l.strip()]
    if ctx.comm.is_distributed:
        from ..data.table import shard_range
        a, b = shard_range(len(lines), ctx.comm.rank, ctx.comm.world)
        lines = lines[a:b]
    out = []
    for l in lines:
        p = sp(l)
        if p[0] in post:
            c, pr = post[p[0]]
            out.append(d.join([p[1], p[4], p[0], p[2], c, pr]))
    ctx.emit(out)


def _cond_prob_joiner_native(ctx, prob_files, pair_files):
    """Native, data-parallel join (J/knn/FeatureCondProbJoiner.java:105-178 without the shuffle).

    * The posterior table (one prob-only line per TRAINING record, the small side) is tokenized
      whole by every rank — ``id,prior,cls,prob,...,cls,prob,actualClass`` — and reduced on the
      device to one (class code, probability code) per line: the first ``cls`` equal to the line's
      last token (the reducer's ``classVal`` search, :152-158), as strings of its dictionary.
    * The distance pairs (``trainId,testId,dist,trainClass,testClass``: the O(test x train) side)
      are tokenized by byte range — each rank reads only its range — with only ``trainId``
      dictionary-coded; one host pass over the DICTIONARY (not the pairs) maps train-id codes to
      posterior lines, and the join itself is one device gather.
    * Output ``testId,testClass,trainId,dist,trainClass,postProb`` (:170-175) is assembled by the
      native formatter from raw input fields and the posterior strings (device formatter for
      large outputs).  Pairs whose training id has no posterior line are dropped."""
    lit = ctx.native_delim()
    prob = ctx.records([str(f) for f in prob_files], shard=False, modes="", tail_mode="d")
    P = prob.n_lines
    dev = prob.device
    M, cnt = prob.padded(dtype=torch.int32)
    if P and M.shape[1] >= 4:
        last = prob.codes[prob.off[1:] - 1].to(torch.int32)
        cand = M[:, 2:M.shape[1] - 1:2]                                  # cls tokens at 2, 4, ...
        pos = 2 + 2 * torch.arange(cand.shape[1], device=dev)
        match = (cand == last.view(-1, 1)) & (pos.view(1, -1) < (cnt.view(-1, 1) - 1))
        has = match.any(1)
        first = match.int().argmax(1)
        rows = torch.arange(P, device=dev)
        cls_code = M[rows, 2 + 2 * first]
        prob_code = M[rows, 3 + 2 * first]
    else:
        has = torch.zeros(P, dtype=torch.bool, device=dev)
        cls_code = prob_code = torch.zeros(P, dtype=torch.int32, device=dev)
    ids = prob.strings(M[:, 0].cpu()) if P else []
    ok_host = has.cpu().tolist()
    line_of = {}
    for i, (k, ok) in enumerate(zip(ids, ok_host)):
        if ok and k not in line_of:
            line_of[k] = i
    pairs = ctx.records([str(f) for f in pair_files], modes="d", tail_mode="x")
    lut = torch.tensor([line_of.get(v, -1) for v in pairs.vocab] + [-1], dtype=torch.int64, device=pairs.device)
    tid = pairs.field(0).long()
    line = lut[torch.where(tid >= 0, tid, torch.full_like(tid, len(pairs.vocab)))]
    keep = torch.nonzero(line >= 0).view(-1)
    sel = line[keep].to(cls_code.device)
    spans = pairs.line_spans().select(keep)
    cols = [spans.column("rf", 1, lit), spans.column("rf", 4, lit), spans.column("rf", 0, lit),
            spans.column("rf", 2, lit), ("s", prob.vocab, cls_code[sel].to(pairs.device)),
            ("s", prob.vocab, prob_code[sel].to(pairs.device))]
    ctx.emit_columns(cols, int(keep.numel()))


@job("nearestNeighbor", "kNN from precomputed distance pairs (J/knn/NearestNeighbor.java, nen.*; R/knn.sh knnClassifier)")
def nearest_neighbor(args):
    """Input pairs ``trainId,testId,dist,trainClass[,testClass]`` or, class-conditioned, the
    joiner's ``testId,testClass,trainId,dist,trainClass,postProb``.  Per test record the
    ``nen.top.match.count`` nearest (device segmented sort on (test, distance)) are scored by the
    kernel function of ``models/knn.NearestNeighbor`` (none / linearMultiplicative / linearAdditive
    / gaussian, optional inverse-distance and class-conditional weights) and classified (max score,
    decision threshold or cost-based).  Output ``testId[,cls,score...][,actual],predicted``
    (:317-406); ``Validation`` counters on stdout."""
    from ..models.knn import NearestNeighbor
    ctx = JobContext(args, "nen.")
    val = ctx.get_bool("validation.mode", True)
    ccw = ctx.get_bool("class.condtion.weighted", False) or ctx.get_bool("class.condition.weighted", False)
    k = ctx.get_int("top.match.count", 10)
    out_distr = ctx.get_bool("output.class.distr", False)
    from ..data.table import _literal
    lit = _literal(ctx.delim_in)
    if lit is not None and len(lit) == 1:
        rec = ctx.records(modes="ddxndn" if ccw else "xdnd", tail_mode="d", numeric=True)
        W = rec.width()
        widths = ctx.comm.all_gather_object(W) if ctx.comm.is_distributed else [W]
        ok_w = {w for w in widths if w not in (0, None)}
        if len(ok_w) <= 1 and None not in widths and (ok_w <= ({6} if ccw else {4, 5})):
            return _nearest_neighbor_native(ctx, rec, next(iter(ok_w), 6 if ccw else 4), ccw, val, k, out_distr)
    rows = ctx.rows(shard=False)
    if ccw:
        te_id = [r[0] for r in rows]
        te_cls = [r[1] for r in rows]
        dist = [float(r[3]) for r in rows]
        tr_cls = [r[4] for r in rows]
        w = [float(r[5]) for r in rows]
    else:
        te_id = [r[1] for r in rows]
        dist = [float(r[2]) for r in rows]
        tr_cls = [r[3] for r in rows]
        te_cls = [r[4] if len(r) > 4 else "" for r in rows]
        w = None
    classes = ctx.get_list("class.attribute.values", None) or sorted(set(tr_cls))
    ci = {c: i for i, c in enumerate(classes)}
    tests = sorted(set(te_id))
    if ctx.comm.is_distributed:
        from ..data.table import shard_range
        a, b = shard_range(len(tests), ctx.comm.rank, ctx.comm.world)
        mine = set(tests[a:b])
        sel = [i for i, t in enumerate(te_id) if t in mine]
        tests = tests[a:b]
    else:
        sel = list(range(len(rows)))
    ti = {t: i for i, t in enumerate(tests)}
    T = torch.tensor([ti[te_id[i]] for i in sel], dtype=torch.long)
    Dv = torch.tensor([dist[i] for i in sel], dtype=torch.float64)
    Cv = torch.tensor([ci[tr_cls[i]] for i in sel], dtype=torch.long)
    order = torch.argsort(Dv, stable=True)
    order = order[torch.argsort(T[order], stable=True)]
    T, Dv, Cv = T[order], Dv[order], Cv[order]
    Wv = torch.tensor([w[sel[i]] for i in order.tolist()], dtype=torch.float64) if w is not None else None
    first = torch.ones_like(T, dtype=torch.bool)
    first[1:] = T[1:] != T[:-1]
    from ..data.records import segment_rank
    rank = segment_rank(first)
    keep = rank < k
    nn = NearestNeighbor.from_config(ctx.cfg)
    nt, C = len(tests), len(classes)
    dk = torch.full((nt, k), math.inf, dtype=torch.float32)
    ck = torch.zeros((nt, k), dtype=torch.long)
    dk[T[keep], rank[keep]] = (Dv[keep] / 1000.0).float()     # distances are scaled by 1000 upstream
    ck[T[keep], rank[keep]] = Cv[keep]
    s = nn._kernel_scores(dk)
    s = torch.where(torch.isfinite(dk), s, torch.zeros_like(s))   # empty neighbour slots do not vote
    if Wv is not None:
        wk = torch.zeros((nt, k), dtype=torch.float32)
        wk[T[keep], rank[keep]] = Wv[keep].float()
        s = s * wk
    scores = torch.zeros((nt, C), dtype=torch.float32).scatter_add_(1, ck, s.float())
    pred = scores.argmax(1)
    if nn.decision_threshold > 0 and C == 2:
        ratio = scores[:, 1] / scores[:, 0].clamp_min(1e-12)
        pred = (ratio > nn.decision_threshold).long()
    actual = {}
    for i in sel:
        actual[te_id[i]] = te_cls[i]
    d = ctx.delim_out
    out = []
    correct = 0
    for t, name in enumerate(tests):
        parts = [name]
        if out_distr:
            for c in range(C):
                parts += [classes[c], f"{float(scores[t, c]):g}"]
        if val:
            parts.append(actual[name])
        pv = classes[int(pred[t])]
        parts.append(pv)
        correct += int(val and actual[name] == pv)
        out.append(d.join(parts))
    ctx.emit(out)
    if val:
        acc = torch.tensor([float(correct), float(len(tests))])
        ctx.all_reduce(acc)
        ctx.report({"Validation": {"Correct": int(acc[0]), "Incorrect": int(acc[1] - acc[0])}})


def _nearest_neighbor_native(ctx, rec, W, ccw, val, k, out_distr):
    """nearestNeighbor on the native record table: candidate pairs shuffled to the rank owning the
    test record (test ids in string order, contiguous blocks: the reducer key order), a device
    segmented sort on (test, distance) with the global input order as tie-break, the kernel-weighted
    vote of models/knn.NearestNeighbor as [tests, k] tensors, and the native formatter for the
    output (J/knn/NearestNeighbor.java:317-406)."""
    from ..data.records import format_lines, owner_of, shuffle, sorted_keys
    from ..models.knn import NearestNeighbor
    comm = ctx.comm
    dev = rec.device
    n = rec.n_lines
    Cd = rec.codes.view(n, W).long() if n else rec.codes.view(0, W).long()
    Nd = rec.nums.view(n, W) if n else rec.nums.view(0, W)
    if ccw:
        te, te_c, dist, tr_c, w = Cd[:, 0], Cd[:, 1], Nd[:, 3], Cd[:, 4], Nd[:, 5]
    else:
        te, dist, tr_c = Cd[:, 1], Nd[:, 2], Cd[:, 3]
        te_c = Cd[:, 4] if W > 4 else torch.full_like(te, -1)
        w = None
    classes = ctx.get_list("class.attribute.values", None)
    if classes is None:
        present = torch.unique(tr_c[tr_c >= 0]).tolist()
        classes = ctx.union(rec.vocab[c] for c in present)
    C = len(classes)
    ci = rec.index(classes).long() if len(rec.vocab) else torch.zeros(0, dtype=torch.long, device=dev)
    cls_idx = ci[tr_c.clamp_min(0)] if n and ci.numel() else torch.full_like(tr_c, -1)
    keys, pos = sorted_keys(rec, te, comm)
    E = keys.numel()
    tpos = pos[te] if n else te
    seq = torch.arange(n, device=dev) + rec.line_base
    owner = owner_of(tpos, E, comm.world) if comm.is_distributed else torch.zeros_like(tpos)
    cols = [tpos, dist, cls_idx, te_c, seq] + ([w] if w is not None else [])
    cols = shuffle(comm, owner, cols)
    tpos, dist, cls_idx, te_c, seq = cols[:5]
    w = cols[5] if len(cols) > 5 else None
    # this rank's tests: the contiguous block of sorted positions it owns
    from ..data.table import shard_range
    a, b = shard_range(E, comm.rank, comm.world) if comm.is_distributed else (0, E)
    nt = b - a
    t = tpos - a
    o = torch.argsort(seq, stable=True)
    o = o[torch.argsort(dist[o], stable=True)]
    o = o[torch.argsort(t[o], stable=True)]
    t, dist, cls_idx, te_c, seq = t[o], dist[o], cls_idx[o], te_c[o], seq[o]
    w = w[o] if w is not None else None
    m = t.numel()
    first = torch.ones(m, dtype=torch.bool, device=dev)
    if m > 1:
        first[1:] = t[1:] != t[:-1]
    from ..data.records import segment_rank
    rank = segment_rank(first)
    keep = (rank < k) & (cls_idx >= 0)      # neighbours of an unknown class do not vote
    nn = NearestNeighbor.from_config(ctx.cfg)
    dk = torch.full((nt, k), math.inf, dtype=torch.float32, device=dev)
    ck = torch.zeros((nt, k), dtype=torch.long, device=dev)
    dk[t[keep], rank[keep]] = (dist[keep] / 1000.0).float()   # distances are scaled by 1000 upstream
    ck[t[keep], rank[keep]] = cls_idx[keep]
    s = nn._kernel_scores(dk)
    s = torch.where(torch.isfinite(dk), s, torch.zeros_like(s))   # empty neighbour slots do not vote
    if w is not None:
        wk = torch.zeros((nt, k), dtype=torch.float32, device=dev)
        wk[t[keep], rank[keep]] = w[keep].float()
        s = s * wk
    scores = torch.zeros((nt, max(C, 1)), dtype=torch.float32, device=dev).scatter_add_(1, ck, s.float())
    pred = scores.argmax(1)
    if nn.decision_threshold > 0 and C == 2:
        ratio = scores[:, 1] / scores[:, 0].clamp_min(1e-12)
        pred = (ratio > nn.decision_threshold).long()
    # actual class of a test: its last candidate row in input order
    last = torch.full((nt,), -1, dtype=torch.long, device=dev)
    if m:
        last.scatter_reduce_(0, t, seq, "amax")
        at = torch.full((nt,), -1, dtype=torch.long, device=dev)
        hit = seq == last[t]
        at[t[hit]] = te_c[hit]
    else:
        at = torch.full((nt,), -1, dtype=torch.long, device=dev)
    names = keys[a:b]
    voc = rec.vocab
    cols_f = [("s", voc, names.int().cpu())]
    if out_distr:
        sc = scores.double().cpu()
        for c in range(C):
            cols_f += [("c", classes[c]), ("f", sc[:, c].contiguous(), -1)]
    if val:
        cols_f.append(("s", voc, at.int().cpu()))
    cols_f.append(("s", list(classes), pred.int().cpu()))
    ctx.emit_columns(cols_f, nt)
    if val:
        av = rec.index(classes).long()
        act_cls = torch.where(at >= 0, av[at.clamp_min(0)] if av.numel() else at, torch.full_like(at, -2))
        correct = float((act_cls == pred).sum())
        acc = torch.tensor([correct, float(nt)], dtype=torch.float64)
        ctx.all_reduce(acc)
        ctx.report({"Validation": {"Correct": int(acc[0]), "Incorrect": int(acc[1] - acc[0])}})


# ================================================================================================
# model prediction / data partitioning
# ================================================================================================
@job("modelPredictor", "decision-tree model (ensemble) predictor (J/model/ModelPredictor.java, mop.*)")
def model_predictor(args):
    """``mop.model.dir.path`` + ``mop.model.file.names`` (decision-path JSON or native tree state
    files; several = weighted voting ensemble), ``mop.output.mode`` withRecord | withKId |
    withActualClassAttr; the error rate goes to ``map.error.rate.file.path`` when given."""
    from ..models.tree import DecisionPathModel
    ctx = JobContext(args, "mop.")
    mdir = Path(ctx.path("model.dir.path", "model"))
    names = ctx.get_list("model.file.names", None) or sorted(p.name for p in mdir.glob("*.json"))
    models = [DecisionPathModel(json.loads((mdir / n).read_text())) for n in names]
    weights = ctx.get_float_list("ensemble.memeber.weights", None) or [1.0] * len(models)
    classes = sorted({c for m in models for c in m.class_values})
    mode = ctx.get_str("output.mode", "withRecord")
    id_o = ctx.get_int("rec.id.ordinal", 0)
    co = ctx.get_int("rec.class.attr.ordinal", ctx.get_int("class.attr.ord", -1))
    from ..data.table import _literal
    lit = _literal(ctx.delim_in)
    if lit is None or len(lit) != 1:
        return _model_predictor_rows(ctx, models, weights, classes, mode, id_o, co)
    from ..data.records import format_lines, numeric_lut
    from ..utils.rules import RecordColumns
    # native path: the predicate fields are tokenized once ('d' for categorical sets and the class,
    # 'n' for thresholds), every model's paths are evaluated column-wise on the device, and the
    # output comes from the raw line bytes + the vote winners
    cat, num = set(), set()
    for m in models:
        for pth in m.paths:
            for pr in pth["predicates"]:
                it = pr["predicateStr"].split()
                if len(it) >= 3 and it[0].lstrip("-").isdigit():
                    (cat if it[1] == "in" else num).add(int(it[0]))
    dict_ords = cat | ({co} if co >= 0 else set())
    top = max(list(cat | num) + [co, 0]) + 1
    modes = "".join("d" if i in dict_ords else ("n" if i in num else "x") for i in range(top))
    rec = ctx.records(modes=modes, tail_mode="x", numeric=True, trim=True)
    cols_src = RecordColumns(rec)
    both = num & dict_ords
    if both:   # a field used as a category and as a number: its numbers from the dictionary strings
        lut = numeric_lut(rec.vocab, rec.device)
        plain = cols_src.numeric
        cols_src.numeric = lambda o: (torch.where(rec.field(o) >= 0, lut[rec.field(o).long().clamp_min(0)],
                                                  torch.full((rec.n_lines,), float("nan"), dtype=torch.float64,
                                                             device=rec.device))
                                      if o in both else plain(o))
    n = rec.n_lines
    votes = torch.zeros((n, len(classes)), dtype=torch.float64, device=rec.device)
    for m, w in zip(models, weights):
        pr, _ = m.predict_proba_cols(cols_src)
        idx = torch.tensor([classes.index(c) for c in m.class_values], dtype=torch.long, device=rec.device)
        win = idx[pr.argmax(1)]
        votes.scatter_add_(1, win.view(-1, 1), torch.full((n, 1), float(w), dtype=torch.float64, device=rec.device))
    pred = votes.argmax(1)
    spans = rec.line_spans()
    pcol = ("s", list(classes), pred.int())
    if mode == "withKId":
        cols = [spans.column("rf", id_o, lit), pcol]
    elif mode == "withActualClassAttr":
        cols = [spans.column("rf", id_o, lit), spans.column("rf", co, lit), pcol]
    else:
        cols = [spans.column("r", delims=lit), pcol]
    ctx.emit_columns(cols, n)
    if co >= 0:
        has = rec.lens() > co
        actual = rec.map_codes(rec.field(co), classes).long()
        err = torch.tensor([float(((actual != pred) & has).sum()), float(has.sum())], dtype=torch.float64)
    else:
        err = torch.zeros(2, dtype=torch.float64)
    _report_error_rate(ctx, err)


def _report_error_rate(ctx, err: torch.Tensor) -> None:
    ctx.all_reduce(err)
    rate = float(err[0]) / max(float(err[1]), 1)
    ep = ctx.cfg.values.get("map.error.rate.file.path")
    ctx.check()
    if ep and ctx.is_root:
        Path(ep).parent.mkdir(parents=True, exist_ok=True)
        Path(ep).write_text(f"errorRate={rate:.6f}\n")
    ctx.report({"errorRate": rate})


def _model_predictor_rows(ctx, models, weights, classes, mode, id_o, co):
    """Regex delimiters: the split-row path."""
    rows = ctx.rows()
    votes = torch.zeros((len(rows), len(classes)), dtype=torch.float64)
    for m, w in zip(models, weights):
        pr, _ = m.predict_proba_rows(rows)
        idx = torch.tensor([classes.index(c) for c in m.class_values], dtype=torch.long)
        win = idx[pr.argmax(1)]
        votes.scatter_add_(1, win.view(-1, 1), torch.full((len(rows), 1), float(w), dtype=torch.float64))
    pred = votes.argmax(1).tolist()
    d = ctx.delim_out
    out, errors, total = [], 0, 0
    for r, p in zip(rows, pred):
        pv = classes[p]
        if co >= 0 and co < len(r):
            total += 1
            errors += int(r[co].strip() != pv)
        if mode == "withKId":
            out.append(f"{r[id_o]}{d}{pv}")
        elif mode == "withActualClassAttr":
            out.append(f"{r[id_o]}{d}{r[co]}{d}{pv}")
        else:
            out.append(f"{d.join(r)}{d}{pv}")
    ctx.emit(out)
    _report_error_rate(ctx, torch.tensor([float(errors), float(total)], dtype=torch.float64))


@job("dataPartitioner", "partition records by the best (or random top) split of classPartitionGenerator (J/tree/DataPartitioner.java, dap.*)")
def data_partitioner(args):
    """Split candidates ``attr,splitKey,stat`` from ``dap.split.path``; ``dap.split.selection.strategy``
    best (max stat) or randomAmongTop (``dap.num.top.splits``); records are routed by the split's
    segment index (the K bucketize op) into ``<out>/split=<attr>/segment=<j>/part-NNNNN``."""
    from ..models.splitstat import parse_split_key
    ctx = JobContext(args, "dap.")
    schema = ctx.schema()
    cands = [ctx.split(l) for l in ctx.all_lines(ctx.path("split.path", "model"))]
    cands.sort(key=lambda p: -float(p[-1]))
    strat = ctx.get_str("split.selection.strategy", "best")
    if strat == "best":
        pick = cands[0]
    else:
        g = torch.Generator().manual_seed(ctx.get_int("random.seed", 0))
        pick = cands[int(torch.randint(0, min(ctx.get_int("num.top.splits", 5), len(cands)), (1,), generator=g))]
    attr = int(pick[0])
    key = ",".join(pick[1:-1]) if len(pick) > 3 else pick[1]
    f = schema.find_field_by_ordinal(attr)
    rec = ctx.try_records(modes=field_modes({attr: "d" if f.is_categorical else "n"}), tail_mode="x",
                          numeric=not f.is_categorical)
    if rec is not None:
        # native: the split field tokenized once, segments from one lookup / bucketize, every
        # segment's lines written from their raw bytes by the native formatter
        if f.is_categorical:
            groups = parse_split_key(key, "cat")
            lut = {v: j for j, g in enumerate(groups) for v in g}
            tab = torch.tensor([lut.get(v, len(groups) - 1) for v in rec.vocab] or [0], dtype=torch.long)
            c = rec.field(attr).long().cpu()
            seg = torch.where(c >= 0, tab[c.clamp_min(0)], torch.full_like(c, len(groups) - 1))
        else:
            pts = torch.tensor(parse_split_key(key, "num"), dtype=torch.float64)
            seg = torch.bucketize(rec.field(attr, numeric=True).double().cpu(), pts, right=False)
        spans = rec.line_spans()
        base = Path(args.output) / f"split={attr}"
        segs = torch.unique(seg).tolist()
        for sv in segs:
            p = base / f"segment={sv}"
            p.mkdir(parents=True, exist_ok=True)
            sel = spans.select(seg == sv)
            from ..data.records import format_lines
            format_lines([sel.column("r", delims=ctx.native_delim())], len(sel), ctx.delim_out,
                         path=str(p / f"part-{ctx.comm.rank:05d}"))
        ctx.report({"split": attr, "key": key, "segments": len(segs)})
        return
    rows = ctx.rows()
    if f.is_categorical:
        groups = parse_split_key(key, "cat")
        lut = {v: j for j, g in enumerate(groups) for v in g}
        seg = [lut.get(r[attr], len(groups) - 1) for r in rows]
    else:
        pts = torch.tensor(parse_split_key(key, "num"), dtype=torch.float64)
        x = torch.tensor([float(r[attr]) for r in rows], dtype=torch.float64)
        seg = torch.bucketize(x, pts, right=False).tolist()
    d = ctx.delim_out
    by = defaultdict(list)
    for r, s in zip(rows, seg):
        by[s].append(d.join(r))
    base = Path(args.output) / f"split={attr}"
    ctx.check()
    for s, ls in sorted(by.items()):
        p = base / f"segment={s}"
        p.mkdir(parents=True, exist_ok=True)
        (p / f"part-{ctx.comm.rank:05d}").write_text("\n".join(ls) + "\n")
    ctx.report({"split": attr, "key": key, "segments": len(by)})


# ================================================================================================
# batch bandits (MR map-only, per group)
# ================================================================================================
def _batch_bandit(args, prefix: str, strategy_fn):
    """Rows ``group,item,count,reward`` (ordinals ``count.ordinal`` / ``reward.ordinal``); per group
    (string order) the selected batch of items, lines ``group,item``.  Native path: each rank
    reads its byte range, rows go to the rank owning their group (one all-to-all; input order kept
    inside a group), the dense [groups, items] state is one scatter, and the selection's draws are
    keyed by the global group index (``batch_select(group_base=...)``), so the output does not
    depend on the world size."""
    from functools import partial
    from ..data.table import _literal, shard_range
    from ..models.bandit import batch_select
    ctx = JobContext(args, prefix)
    co, ro = ctx.get_int("count.ordinal", 2), ctx.get_int("reward.ordinal", 3)
    mean_in = ctx.get_bool("reward.is.mean", True)
    comm = ctx.comm
    bs = {}
    cp = ctx.get_str("group.item.count.path", None)
    if cp and Path(cp).exists():
        for l in ctx.all_lines(cp):
            p = ctx.split(l)
            bs[p[0]] = int(p[1])
    glob = ctx.get_int("global.batch.size", 1)
    rnd = ctx.get_int("current.round.num", 1)
    lit = _literal(ctx.delim_in)
    if lit is None or len(lit) != 1:
        return _batch_bandit_rows(ctx, co, ro, mean_in, bs, glob, rnd, strategy_fn)
    from ..data.records import format_lines, owner_of, segment_rank, shuffle, sorted_keys
    top = max(2, co + 1, ro + 1)
    modes = "dd" + "".join("n" if i in (co, ro) else "x" for i in range(2, top))
    rec = ctx.records(modes=modes, tail_mode="x", numeric=True)
    dev = rec.device
    zero = torch.zeros(rec.n_lines, dtype=torch.float64, device=dev)
    gcode, icode = rec.field(0).long(), rec.field(1).long()
    c = rec.field(co, numeric=True) if co >= 0 else zero
    w = rec.field(ro, numeric=True) if ro >= 0 else zero
    keys, pos = sorted_keys(rec, gcode, comm)
    G = keys.numel()
    gp = pos[gcode]
    owner = owner_of(gp, G, comm.world) if comm.is_distributed else torch.zeros_like(gp)
    gp, ic, c, w = shuffle(comm, owner, [gp, icode, c, w])
    o = torch.argsort(gp, stable=True)
    gp, ic, c, w = gp[o], ic[o], c[o], w[o]
    first = torch.ones_like(gp, dtype=torch.bool)
    first[1:] = gp[1:] != gp[:-1]
    j = segment_rank(first)
    a, b = shard_range(G, comm.rank, comm.world) if comm.is_distributed else (0, G)
    Gl = b - a
    nmax = torch.tensor([int(j.max()) + 1 if j.numel() else 1], dtype=torch.long)
    gstr = [rec.vocab[int(x)] for x in keys[a:b].tolist()]
    kv = torch.tensor([bs.get(g_, glob) for g_ in gstr], dtype=torch.long)
    kmax = torch.tensor([int(kv.max()) if kv.numel() else 1], dtype=torch.long)
    if comm.is_distributed:
        comm.all_reduce(nmax, "max")
        comm.all_reduce(kmax, "max")
    I, kmax = int(nmax), max(1, int(kmax))
    lg = (gp - a)
    cnt = torch.zeros((Gl, I), dtype=torch.float64, device=dev)
    rew = torch.zeros((Gl, I), dtype=torch.float64, device=dev)
    valid = torch.zeros((Gl, I), dtype=torch.bool, device=dev)
    items = torch.full((Gl, I), -1, dtype=torch.long, device=dev)
    cnt[lg, j] = c
    rew[lg, j] = w * c.clamp_min(1.0) if mean_in else w
    valid[lg, j] = True
    items[lg, j] = ic
    ctx.global_max_items = I
    sel = strategy_fn(ctx, cnt.cpu(), rew.cpu(), valid.cpu(), kmax, rnd, partial(batch_select, group_base=a))
    n_items = valid.sum(1).cpu()
    kk = torch.minimum(kv, n_items)
    take = (torch.arange(sel.shape[1]).view(1, -1) < kk.view(-1, 1)) & (sel < n_items.view(-1, 1))
    gi, si = torch.nonzero(take, as_tuple=True)
    chosen = items.cpu()[gi, sel[gi, si]]
    cols = [("s", rec.vocab, keys[a:b].cpu()[gi].int()), ("s", rec.vocab, chosen.int())]
    ctx.emit_columns(cols, int(gi.numel()))


def _batch_bandit_rows(ctx, co, ro, mean_in, bs, glob, rnd, strategy_fn):
    """Regex delimiters: the split-row path (every rank reads the input, selects a block of groups)."""
    from functools import partial
    from ..data.table import shard_range
    from ..models.bandit import batch_select
    rows = ctx.rows(shard=False)
    groups = sorted({r[0] for r in rows})
    items = defaultdict(list)
    for r in rows:
        items[r[0]].append((r[1], float(r[co]) if co >= 0 else 0.0, float(r[ro]) if ro >= 0 else 0.0))
    I = max([len(v) for v in items.values()] + [1])
    kmax = max([bs.get(g, glob) for g in groups] + [1])
    a, b = shard_range(len(groups), ctx.comm.rank, ctx.comm.world) if ctx.comm.is_distributed else (0, len(groups))
    groups = groups[a:b]
    G = len(groups)
    cnt = torch.tensor([[x[1] for x in items[g]] + [0.0] * (I - len(items[g])) for g in groups],
                       dtype=torch.float64).view(G, I)
    rw = torch.tensor([[x[2] for x in items[g]] + [0.0] * (I - len(items[g])) for g in groups],
                      dtype=torch.float64).view(G, I)
    rew = rw * cnt.clamp_min(1.0) if mean_in else rw
    valid = torch.tensor([[True] * len(items[g]) + [False] * (I - len(items[g])) for g in groups],
                         dtype=torch.bool).view(G, I)
    ctx.global_max_items = I
    sel = strategy_fn(ctx, cnt, rew, valid, kmax, rnd, partial(batch_select, group_base=a))
    d = ctx.delim_out
    out = []
    for gi_, g in enumerate(groups):
        k = min(bs.get(g, glob), len(items[g]))
        for j in sel[gi_, :k].tolist():
            if j < len(items[g]):
                out.append(f"{g}{d}{items[g][j][0]}")
    ctx.emit(out)


def _mask(score, valid):
    return torch.where(valid, score, torch.full_like(score, -math.inf))


@job("greedyRandomBandit", "epsilon-greedy / Auer greedy batch selection per group (J/reinforce/GreedyRandomBandit.java)")
def greedy_random_bandit(args):
    def fn(ctx, cnt, rew, valid, k, rnd, batch_select):
        alg = ctx.get_str("prob.reduction.algorithm", "linear")
        strat = {"linear": "linear", "logLinear": "logLinear", "auerGreedy": "auerGreedy"}.get(alg, "linear")
        sel = batch_select(cnt, _mask(rew, valid).nan_to_num(neginf=-1e30), k, strat, rnd,
                           epsilon=ctx.get_float("random.selection.prob", 0.5), seed=ctx.get_int("random.seed", 0))
        return sel
    _batch_bandit(args, "", fn)


@job("auerDeterministic", "deterministic UCB1 batch selection per group (J/reinforce/AuerDeterministic.java)")
def auer_det(args):
    def fn(ctx, cnt, rew, valid, k, rnd, batch_select):
        cnt = torch.where(valid, cnt, torch.full_like(cnt, 1e30))
        return batch_select(cnt, rew, k, "auerDeterministic", rnd)
    _batch_bandit(args, "", fn)


@job("softMaxBandit", "softmax batch selection per group (J/reinforce/SoftMaxBandit.java)")
def softmax_bandit(args):
    def fn(ctx, cnt, rew, valid, k, rnd, batch_select):
        rew = torch.where(valid, rew, torch.full_like(rew, -1e30))
        return batch_select(cnt.clamp_min(1), rew, k, "softMax", rnd, temp=ctx.get_float("temp.constant", 1.0),
                            seed=ctx.get_int("random.seed", 0))
    _batch_bandit(args, "", fn)


@job("randomFirstGreedyBandit", "explore-first then greedy batch selection (J/reinforce/RandomFirstGreedyBandit.java)")
def random_first_bandit(args):
    def fn(ctx, cnt, rew, valid, k, rnd, batch_select):
        from ..models.bandit import pac_exploration_count
        I = getattr(ctx, "global_max_items", int(valid.sum(1).max()))   # over ALL groups (world-invariant)
        if ctx.get_str("exploration.count.strategy", "simple") == "pac":
            ex = pac_exploration_count(I, ctx.get_float("pac.reward.diff", 0.2), ctx.get_float("pac.prob.diff", 0.2))
        else:
            ex = ctx.get_int("exploration.count.factor", 2) * I
        ex = max(1, ex // max(k, 1))
        rew = torch.where(valid, rew, torch.full_like(rew, -1e30))
        return batch_select(cnt.clamp_min(1), rew, k, "randomFirst", rnd, explore_count=ex, seed=ctx.get_int("random.seed", 0))
    _batch_bandit(args, "", fn)


# ================================================================================================
# record similarity
# ================================================================================================
@job("recordSimilarity", "all-pairs record distances, optionally between two sets (S/similarity/RecordSimilarity.scala, chombo RecordSimilarity)")
def record_similarity(args):
    """Numeric fields ``attr.ordinals`` (range-normalised over both sets), ids at ``id.ordinal``;
    distances of all pairs (i < j within one set, or every (base, other) pair with ``--train``)
    scaled by ``distance.scale`` and rounded; pairs above ``dist.threshold`` dropped.  Output
    ``id1,id2,[rec1,rec2,]dist`` (``output.record``), in (i, j) order.

    Data-parallel (the reference replicates every record into ``num.buckets`` bucket pairs,
    S/similarity/RecordSimilarity.scala:80-150): every rank reads only its byte range of each set;
    its base rows stay put while the other set's row blocks — numeric columns plus the raw line
    bytes — travel around the ring (``Comm.ring_iter``: the next block's transfer is posted before
    the distance tiles of the current one run on the device).  Each rank writes the pairs of its own
    base rows, sorted by (i, j), so the rank-ordered output equals the single-rank one."""
    from ..data.table import _literal
    ctx = JobContext(args, "resi.", app="recordSimilarity")
    lit = _literal(ctx.delim_in)
    if lit is None or len(lit) != 1:
        return _record_similarity_rows(ctx, args)
    from ..data.lines import LineSpans
    from ..data.records import format_lines
    from ..ops.distance import pairwise
    ords = ctx.get_int_list("attr.ordinals")
    idc = ctx.get_int("id.ordinal", 0)
    scale = ctx.get_float("distance.scale", 1000.0)
    thr = ctx.get_float("dist.threshold", math.inf)
    out_rec = ctx.get_bool("output.record", False)
    comm = ctx.comm
    top = max(list(ords) + [idc]) + 1
    modes = "".join("n" if i in ords else "x" for i in range(top))
    rA = ctx.records(modes=modes, tail_mode="x", numeric=True)
    rB = ctx.records(args.train, modes=modes, tail_mode="x", numeric=True) if args.train else None
    dev = ctx.device
    num = lambda r: (torch.stack([r.field(o, numeric=True) for o in ords], 1).float().to(dev) if r.n_lines
                     else torch.zeros((0, len(ords)), dtype=torch.float32, device=dev))
    XA = num(rA)
    XB = num(rB) if rB is not None else XA
    both = torch.cat([XA, XB]) if rB is not None else XA
    big = torch.full((len(ords),), float("inf"), device=dev)
    lo = torch.where(torch.isnan(both), big, both).amin(0) if both.shape[0] else big.clone()
    hi = torch.where(torch.isnan(both), -big, both).amax(0) if both.shape[0] else -big
    if comm.is_distributed:
        comm.all_reduce(lo, "min")
        comm.all_reduce(hi, "max")
    rng = (hi - lo).clamp_min(1e-12)
    A = (XA - lo) / rng
    B = (XB - lo) / rng if rB is not None else A
    spA = rA.line_spans()
    spB = rB.line_spans() if rB is not None else spA
    a_base = rA.line_base
    b_rec = rB if rB is not None else rA
    nB = torch.tensor([b_rec.n_lines], dtype=torch.long)
    ctx.all_reduce(nB)
    NB = int(nB)
    bbuf, boff = spB.pack()
    cdev = comm.device if (comm.is_distributed and comm.pg_backend == "nccl") else torch.device("cpu")
    payload = [B.to(cdev), torch.tensor([b_rec.line_base], dtype=torch.long, device=cdev), bbuf.to(cdev),
               boff.to(cdev)]
    nf = math.sqrt(max(len(ords), 1))
    tile = max(1, min(4096, (1 << 26) // max(1, NB // max(1, comm.world))))
    fused = (dev.type == "cuda" and math.isfinite(thr) and 1 <= len(ords) <= 64
             and os.environ.get("AVMI_RS_FUSED", "1") != "0")
    I, J, Dv, H = [], [], [], []
    blocks = []
    for h, (owner, (Bc, bbase, bb, bo)) in enumerate(comm.ring_iter(payload)):
        Bc = Bc.to(dev)
        b0 = int(bbase.cpu()[0]) if bbase.numel() else 0
        blocks.append(LineSpans.from_packed(bb, bo))
        nb = Bc.shape[0]
        if rB is None and nb and b0 + nb - 1 <= a_base:
            continue        # self-join hop entirely at or below this rank's rows: no j > i (still forwarded)
        if fused and nb and A.shape[0]:
            # GPU: one fused distance + threshold + append launch per hop (distance.hip
            # pairs_within_kernel), pairs sorted by (i, j) — no [tile, nB] distance blocks
            qi, jj, dd = _native.C().pairs_within(A.contiguous(), Bc.float().contiguous(), nf, scale, thr, rB is None,
                                                  int(a_base), int(b0))
            if qi.numel():
                I.append(qi)
                J.append(jj + b0)
                Dv.append(dd)
                H.append(torch.full_like(jj, h) * (1 << 40) + jj)
            continue
        for s in range(0, A.shape[0], tile):
            e = min(A.shape[0], s + tile)
            if nb == 0:
                break
            D = torch.round(pairwise(A[s:e], Bc) / nf * scale)
            keep = D <= thr if math.isfinite(thr) else torch.ones_like(D, dtype=torch.bool)
            if rB is None:   # upper triangle of the global index: j > i
                keep &= (torch.arange(b0, b0 + nb, device=dev).view(1, -1)
                         > torch.arange(a_base + s, a_base + e, device=dev).view(-1, 1))
            qi, jj = torch.nonzero(keep, as_tuple=True)
            if qi.numel():
                I.append(qi + s)
                J.append(jj + b0)
                Dv.append(D[qi, jj].long())
                H.append(torch.full_like(jj, h) * (1 << 40) + jj)
    sp_own = spB if rB is not None else spA
    if (I and not comm.is_distributed and dev.type == "cuda" and spA.dev is not None and sp_own.dev is not None
            and I[0].is_cuda):
        # one rank: both sides' lines are this rank's uploaded bytes, so the pairs stay on the
        # device and the output rows are formatted there (format.hip) instead of on the host
        I, J, Dv = torch.cat(I), torch.cat(J), torch.cat(Dv)
        if len(Dv) > 1:
            order = torch.argsort(I * max(1, NB) + J)
            I, J, Dv = I[order], J[order], Dv[order]
        spI, spJ = spA.select(I), sp_own.select(J - b_rec.line_base)
        cols = [spI.column("rf", idc, lit), spJ.column("rf", idc, lit)]
        if out_rec:
            cols += [spI.column("r", delims=lit), spJ.column("r", delims=lit)]
        cols.append(("i", Dv))
        ctx.emit_columns(cols, int(I.numel()))
        return
    if I:
        I, J, Dv, H = torch.cat(I), torch.cat(J), torch.cat(Dv), torch.cat(H)
        order = torch.argsort(I * max(1, NB) + J)
        I, Dv, H = I[order].cpu(), Dv[order].cpu(), H[order].cpu()
    else:
        I = Dv = H = torch.zeros(0, dtype=torch.long)
    # the B side of every pair: its hop's received line block, row jj
    hop, jl = H >> 40, H & ((1 << 40) - 1)
    hop_base = torch.tensor([0] + [len(b) for b in blocks], dtype=torch.long).cumsum(0)
    addr = torch.cat([b.spans()[1] for b in blocks]) if blocks else torch.zeros(0, dtype=torch.long)
    lens = torch.cat([b.spans()[2] for b in blocks]) if blocks else torch.zeros(0, dtype=torch.long)
    gi = hop_base[:-1][hop] + jl if hop.numel() else hop
    spJ = LineSpans(blocks, addr[gi], lens[gi])
    spI = spA.select(I)
    cols = [spI.column("rf", idc, lit), spJ.column("rf", idc, lit)]
    if out_rec:
        cols += [spI.column("r", delims=lit), spJ.column("r", delims=lit)]
    cols.append(("i", Dv))
    ctx.emit_columns(cols, int(I.numel()))


def _numeric_matrix(ctx, rows, ords):
    return torch.tensor([[float(r[o]) for o in ords] for r in rows], dtype=torch.float32, device=ctx.device)


def _record_similarity_rows(ctx, args):
    """Regex delimiters: the split-row path (every rank reads both sets, computes its block of
    base rows)."""
    from ..ops.distance import pairwise
    ords = ctx.get_int_list("attr.ordinals")
    idc = ctx.get_int("id.ordinal", 0)
    scale = ctx.get_float("distance.scale", 1000.0)
    thr = ctx.get_float("dist.threshold", math.inf)
    out_rec = ctx.get_bool("output.record", False)
    rows = ctx.rows(shard=False)
    other = ctx.rows(args.train, shard=False) if args.train else None
    allx = _numeric_matrix(ctx, rows + (other or []), ords)
    lo, hi = allx.min(0).values, allx.max(0).values
    rng = (hi - lo).clamp_min(1e-12)
    A = (_numeric_matrix(ctx, rows, ords) - lo) / rng
    B = (_numeric_matrix(ctx, other, ords) - lo) / rng if other else A
    Brows = other or rows
    from ..data.table import shard_range
    a, b = shard_range(len(rows), ctx.comm.rank, ctx.comm.world)
    d = ctx.delim_out
    out = []
    nf = math.sqrt(max(len(ords), 1))
    nB = len(Brows)
    for s in range(a, b, 2048):
        e = min(b, s + 2048)
        D = torch.round(pairwise(A[s:e], B) / nf * scale)
        keep = D <= thr if math.isfinite(thr) else torch.ones_like(D, dtype=torch.bool)
        if other is None:   # upper triangle: j > i
            keep &= torch.arange(nB, device=D.device).view(1, -1) > torch.arange(s, e, device=D.device).view(-1, 1)
        qi, jj = torch.nonzero(keep, as_tuple=True)          # row-major: (i, j) ascending
        vals = D[qi, jj].long().tolist()
        for q, j, v in zip(qi.tolist(), jj.tolist(), vals):
            i = s + q
            parts = [rows[i][idc], Brows[j][idc]]
            if out_rec:
                parts += rows[i] + Brows[j]
            out.append(d.join(parts + [str(v)]))
    ctx.emit(out)


@job("groupedRecordSimilarity", "pairwise distances within each group (S/similarity/GroupedRecordSimilarity.scala)")
def grouped_similarity(args):
    """Distances of every pair of records (i < j in input order) inside each group of
    ``group.field.ordinals``; output ``key..,id_i,id_j,dist`` by group in key order.  Native path:
    each rank reads its byte range; records move to the rank owning their group (one all-to-all,
    groups in string order cut into contiguous blocks); every rank runs the batched in-group
    distance launches of ``GroupedRecordSimilarity`` on its groups and writes them."""
    from ..data.table import _literal
    ctx = JobContext(args, app="groupedRecordSimilarity")
    lit = _literal(ctx.delim_in)
    if lit is None or len(lit) != 1:
        return _grouped_similarity_rows(ctx)
    from ..data.records import format_lines, owner_of, shuffle, sorted_key_tuples
    from ..data.table import shard_range
    from ..models.similarity import GroupedRecordSimilarity
    kords = ctx.get_int_list("group.field.ordinals", None) or ctx.get_int_list("key.field.ordinals")
    ords = ctx.get_int_list("attr.ordinals")
    idc = ctx.get_int("id.ordinal", 0)
    prec = ctx.get_int("output.precision", 3)
    comm = ctx.comm
    top = max(list(kords) + list(ords) + [idc]) + 1
    modes = "".join("d" if (i in kords or i == idc) else ("n" if i in ords else "x") for i in range(top))
    rec = ctx.records(modes=modes, tail_mode="x", numeric=True)
    kpos, G, ktab = sorted_key_tuples(rec, [rec.field(o) for o in kords], comm)
    owner = owner_of(kpos, G, comm.world) if comm.is_distributed else torch.zeros_like(kpos)
    cols = shuffle(comm, owner, [kpos, rec.field(idc).long()] + [rec.field(o, numeric=True) for o in ords])
    kp, ids = cols[0], cols[1]
    X = torch.stack(cols[2:], 1).float().to(ctx.device) if ords else torch.zeros((kp.numel(), 0), device=ctx.device)
    a, _ = shard_range(G, comm.rank, comm.world) if comm.is_distributed else (0, G)
    ii, jj, dd = GroupedRecordSimilarity().pairs(X, (kp - a).to(ctx.device))
    ii, jj = ii.cpu(), jj.cpu()
    kp_c, ids_c = kp.cpu(), ids.cpu().int()
    out = [("s", rec.vocab, ktab[kp_c[ii], j].int().contiguous()) for j in range(len(kords))]
    out += [("s", rec.vocab, ids_c[ii]), ("s", rec.vocab, ids_c[jj]), ("f", dd.double().cpu(), prec)]
    ctx.emit_columns(out, int(ii.numel()))


def _grouped_similarity_rows(ctx):
    """Regex delimiters: the split-row path (every rank reads the input, handles a block of groups)."""
    from ..ops.distance import pairwise  # noqa: F401
    kords = ctx.get_int_list("group.field.ordinals", None) or ctx.get_int_list("key.field.ordinals")
    ords = ctx.get_int_list("attr.ordinals")
    idc = ctx.get_int("id.ordinal", 0)
    prec = ctx.get_int("output.precision", 3)
    g = defaultdict(list)
    for r in ctx.rows(shard=False):
        g[tuple(r[o] for o in kords)].append(r)
    keys = sorted(g)
    from ..data.table import shard_range
    a, b = shard_range(len(keys), ctx.comm.rank, ctx.comm.world)
    d = ctx.delim_out
    out = []
    from ..models.similarity import GroupedRecordSimilarity
    mine = [(gi, r) for gi, k in enumerate(keys[a:b]) for r in g[k]]
    if mine:
        X = _numeric_matrix(ctx, [r for _, r in mine], ords)
        gid = torch.tensor([gi for gi, _ in mine], dtype=torch.long, device=X.device)
        ii, jj, dd = GroupedRecordSimilarity().pairs(X, gid)
        for i, j, v in zip(ii.tolist(), jj.tolist(), dd.tolist()):
            gi, ri = mine[i]
            out.append(d.join(list(keys[a + gi]) + [ri[idc], mine[j][1][idc], fmt(v, prec)]))
    ctx.emit(out)


@job("nearestRecords", "per record the top-k nearest from pair distances, by count or distance (S/similarity/NearestRecords.scala)")
def nearest_records(args):
    """Pair rows ``id1,id2,...,dist`` (both directions considered); per first record the nearest
    ``neighbor.count`` (or all within ``neighbor.dist.threshold``), output ``id,n1,n2,...`` in id
    order, neighbours by distance then id.  Native path: each rank reads its byte range, both
    directions of every pair go to the rank owning the record (all-to-all), one device sort by
    (record, distance, neighbour) per rank."""
    from ..data.table import _literal
    ctx = JobContext(args, app="nearestRecords")
    lit = _literal(ctx.delim_in)
    k = ctx.get_int("neighbor.count", 5)
    thr = ctx.get_float("neighbor.dist.threshold", math.inf)
    if lit is None or len(lit) != 1:
        return _nearest_records_rows(ctx, k, thr)
    from ..data.records import format_lines, owner_of, segment_rank, shuffle, sorted_keys
    from ..data.table import shard_range
    comm = ctx.comm
    rec = ctx.records(modes="dd", tail_mode="x", numeric=True, last_mode="n")
    ok = rec.lens() >= 3
    a_, b_, dist = rec.field(0)[ok].long(), rec.field(1)[ok].long(), rec.field(-1, numeric=True)[ok]
    x = torch.cat([a_, b_])
    y = torch.cat([b_, a_])
    dd = torch.cat([dist, dist])
    keys, pos = sorted_keys(rec, x, comm)
    G = keys.numel()
    xp, yp = pos[x], pos[y]
    owner = owner_of(xp, G, comm.world) if comm.is_distributed else torch.zeros_like(xp)
    xp, yp, dd = shuffle(comm, owner, [xp, yp, dd])
    o = torch.argsort(yp, stable=True)
    o = o[torch.argsort(dd[o], stable=True)]
    o = o[torch.argsort(xp[o], stable=True)]
    xp, yp, dd = xp[o], yp[o], dd[o]
    first = torch.ones_like(xp, dtype=torch.bool)
    first[1:] = xp[1:] != xp[:-1]
    keep = (segment_rank(first) < k) & (dd <= thr)
    a, b = shard_range(G, comm.rank, comm.world) if comm.is_distributed else (0, G)
    cnt = torch.bincount((xp - a)[keep], minlength=b - a) if b > a else torch.zeros(0, dtype=torch.long)
    off = torch.cat([torch.zeros(1, dtype=torch.long, device=cnt.device), torch.cumsum(cnt, 0)]).cpu()
    kc = keys.cpu()
    cols = [("s", rec.vocab, kc[a:b].int().contiguous()), ("l", rec.vocab, kc[yp[keep].cpu()].int(), off)]
    ctx.emit_columns(cols, b - a)


def _nearest_records_rows(ctx, k, thr):
    nb = defaultdict(list)
    for r in ctx.rows(shard=False):
        dd = float(r[-1])
        nb[r[0]].append((dd, r[1]))
        nb[r[1]].append((dd, r[0]))
    keys = sorted(nb)
    from ..data.table import shard_range
    a, b = shard_range(len(keys), ctx.comm.rank, ctx.comm.world)
    d = ctx.delim_out
    ctx.emit([d.join([x] + [y for dd, y in sorted(nb[x])[:k] if dd <= thr]) for x in keys[a:b]])


# ================================================================================================
# population optimisers (Spark)
# ================================================================================================
def _domain(ctx):
    from ..optimize import TaskScheduleSearch
    return TaskScheduleSearch.from_json(ctx.path("domain.callback.config.file", "domain"), ctx.device)


@job("geneticAlgorithm", "island-model GA over a task-schedule domain (S/optimize/GeneticAlgorithm.scala)")
def genetic(args):
    from ..optimize.search import GeneticAlgorithm
    ctx = JobContext(args, app="geneticAlgorithm")
    d = _domain(ctx)
    pop = ctx.get_int("population.size", 16)
    ga = GeneticAlgorithm(d, islands=ctx.get_int("num.optimizers", 4), pool=pop, mating=max(2, pop // 2),
                          replacement=max(1, pop // 2), generations=ctx.get_int("num.generations", 100),
                          seed=ctx.get_int("random.seed", 0), comm=ctx.comm)
    r = ga.run()
    o = ctx.delim_out
    lines = [f"{d.format_solution(s)}{o}{c:.6f}" for s, c in zip(r.solutions.tolist(), r.costs.tolist())]
    ctx.emit_root(sorted(lines, key=lambda l: float(l.rsplit(o, 1)[1])))
    ctx.report({"best_cost": r.best_cost})


@job("randomSearch", "random multi-start search + local search around the best (S/optimize/RandomSearch.scala)")
def random_search(args):
    from ..optimize.search import RandomSearch
    ctx = JobContext(args, app="randomSearch")
    d = _domain(ctx)
    rs = RandomSearch(d, n=ctx.get_int("max.num.iterations", 100) * ctx.get_int("num.optimizers", 4),
                      local="focussed" if ctx.get_bool("locally.optimize", False) else None,
                      seed=ctx.get_int("random.seed", 0), comm=ctx.comm)
    r = rs.run()
    o = ctx.delim_out
    lines = [f"{d.format_solution(s)}{o}{c:.6f}" for s, c in zip(r.solutions.tolist(), r.costs.tolist())]
    ctx.emit_root(lines)
    ctx.report({"best_cost": r.best_cost})
