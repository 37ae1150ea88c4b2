"""Exploration, encoding, sampling and feature-relevance jobs (J/explore/*, S/explore/*, S/util/*).

Counting jobs build a dense per-rank tensor (contingency tables, class counts, moments) with the
device histogram kernels, all-reduce it once over RCCL and write from rank 0 (the reference's
combiner + single reducer); record-wise jobs (samplers, encoders, mappers) transform their input
shard and write one part file per rank (the reference's map-only jobs).
"""
from __future__ import annotations

import math
from collections import Counter, defaultdict

import torch

from .common import JobContext, fmt, job


def _schema_or_none(ctx: JobContext, key: str):
    try:
        return ctx.schema(key)
    except SystemExit:
        return None


def _pairs(spec: str) -> list[tuple[int, int]]:
    """``a:b,c:d`` (chombo ``assertIntPairListConfigParam``)."""
    return [tuple(int(x) for x in p.split(":")) for p in spec.split(",") if p.strip()]


# ================================================================================================
# categorical / numerical correlation
# ================================================================================================
def _contingency_job(ctx: JobContext, src_key: str, dst_key: str, stat_fn) -> None:
    """Shared driver of CramerCorrelation / HeterogeneityReductionCorrelation
    (J/explore/CategoricalCorrelation.java:52-209): one multi-pair 2-D histogram launch (K3) per
    rank, ONE all-reduce of every contingency table, ``srcName,dstName,stat`` lines."""
    from ..models.explore import ContingencyStats
    from ..ops import histogram as H
    schema = ctx.schema("feature.schema.file.path")
    src = ctx.get_int_list(src_key)
    dst = ctx.get_int_list(dst_key)
    pairs = [(s, d) for s in src for d in dst if s != d]
    ords = sorted({o for p in pairs for o in p})
    t = ctx.table(schema=_with_features(schema, ords))
    pos = {f.ordinal: j for j, f in enumerate(t.binned_fields)}
    tabs = H.pair_histogram(t.codes, t.n, t.bins, [(pos[a], pos[b]) for a, b in pairs], None, 1)
    tabs = [tb[0].clone() for tb in tabs]
    ctx.all_reduce(*tabs)
    d = ctx.delim_out
    lines = []
    for (a, b), tb in zip(pairs, tabs):
        fa, fb = schema.find_field_by_ordinal(a), schema.find_field_by_ordinal(b)
        lines.append(f"{fa.name}{d}{fb.name}{d}{stat_fn(ContingencyStats(tb))}")
    ctx.emit_root(lines)


def _with_features(schema, ords):
    """A copy of the schema whose feature set is exactly ``ords`` (class attribute dropped)."""
    import copy
    s = copy.deepcopy(schema)
    for f in s.fields:
        f.feature = f.ordinal in set(ords)
        if f.ordinal in set(ords):
            f.class_attr = False
    return s


@job("cramerCorrelation", "Cramer index per categorical attribute pair (J/explore/CramerCorrelation.java, crc.*)")
def cramer(args):
    ctx = JobContext(args, "crc.")
    _contingency_job(ctx, "source.attributes", "dest.attributes", lambda c: c.cramer_index())


@job("heterogeneityReductionCorrelation",
     "concentration (gini) / uncertainty coefficient per attribute pair (J/explore/HeterogeneityReductionCorrelation.java)")
def hetero(args):
    ctx = JobContext(args, "cac.")
    alg = ctx.cfg.values.get("hrc.heterogeneity.algorithm", "gini")
    _contingency_job(ctx, "first.set.attributes", "second.set..attributes" if ctx.has("second.set..attributes")
                     else "second.set.attributes",
                     (lambda c: c.concentration_coeff()) if alg == "gini" else (lambda c: c.uncertainty_coeff()))


@job("numericalCorrelation", "Pearson correlation of attribute pairs (J/explore/NumericalCorrelation.java, nuc.*)")
def numcorr(args):
    """``nuc.attr.pairs=a:b,...``; means/std-devs come from ``nuc.stats.file.path`` (chombo
    NumericalAttrStats lines ``attr,...,mean,...,stdDev``) when given, else from the same pass (one
    fused moments reduction: counts, sums and the cross-product GEMM, one all-reduce)."""
    ctx = JobContext(args, "nuc.")
    pairs = _pairs(ctx.get_str("attr.pairs"))
    ords = sorted({o for p in pairs for o in p})
    X, _ = ctx.numeric_matrix(ords)
    n = torch.tensor([float(X.shape[0])], dtype=torch.float64, device=ctx.device)
    s = X.sum(0)
    # a few columns over millions of rows: one reduction pass per column instead of an fp64 GEMM
    # with a 2 x 2 output (the library's pick for that shape took ~0.2 s at 2^21 rows)
    G = (torch.stack([(X * X[:, i:i + 1]).sum(0) for i in range(X.shape[1])]) if X.shape[1] <= 16
         else X.T @ X)
    ctx.all_reduce(n, s, G)
    mean = s / n
    cov = G / n - mean.view(-1, 1) * mean.view(1, -1)
    sd = cov.diag().clamp_min(1e-300).sqrt()
    if ctx.has("stats.file.path"):
        st = {}
        for l in ctx.all_lines(ctx.path("stats.file.path")):
            p = ctx.split(l)
            st[int(p[0])] = float(p[-1])
        sd = torch.tensor([st.get(o, float(sd[i])) for i, o in enumerate(ords)], dtype=torch.float64, device=ctx.device)
    ix = {o: i for i, o in enumerate(ords)}
    d = ctx.delim_out
    ctx.emit_root([f"{a}{d}{b}{d}{float(cov[ix[a], ix[b]] / (sd[ix[a]] * sd[ix[b]]))}" for a, b in pairs])


# ================================================================================================
# rules
# ================================================================================================
@job("ruleEvaluator", "confidence and support of named rules rue.rule.<name>=<cond> > <class> (J/explore/RuleEvaluator.java)")
def rule_evaluator(args):
    """Each rule's antecedent is evaluated column-wise over the shard (``utils/rules.py``), the
    per-rule class counts are one ``[R, C]`` tensor, all-reduced once; output
    ``name,confidence,support`` with ``rue.conf.strategy`` confAccuracy | confEntropy
    (:231-268; support divides by ``rue.data.size`` when given, else by the global record count)."""
    from ..utils.rules import ColumnCache, RecordColumns, rule_field_modes, rules_from_config
    from .common import field_modes
    ctx = JobContext(args, "rue.")
    rules = rules_from_config(ctx.cfg)
    cls_ord = ctx.get_int("class.attr.ord")
    classes = ctx.get_list("class.values", None)
    fm = rule_field_modes(rules.values(), {cls_ord: "d"})
    rec = ctx.try_records(modes=field_modes(fm), tail_mode="x", numeric=True, trim=True)
    if rec is not None:           # native: predicate fields tokenized once, rules evaluated on the device
        cols = RecordColumns(rec, [o for o, m in fm.items() if m == "n"])
        cc = rec.field(cls_ord)
        if not classes:
            classes = ctx.union(rec.strings(torch.unique(cc[cc >= 0])))
        lab = rec.map_codes(cc, classes).long()
        n_rows = rec.n_lines
    else:
        rows = ctx.rows(keep_empty=True)
        cols = ColumnCache(rows, ctx.device)
        if not classes:
            classes = ctx.union(r[cls_ord] for r in rows)
        ci = {c: i for i, c in enumerate(classes)}
        lab = torch.tensor([ci.get(r[cls_ord], -1) for r in rows], dtype=torch.long, device=ctx.device)
        n_rows = len(rows)
    ci = {c: i for i, c in enumerate(classes)}
    C, R = len(classes), len(rules)
    counts = torch.zeros((R, C), dtype=torch.float64, device=ctx.device)
    for k, (name, rexp) in enumerate(rules.items()):
        m = rexp.evaluate(cols) & (lab >= 0)
        counts[k] = torch.bincount(lab[m], minlength=C)[:C].double()
    n = torch.tensor([float(n_rows)], dtype=torch.float64, device=ctx.device)
    ctx.all_reduce(counts, n)
    size = ctx.get_int("data.size", None) or int(n)
    strat = ctx.get_str("conf.strategy", "confAccuracy")
    d = ctx.delim_out
    lines = []
    for k, (name, rexp) in enumerate(rules.items()):
        tot = float(counts[k].sum())
        cons = ci.get(rexp.consequent, 0)
        if strat == "confEntropy":
            p1 = float(counts[k, cons]) / max(tot, 1)
            p2 = float(counts[k, cons ^ 1]) / max(tot, 1) if C > 1 else 0.0
            ent = sum(p * math.log(p) for p in (p1, p2) if p > 0)
            conf = ent / math.log(2) + 1.0
        else:
            conf = float(counts[k, cons]) / max(tot, 1)
        lines.append(f"{name}{d}{fmt(conf)}{d}{fmt(tot / max(size, 1))}")
    ctx.emit_root(lines)


# ================================================================================================
# feature relevance / neighbourhoods
# ================================================================================================
@job("reliefFeatureRelevance", "Relief feature relevance (J/explore/ReliefFeatureRelevance.java, ffr.* / S FeatureRelevanceByRelief)",
     aliases=("featureRelevanceByRelief",))
def relief_job(args):
    """Two input forms:

    * ``ffr.neighborhood.file.path`` given (MR form): records keyed by ``ffr.id.ord`` plus a
      neighbourhood file of ``srcId,srcClass,trgClass,trgId,...`` lines (ClassBasedNeighborhood);
      every (src, trg) pair adds -|diff| on a hit and +|diff| on a miss, normalised by the
      attribute range, divided by the pair count;
    * otherwise: the neighbourhoods are computed here with the fused kNN kernel (nearest hit and
      miss per record, ``ffr.neighbor.count``), over the schema's feature attributes.

    Output ``attrOrd,score`` (3 decimals)."""
    from ..models.sampling import relief
    ctx = JobContext(args, "ffr.")
    attrs = ctx.get_int_list("attr.ordinals", None)
    schema = _schema_or_none(ctx, "attr.schema.file.path")
    d = ctx.delim_out
    if ctx.has("neighborhood.file.path") and ctx.native_delim() is not None:
        _relief_pairs_native(ctx, attrs, schema)
        return
    if ctx.has("neighborhood.file.path"):
        id_ord = ctx.get_int("id.ord")
        recs = {r[id_ord]: r for r in ctx.rows(shard=False)}
        pairs = []
        for l in ctx.all_lines(ctx.path("neighborhood.file.path")):
            p = ctx.split(l)
            for trg in p[3:]:
                if p[0] in recs and trg in recs:
                    pairs.append((p[0], trg, p[1] == p[2]))
        if ctx.comm.is_distributed:
            from ..data.table import shard_range
            a, b = shard_range(len(pairs), ctx.comm.rank, ctx.comm.world)
            pairs = pairs[a:b]
        score = torch.zeros(len(attrs), dtype=torch.float64)
        for j, o in enumerate(attrs):
            f = schema.find_field_by_ordinal(o) if schema else None
            if f is not None and f.is_categorical:
                diff = torch.tensor([float(recs[s][o] != recs[t][o]) for s, t, _ in pairs], dtype=torch.float64)
            else:
                rng = (f.max - f.min) if f is not None and f.max is not None and f.min is not None else 1.0
                diff = torch.tensor([abs(float(recs[s][o]) - float(recs[t][o])) / rng for s, t, _ in pairs],
                                    dtype=torch.float64)
            sign = torch.tensor([-1.0 if hit else 1.0 for _, _, hit in pairs], dtype=torch.float64)
            score[j] = (diff * sign).sum() if pairs else 0.0
        npairs = torch.tensor([float(len(pairs))], dtype=torch.float64)
        ctx.all_reduce(score, npairs)
        ctx.emit_root([f"{o}{d}{fmt(float(score[j]) / max(float(npairs), 1))}" for j, o in enumerate(attrs)])
        return
    t = ctx.table(raw_numeric=True, schema=schema)
    X = t.dense_features()
    ords = [f.ordinal for f in t.binned_fields] + [f.ordinal for f in t.numeric_fields]
    s = relief(X, t.labels[: t.n].long(), ctx.get_int("neighbor.count", 1))
    keep = attrs or ords
    ctx.emit_root([f"{o}{d}{fmt(float(s[ords.index(o)]))}" for o in keep if o in ords])


def _relief_pairs_native(ctx, attrs, schema):
    """reliefFeatureRelevance (MR form) on token tables: the records (every rank reads them whole:
    the join side) with the id as a dictionary code and the attributes as numbers / codes, the
    neighbourhood file as this rank's byte range of dictionary tokens; pairs join the records by
    code (one dictionary-level map between the two files), every attribute's signed differences are
    one masked reduction, one all-reduce."""
    from .common import field_modes
    id_ord = ctx.get_int("id.ord")
    cat = {o for o in attrs if schema is not None and schema.find_field_by_ordinal(o) is not None
           and schema.find_field_by_ordinal(o).is_categorical}
    recs = ctx.records(shard=False, modes=field_modes({id_ord: "d", **{o: ("d" if o in cat else "n") for o in attrs}}),
                       tail_mode="x", numeric=True)
    V = len(recs.vocab)
    idc = recs.field(id_ord).long()
    row_of = torch.full((max(V, 1),), -1, dtype=torch.long, device=recs.device)
    if recs.n_lines:
        row_of.scatter_reduce_(0, idc.clamp_min(0), torch.arange(recs.n_lines, device=recs.device), "amax")
    nb = ctx.records(ctx.path("neighborhood.file.path"), tail_mode="d")
    vi = {v: i for i, v in enumerate(recs.vocab)}
    lut = torch.tensor([vi.get(v, -1) for v in nb.vocab] or [-1], dtype=torch.long, device=nb.device)
    pad, cnt = nb.padded(dtype=torch.long)
    dev = recs.device
    score = torch.zeros(len(attrs), dtype=torch.float64, device=dev)
    npairs = torch.zeros(1, dtype=torch.float64, device=dev)
    if pad.shape[0] and pad.shape[1] > 3:
        src, hit = pad[:, 0], pad[:, 1] == pad[:, 2]
        trg = pad[:, 3:]
        tv = torch.arange(trg.shape[1], device=pad.device).view(1, -1) < (cnt.view(-1, 1) - 3)
        def to_row(c):
            k = torch.where(c >= 0, lut[c.clamp_min(0)], torch.full_like(c, -1))
            return torch.where(k >= 0, row_of[k.clamp_min(0)], torch.full_like(k, -1))
        rs = to_row(src).view(-1, 1).expand_as(trg)
        rt = to_row(trg)
        ok = tv & (rs >= 0) & (rt >= 0)
        rs, rt = rs[ok].to(dev), rt[ok].to(dev)
        sign = torch.where(hit.view(-1, 1).expand_as(trg)[ok], -1.0, 1.0).double().to(dev)
        npairs[0] = float(rs.numel())
        for j, o in enumerate(attrs):
            f = schema.find_field_by_ordinal(o) if schema else None
            if o in cat:
                c = recs.field(o)
                diff = (c[rs] != c[rt]).double()
            else:
                rng = (f.max - f.min) if f is not None and f.max is not None and f.min is not None else 1.0
                x = recs.field(o, numeric=True).double()
                diff = (x[rs] - x[rt]).abs() / rng
            score[j] = (diff * sign).sum()
    ctx.all_reduce(score, npairs)
    d = ctx.delim_out
    ctx.emit_root([f"{o}{d}{fmt(float(score[j]) / max(float(npairs), 1))}" for j, o in enumerate(attrs)])


@job("topMatchesByClass", "same-class nearest neighbours from pair distances (J/explore/TopMatchesByClass.java, tmc.*)")
def top_matches(args):
    """Input: ``srcId,trgId,srcRec...,trgRec...,rank`` (recordSimilarity with record output), or
    ``srcId,trgId,rank`` when ``tmc.include.rec.in.output=false``.  Both directions of every
    same-class pair are ranked per source (a device segmented sort on (src, rank)); the top
    ``tmc.top.match.count`` (or all within ``tmc.top.match.distance``) are written per source, one
    line per neighbour or one compact line (``tmc.compact.output``).  The reference's reducer stops
    one short of ``top.match.count`` (``++count >= topMatchCount``); here exactly that many are
    kept."""
    ctx = JobContext(args, "tmc.")
    cls_ord = ctx.get_int("class.attr.ord")
    filt = ctx.get_str("filer.class.value", None)
    inc_rec = ctx.get_bool("include.rec.in.output", True)
    by_count = ctx.get_bool("nearest.by.count", True)
    by_dist = ctx.get_bool("nearest.by.distance", False)
    topn = ctx.get_int("top.match.count", 10) if by_count else None
    maxd = ctx.get_int("top.match.distance", 200) if (by_dist or not by_count) else None
    compact = ctx.get_bool("compact.output", False)
    inc_cls = ctx.get_bool("include.class.in.output", True)
    from ..data.table import _literal
    lit = _literal(ctx.delim_in)
    if lit is not None and len(lit) == 1:
        rec = ctx.records(last_mode="n", numeric=True)     # the trailing rank parsed as a number
        W = rec.width()
        if ctx.comm.is_distributed:
            W = ctx.comm.all_gather_object(W)
            W = W[0] if all(w == W[0] or w == 0 for w in W) else None
            W = W if W != 0 else None
        if W is not None and W >= 5 and (W - 3) % 2 == 0:
            return _top_matches_native(ctx, rec, W, cls_ord, filt, inc_rec, topn, maxd, compact, inc_cls)
    rows = ctx.rows(shard=False)
    src, trg, rank, cls = [], [], [], []
    recs = {}
    for r in rows:
        L = (len(r) - 3) // 2
        s_id, t_id = r[0], r[1]
        s_rec, t_rec = r[2:2 + L], r[2 + L:2 + 2 * L]
        sc, tc = s_rec[cls_ord], t_rec[cls_ord]
        if sc != tc or (filt is not None and sc != filt):
            continue
        recs[s_id], recs[t_id] = s_rec, t_rec
        rk = int(float(r[-1]))
        src += [s_id, t_id]
        trg += [t_id, s_id]
        rank += [rk, rk]
        cls += [sc, sc]
    ids = sorted(recs)
    ii = {v: i for i, v in enumerate(ids)}
    if not src:
        ctx.emit_root([])
        return
    S = torch.tensor([ii[x] for x in src])
    Tt = torch.tensor([ii[x] for x in trg])
    Rk = torch.tensor(rank)
    order = torch.argsort(Rk, stable=True)
    order = order[torch.argsort(S[order], stable=True)]
    S, Tt, Rk = S[order], Tt[order], Rk[order]
    first = torch.ones_like(S, dtype=torch.bool)
    first[1:] = S[1:] != S[:-1]
    from ..data.records import segment_rank
    pos = segment_rank(first)
    keep = torch.ones_like(S, dtype=torch.bool)
    if topn is not None:
        keep &= pos < topn
    if maxd is not None:
        keep &= Rk <= maxd
    d = ctx.delim_out
    out = defaultdict(list)
    for s, t in zip(S[keep].tolist(), Tt[keep].tolist()):
        out[s].append(d.join(recs[ids[t]]) if inc_rec else ids[t])
    lines = []
    clsmap = dict(zip(src, cls))
    for s in sorted(out):
        head = d.join(recs[ids[s]]) if inc_rec else ids[s]
        if inc_cls:
            head += d + clsmap[ids[s]]
        if compact:
            lines.append(d.join([head] + out[s]))
        else:
            lines += [f"{head}{d}{x}" for x in out[s]]
    ctx.emit_root(lines)


def _top_matches_native(ctx, rec, W, cls_ord, filt, inc_rec, topn, maxd, compact, inc_cls):
    """topMatchesByClass on the native record table: same-class pairs both ways, shuffled to the
    rank owning the source entity (entities in string order, contiguous blocks per rank: the
    reference's reducer key order), a device segmented sort on (source, rank) with the global
    input order as tie-break, and the output assembled by the native formatter."""
    from ..data.records import format_lines, owner_of, shuffle, sorted_keys
    comm = ctx.comm
    dev = rec.device
    Lr = (W - 3) // 2
    M = rec.codes.view(rec.n_lines, W).long()
    sc, tc = M[:, 2 + cls_ord], M[:, 2 + Lr + cls_ord]
    ok = sc == tc
    if filt is not None:
        fc = rec.vocab.index(filt) if filt in rec.vocab else -2
        ok &= sc == fc
    rk = torch.nan_to_num(torch.trunc(rec.field(-1, numeric=True)), nan=float(2 ** 62)).long()
    Mo = M[ok]
    rko = rk[ok]
    seq = (torch.nonzero(ok).view(-1) + rec.line_base) * 2
    # both directions: (s -> t) then (t -> s), interleaved in input order via the sequence number
    src = torch.cat([Mo[:, 0], Mo[:, 1]])
    trg = torch.cat([Mo[:, 1], Mo[:, 0]])
    srec = torch.cat([Mo[:, 2:2 + Lr], Mo[:, 2 + Lr:2 + 2 * Lr]])
    trec = torch.cat([Mo[:, 2 + Lr:2 + 2 * Lr], Mo[:, 2:2 + Lr]])
    sq = torch.cat([seq, seq + 1])
    rr = torch.cat([rko, rko])
    keys, pos = sorted_keys(rec, src, comm)
    E = keys.numel()
    if E == 0:
        ctx.emit_root([])
        return
    spos = pos[src]
    owner = owner_of(spos, E, comm.world) if comm.is_distributed else torch.zeros_like(spos)
    cols = [spos, trg, rr, sq] + [srec[:, j] for j in range(Lr)] + [trec[:, j] for j in range(Lr)]
    cols = shuffle(comm, owner, cols)
    spos, trg, rr, sq = cols[:4]
    srec = torch.stack(cols[4:4 + Lr], 1) if Lr else None
    trec = torch.stack(cols[4 + Lr:], 1) if Lr else None
    # (source, rank, input order) sort: ONE argsort of a packed int64 key when the three ranges fit
    # 62 bits (the usual case: ~20 + ~10 + ~25 bits), else three stable passes
    o = None
    if sq.numel():
        r_lo, r_hi = int(rr.min()), int(rr.max())
        q_hi = int(sq.max())
        bq, br = max(1, q_hi.bit_length()), max(1, (r_hi - r_lo).bit_length())
        if max(1, E.bit_length()) + br + bq <= 62 and r_lo >= -(1 << 61):
            o = torch.argsort((spos << (br + bq)) | ((rr - r_lo) << bq) | sq)
    if o is None:
        o = torch.argsort(sq, stable=True)
        o = o[torch.argsort(rr[o], stable=True)]
        o = o[torch.argsort(spos[o], stable=True)]
    spos, trg, rr = spos[o], trg[o], rr[o]
    srec, trec = srec[o], trec[o]
    n = spos.numel()
    first = torch.ones(n, dtype=torch.bool, device=dev)
    if n > 1:
        first[1:] = spos[1:] != spos[:-1]
    from ..data.records import segment_rank
    rank_in = segment_rank(first)
    keep = torch.ones(n, dtype=torch.bool, device=dev)
    if topn is not None:
        keep &= rank_in < topn
    if maxd is not None:
        keep &= rr <= maxd
    head_cols = (srec if inc_rec else keys[spos].view(-1, 1))
    tail_cols = (trec if inc_rec else trg.view(-1, 1))
    voc = rec.vocab
    d = ctx.delim_out
    if compact:
        heads = torch.nonzero(first).view(-1)
        kept = keep.long()
        cnt = torch.zeros(heads.numel(), dtype=torch.long, device=dev).index_add_(
            0, torch.cumsum(first.long(), 0)[keep] - 1, kept[keep])
        has = cnt > 0
        heads, cnt = heads[has], cnt[has]
        tails = tail_cols[keep]
        off = torch.zeros(cnt.numel() + 1, dtype=torch.long, device=dev)
        off[1:] = torch.cumsum(cnt * tails.shape[1], 0)
        hc = head_cols[heads]
        cols_f = [("s", voc, hc[:, j].int().cpu()) for j in range(hc.shape[1])]
        if inc_cls:
            cols_f.append(("s", voc, srec[heads][:, cls_ord].int().cpu()))
        cols_f.append(("l", voc, tails.reshape(-1).int().cpu(), off.cpu()))
        n_out = heads.numel()
    else:
        hc, tcs = head_cols[keep], tail_cols[keep]
        cols_f = [("s", voc, hc[:, j].int().cpu()) for j in range(hc.shape[1])]
        if inc_cls:
            cols_f.append(("s", voc, srec[keep][:, cls_ord].int().cpu()))
        cols_f += [("s", voc, tcs[:, j].int().cpu()) for j in range(tcs.shape[1])]
        n_out = hc.shape[0]
    # every rank's part is already in global source order: rank-ordered concatenation
    ctx.emit_columns(cols_f, n_out)


# ================================================================================================
# samplers
# ================================================================================================
@job("underSamplingBalancer", "class-balancing under-sampling (J/explore/UnderSamplingBalancer.java, usb.*)")
def undersampling(args):
    """Keeps a record of a class with global count n_c with probability min_c / n_c (the class
    counts are all-reduced first, instead of the reference's per-mapper warm-up batch estimate);
    the draw of record g is the K25 Philox stream at the GLOBAL record index, so the kept set does
    not depend on the world size (models/sampling.undersample)."""
    from ..models.sampling import undersample
    from .common import field_modes
    ctx = JobContext(args, "usb.")
    cls_ord = ctx.get_int("class.attr.ord")
    rec = ctx.try_records(modes=field_modes({cls_ord: "d"}), tail_mode="x")
    if rec is not None:
        cc = rec.field(cls_ord)
        vals = ctx.union(rec.strings(torch.unique(cc[cc >= 0])))
        y = rec.map_codes(cc, vals).long()           # on the table's device: the Philox draws run there
        keep = undersample(y, seed=ctx.get_int("random.seed", 0), comm=ctx.comm).bool()
        spans = rec.line_spans().select(keep)
        ctx.emit_columns([spans.column("r")], len(spans))
        return
    lines = ctx.lines()
    sp = ctx.split
    vals = ctx.union(sp(l)[cls_ord] for l in lines)
    vi = {v: i for i, v in enumerate(vals)}
    y = torch.tensor([vi[sp(l)[cls_ord]] for l in lines], dtype=torch.long)
    keep = undersample(y, seed=ctx.get_int("random.seed", 0), comm=ctx.comm)
    ctx.emit([l for l, k in zip(lines, keep.tolist()) if k])


@job("baggingSampler", "bootstrap resampling within batches (J/explore/BaggingSampler.java, bas.batch.size)")
def bagging(args):
    """Output slot g (global record order) copies record b0 + floor(u(seed, g) * batch) of its batch
    (models/sampling.bagging_indices, K25 Philox at the global index): the same records whatever
    the world size; picks that another rank holds (batches crossing a shard boundary) are fetched
    with one object all-gather of the requests and one of the answers."""
    from ..models.sampling import bagging_indices
    ctx = JobContext(args, "bas.")
    comm = ctx.comm
    rec = ctx.try_records(tail_mode="x")
    if rec is not None:
        _bagging_native(ctx, rec, bagging_indices)
        return
    lines = ctx.lines()
    sizes = comm.all_gather_object(len(lines)) if comm.is_distributed else [len(lines)]
    base, total = sum(sizes[: comm.rank]), sum(sizes)
    idx = bagging_indices(len(lines), ctx.get_int("batch.size", 10000), seed=ctx.get_int("random.seed", 0),
                          base=base, total=total).tolist()
    remote = sorted({i for i in idx if not base <= i < base + len(lines)})
    got = {}
    if comm.is_distributed:
        reqs = comm.all_gather_object(remote)
        mine = {i: lines[i - base] for r in reqs for i in r if base <= i < base + len(lines)}
        for part in comm.all_gather_object(mine):
            got.update(part)
    ctx.emit([lines[i - base] if base <= i < base + len(lines) else got[i] for i in idx])


def _bagging_native(ctx, rec, bagging_indices):
    """baggingSampler on byte spans: picks this rank holds are span selections; picks of records
    other ranks hold travel as one packed byte payload (all-gathered requests, each owner packs
    the requested lines natively, one all-gather of the payloads)."""
    from ..data.lines import LineSpans
    comm = ctx.comm
    spans = rec.line_spans()
    n = len(spans)
    sizes = comm.all_gather_object(n) if comm.is_distributed else [n]
    base, total = sum(sizes[: comm.rank]), sum(sizes)
    fast = not comm.is_distributed and spans.dev is not None
    idx = bagging_indices(n, ctx.get_int("batch.size", 10000), seed=ctx.get_int("random.seed", 0), base=base,
                          total=total, device=spans.dev[1].device if fast else "cpu").long()
    if fast:
        # one process with the device tokenizer: every pick is a local line — a device selection of
        # the uploaded line bytes, formatted by format.hip (no host line index, no host copy)
        sel = spans.select(idx - base)
        ctx.emit_columns([sel.column("r", delims=ctx.native_delim())], len(sel))
        return
    local = (idx >= base) & (idx < base + n)
    _, addr, ln = spans.spans()
    out_a = torch.zeros(idx.numel(), dtype=torch.int64)
    out_l = torch.zeros(idx.numel(), dtype=torch.int64)
    li = (idx - base).clamp(0, max(n - 1, 0))
    if n:
        out_a[local], out_l[local] = addr[li[local]], ln[li[local]]
    owners = [spans]
    if comm.is_distributed:
        req = torch.unique(comm.all_gather_v(torch.unique(idx[~local])))
        mine = req[(req >= base) & (req < base + n)]
        buf, off = spans.select(mine - base).pack()
        g_idx = comm.all_gather_v(mine)
        g_len = comm.all_gather_v(off[1:] - off[:-1])
        g_buf = comm.all_gather_v(buf)
        got = LineSpans.from_packed(g_buf, torch.cat([torch.zeros(1, dtype=torch.long), torch.cumsum(g_len, 0)]))
        owners.append(got)
        rem = ~local
        if bool(rem.any()):
            j = torch.searchsorted(g_idx, idx[rem])
            _, ga, gl = got.spans()
            out_a[rem], out_l[rem] = ga[j], gl[j]
    res = LineSpans(owners, out_a, out_l)
    ctx.emit_columns([res.column("r", delims=ctx.native_delim())], len(res))


@job("adaBoostError", "weighted misclassification error (J/explore/AdaBoostError.java, abe.*)")
def adaboost_error(args):
    ctx = JobContext(args, "abe.")
    po, ao, bo = (ctx.get_int("pred.class.attr.ord"), ctx.get_int("actual.class.attr.ord"),
                  ctx.get_int("boost.attr.ord"))
    w, wrong, n_rows, _ = _boost_columns(ctx, po, ao, bo)
    acc = torch.stack([(wrong.double() * w).sum(), torch.tensor(float(n_rows), dtype=torch.float64, device=w.device)])
    ctx.all_reduce(acc)
    err = float(acc[0]) if ctx.get_bool("weight.normalized", False) else float(acc[0]) / max(float(acc[1]), 1)
    ctx.emit_root([f"error={fmt(err, ctx.get_int('output.precision', 6))}"])


@job("adaBoostUpdate", "boost weight update from the error file (J/explore/AdaBoostUpdate.java, abu.*)")
def adaboost_update(args):
    ctx = JobContext(args, "abu.")
    err = float(ctx.all_lines(ctx.path("error.file.path"))[0].split("=")[1])
    alpha = 0.5 * math.log((1.0 - err) / err) if 0 < err < 1 else 0.0
    po, ao, bo = (ctx.get_int("pred.class.attr.ord"), ctx.get_int("actual.class.attr.ord"),
                  ctx.get_int("boost.attr.ord"))
    prec = int(ctx.cfg.values.get("abe.output.precision", 6))
    init = ctx.get_float("intial.weight", 1.0)
    w, wrong, n_rows, src = _boost_columns(ctx, po, ao, bo)
    nw = w * torch.exp(torch.where(wrong, torch.full_like(w, alpha), torch.full_like(w, -alpha))) if err < 0.5 \
        else torch.full_like(w, init)
    if not isinstance(src, list):         # native: the raw fields around the new weight
        from .common import field_columns
        width = src.width()
        if width is None:
            raise SystemExit("adaBoostUpdate: records of differing field counts")
        spans = src.line_spans()
        ctx.emit_columns(field_columns(spans, width, ctx.native_delim(), {bo: ("f", nw, prec)}), n_rows)
        return
    rows = src
    d = ctx.delim_out
    out = []
    for r, v in zip(rows, nw.tolist()):
        r = list(r)
        r[bo] = fmt(v, prec)
        out.append(d.join(r))
    ctx.emit(out)


def _boost_columns(ctx, po, ao, bo):
    """(boost weights f64, misclassified bool, record count, Records or the split rows)."""
    from .common import field_modes
    rec = ctx.try_records(modes=field_modes({po: "d", ao: "d", bo: "n"}), tail_mode="x", numeric=True)
    if rec is not None:
        return rec.field(bo, numeric=True).double(), rec.field(po) != rec.field(ao), rec.n_lines, rec
    rows = ctx.rows()
    w = torch.tensor([float(r[bo]) for r in rows], dtype=torch.float64)
    wrong = torch.tensor([r[po] != r[ao] for r in rows], dtype=torch.bool)
    return w, wrong, len(rows), rows


# ================================================================================================
# split generation (tree building blocks)
# ================================================================================================
@job("classPartitionGenerator", "candidate splits with gain ratio per attribute (J/explore/ClassPartitionGenerator.java, cpg.*)",
     aliases=("splitGenerator",))
def class_partition(args):
    """One split-histogram launch over all attributes' candidate splits (K2 over tree-binned
    codes), all-reduced, then every split's stat from one batched ``[S, G, C]`` contraction.
    ``cpg.split.attributes`` restricts the attributes; ``cpg.at.root`` emits the root info only."""
    from ..models.splitstat import class_partition_stats, info_content
    ctx = JobContext(args, "cpg.")
    t = ctx.table(raw_numeric=True)
    alg = ctx.get_str("split.algorithm", "giniIndex")
    d = ctx.delim_out
    if ctx.get_bool("at.root", False):
        C = t.n_classes
        cnt = torch.bincount(t.labels[: t.n].long().cpu(), minlength=C)[:C].double()
        ctx.all_reduce(cnt)
        ctx.emit_root([f"$root{d}{float(info_content(cnt, alg)):.6f}"])
        return
    attrs = ctx.get_int_list("split.attributes", None)
    st = class_partition_stats(t, alg, attrs, comm=ctx.comm)
    ctx.emit_root([f"{s['attr']}{d}{s['key']}{d}{s['gain_ratio']:.6f}" for s in st])


# ================================================================================================
# encodings / mappers
# ================================================================================================
def java_hash(s: str) -> int:
    h = 0
    for ch in s:
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


def fnv_hash(s: str) -> int:
    h = 0x811C9DC5
    for b in s.encode():
        h ^= b
        h = (h * 0x01000193) & 0xFFFFFFFF
    return h


@job("categoricalFeatureHashingEncoding", "hashing-trick encoding (S/explore/CategoricalFeatureHashingEncoding.scala)")
def feature_hashing_job(args):
    """Index hash = Java ``String.hashCode`` mod ``encoding.size``, sign = FNV-1a parity; the vector
    replaces the categorical fields at ``encoding.vecOffset`` among the remaining fields.  Values
    are hashed once per distinct value, the [n, size] encoding is one scatter-add."""
    from .common import field_columns, field_modes
    ctx = JobContext(args, app="categoricalFeatureHashingEncoding")
    cat = ctx.get_int_list("cat.fieldOrdinals")
    size = ctx.get_int("encoding.size")
    rec = ctx.try_records(modes=field_modes({o: "d" for o in cat}), tail_mode="x")
    if rec is not None and rec.width() is not None:
        # native: each distinct value hashed once (dictionary level), the [n, size] encoding one
        # scatter-add on the device, the other fields re-emitted from the raw line bytes
        n, width = rec.n_lines, rec.width()
        codes = torch.stack([rec.field(o).long() for o in cat], 1) if cat else \
            torch.zeros((n, 0), dtype=torch.long, device=rec.device)
        idx = torch.tensor([abs(java_hash(v)) % size for v in rec.vocab] or [0], dtype=torch.long,
                           device=rec.device)
        sgn = torch.tensor([1 if fnv_hash(v) % 2 == 1 else -1 for v in rec.vocab] or [0], dtype=torch.long,
                           device=rec.device)
        enc = torch.zeros((n, size), dtype=torch.long, device=rec.device)
        if n and rec.vocab and cat:
            enc.scatter_add_(1, idx[codes.clamp_min(0)], sgn[codes.clamp_min(0)] * (codes >= 0))
        rem = [i for i in range(width) if i not in set(cat)]
        off = ctx.get_int("encoding.vecOffset", len(rem))
        spans = rec.line_spans()
        dl = ctx.native_delim()
        other = [spans.column("rf", i, dl) for i in rem]
        ctx.emit_columns(other[:off] + [("i", enc[:, j]) for j in range(size)] + other[off:], n)
        return
    rows = ctx.rows()
    n = len(rows)
    vocab: dict[str, int] = {}
    codes = torch.tensor([[vocab.setdefault(r[o], len(vocab)) for o in cat] for r in rows], dtype=torch.long).view(n, -1)
    inv = sorted(vocab, key=vocab.get)
    idx = torch.tensor([abs(java_hash(v)) % size for v in inv], dtype=torch.long)
    sgn = torch.tensor([1 if fnv_hash(v) % 2 == 1 else -1 for v in inv], dtype=torch.long)
    enc = torch.zeros((n, size), dtype=torch.long)
    if n and inv:
        enc.scatter_add_(1, idx[codes], sgn[codes])
    rem = [i for i in range(len(rows[0]) if rows else 0) if i not in set(cat)]
    off = ctx.get_int("encoding.vecOffset", len(rem))
    d = ctx.delim_out
    out = []
    for r, e in zip(rows, enc.tolist()):
        other = [r[i] for i in rem]
        out.append(d.join(other[:off] + [str(v) for v in e] + other[off:]))
    ctx.emit(out)


@job("categoricalLeaveOneOutEncoding", "leave-one-out target encoding (S/explore/CategoricalLeaveOneOutEncoding.scala)")
def loo_encoding(args):
    """Training set: per (field, value) (count, sum of the +1/-1 target) is all-reduced and saved to
    ``target.stat.file.path`` as ``field,value,count,sum``; each value is encoded as
    ``(sum - y) / (count - 1 + reg) * (1 + N(0, rand.std.dev))``.  Validation / test set: the saved
    stats are loaded and ``sum / (count + reg)`` is used (:66-136)."""
    ctx = JobContext(args, app="categoricalLeaveOneOutEncoding")
    cat = ctx.get_int_list("cat.field.ordinals")
    cls_ord = ctx.get_int("class.field.ordinal")
    pos = ctx.get_str("class.pos.val", None)
    reg = ctx.get_float("regularization.factor", 10.0)
    sd = ctx.get_float("rand.std.dev", 0.3)
    prec = ctx.get_int("ouput.precision", 3)
    train = ctx.get_bool("train.data.set", True)
    stat_path = ctx.get_str("target.stat.file.path", None)
    from .common import field_modes
    rec = ctx.try_records(modes=field_modes({**{o: "d" for o in cat}, cls_ord: "d" if pos is not None else "n"}),
                          tail_mode="x", numeric=pos is None)
    if rec is not None and rec.width() is not None:
        _loo_native(ctx, rec, cat, cls_ord, pos, reg, sd, prec, train, stat_path)
        return
    rows = ctx.rows()
    yv = torch.tensor([(1.0 if r[cls_ord] == pos else -1.0) if pos is not None else float(r[cls_ord]) for r in rows],
                      dtype=torch.float64)
    keys = ctx.union((o, r[o]) for r in rows for o in cat)
    ki = {k: i for i, k in enumerate(keys)}
    K = len(keys)
    if train:
        cnt = torch.zeros(K, dtype=torch.float64)
        sm = torch.zeros(K, dtype=torch.float64)
        for j, o in enumerate(cat):
            kk = torch.tensor([ki[(o, r[o])] for r in rows], dtype=torch.long)
            cnt.index_add_(0, kk, torch.ones_like(yv))
            sm.index_add_(0, kk, yv)
        ctx.all_reduce(cnt, sm)
        ctx.check()
        if stat_path and ctx.is_root:
            from pathlib import Path
            Path(stat_path).parent.mkdir(parents=True, exist_ok=True)
            Path(stat_path).write_text("\n".join(f"{o}{ctx.delim_out}{v}{ctx.delim_out}{int(cnt[i])}{ctx.delim_out}{int(sm[i])}"
                                                 for i, (o, v) in enumerate(keys)) + "\n")
        stats = {k: (float(cnt[i]), float(sm[i])) for k, i in ki.items()}
    else:
        stats = {}
        for l in ctx.all_lines(stat_path):
            p = ctx.split(l)
            stats[(int(p[0]), p[1])] = (float(p[2]), float(p[3]))
    seed = ctx.get_int("random.seed", 0)
    base = ctx.line_base(len(rows)) if train else 0
    out = []
    d = ctx.delim_out
    enc = {}
    zc: dict = {}
    for j, o in enumerate(cat):
        c = torch.tensor([stats[(o, r[o])][0] for r in rows], dtype=torch.float64)
        s = torch.tensor([stats[(o, r[o])][1] for r in rows], dtype=torch.float64)
        if train:
            noise = 1.0 + (_loo_noise(seed, j, base, len(rows), None, zc) * sd).clamp(-3 * sd, 3 * sd)
            enc[o] = ((s - yv) / (c - 1 + reg) * noise).tolist()
        else:
            enc[o] = (s / (c + reg)).tolist()
    for i, r in enumerate(rows):
        r = list(r)
        for o in cat:
            r[o] = fmt(enc[o][i], prec)
        out.append(d.join(r))
    ctx.emit(out)


def _loo_noise(seed: int, field: int, base: int, n: int, device=None, cache: dict | None = None) -> torch.Tensor:
    """N(0, 1) noise of the leave-one-out encoding: Philox(seed, field j, GLOBAL line index) from
    the threaded host generator (csrc/host/random.cpp), so a line's noise depends neither on the
    rank that reads it nor on the device (the reference draws from a per-partition
    java.util.Random, S/explore/CategoricalLeaveOneOutEncoding.scala:80-136; torch.randn of 2^21
    doubles on one CPU thread was 25 ms of a 74 ms job, profiles/r6_slow_jobs.jsonl)."""
    from .. import _native
    # fields 2k and 2k + 1 share one Philox draw per line (the two Box-Muller outputs); a device
    # path draws on the GPU with the same fp64 formula (sampler.hip::philox_normal_kernel)
    key = int(field) // 2
    if cache is not None and key in cache:
        return cache[key][:, int(field) % 2]
    dev = torch.device(device) if device is not None else torch.device("cpu")
    z = _native.C().philox_normal(int(seed), key, int(base), int(n), True, dev if dev.type == "cuda" else None)
    if cache is not None:
        cache[key] = z
    return z[:, int(field) % 2]


def _loo_native(ctx, rec, cat, cls_ord, pos, reg, sd, prec, train, stat_path):
    """categoricalLeaveOneOutEncoding on a native token table: per (field, dictionary code) count
    and target sums as one [F, V] scatter-add + all-reduce, the encoding a gather, the output the
    raw line bytes with the encoded fields replaced."""
    from .common import field_columns
    n, V, F = rec.n_lines, max(1, len(rec.vocab)), len(cat)
    dev = rec.device
    if pos is not None:
        pc = rec.vocab.index(pos) if pos in rec.vocab else -2
        yv = torch.where(rec.field(cls_ord) == pc, 1.0, -1.0).double()
    else:
        yv = rec.field(cls_ord, numeric=True).double()
    codes = torch.stack([rec.field(o).long() for o in cat], 1) if F else torch.zeros((n, 0), dtype=torch.long, device=dev)
    flat = (torch.arange(F, device=dev).view(1, -1) * V + codes.clamp_min(0)).view(-1)
    if train:
        if dev.type == "cuda" and F:
            # K23 loo_stats_kernel: the (field, value) sums privatised in LDS — a global fp64
            # index_add_ onto a handful of (field, value) slots serialised on its atomics
            # (2.3 s for 2^21 records x 2 fields: profiles/r5_explore_jobs_scale.jsonl)
            from ..ops.encode_ops import loo_stats
            m = V + 1
            cc = codes.clamp_min(0).t().contiguous()
            s2, k2 = (loo_stats(cc.to(torch.uint8), n, yv) if m <= 256 else loo_stats(cc.int(), n, yv, m))
            cnt = k2[:, :V].double().reshape(-1).contiguous()
            sm = s2[:, :V].reshape(-1).contiguous()
        else:
            cnt = torch.zeros(F * V, dtype=torch.float64, device=dev)
            sm = torch.zeros(F * V, dtype=torch.float64, device=dev)
            cnt.index_add_(0, flat, torch.ones(flat.numel(), dtype=torch.float64, device=dev))
            sm.index_add_(0, flat, yv.view(-1, 1).expand(n, F).reshape(-1))
        ctx.all_reduce(cnt, sm)
        ctx.check()
        if stat_path and ctx.is_root:
            from pathlib import Path
            ch, sh = cnt.view(F, V).cpu(), sm.view(F, V).cpu()
            d = ctx.delim_out
            lines = []
            for o in sorted(set(cat)):      # (field, value) keys in sorted order, as the row path's union
                j = cat.index(o)
                present = torch.nonzero(ch[j] > 0).view(-1).tolist()
                for c in sorted(present, key=lambda c: rec.vocab[c]):
                    lines.append(f"{o}{d}{rec.vocab[c]}{d}{int(ch[j, c])}{d}{int(sh[j, c])}")
            Path(stat_path).parent.mkdir(parents=True, exist_ok=True)
            Path(stat_path).write_text("\n".join(lines) + "\n")
    else:
        cnt = torch.zeros(F * V, dtype=torch.float64)
        sm = torch.zeros(F * V, dtype=torch.float64)
        vi = {v: i for i, v in enumerate(rec.vocab)}
        fi = {o: j for j, o in enumerate(cat)}
        for l in ctx.all_lines(stat_path):
            p = ctx.split(l)
            j, c = fi.get(int(p[0])), vi.get(p[1])
            if j is not None and c is not None:
                cnt[j * V + c], sm[j * V + c] = float(p[2]), float(p[3])
        cnt, sm = cnt.to(dev), sm.to(dev)
    seed = ctx.get_int("random.seed", 0)
    base = ctx.line_base(n) if train else 0
    c_, s_ = cnt[flat].view(n, F), sm[flat].view(n, F)
    rep = {}
    zc: dict = {}
    for j, o in enumerate(cat):
        if train:
            noise = 1.0 + (_loo_noise(seed, j, base, n, dev, zc).to(dev) * sd).clamp(-3 * sd, 3 * sd)
            e = (s_[:, j] - yv) / (c_[:, j] - 1 + reg) * noise
        else:
            e = s_[:, j] / (c_[:, j] + reg)
        rep[o] = ("f", e, prec)
    ctx.emit_columns(field_columns(rec.line_spans(), rec.width(), ctx.native_delim(), rep), n)


@job("binaryDummyVariableGenerator", "one-hot (binary dummy) expansion of categorical fields (S/util/BinaryDummyVariableGenerator.scala)")
def binary_dummy_job(args):
    ctx = JobContext(args, app="binaryDummyVariableGenerator")
    cat = ctx.get_int_list("cat.field.ordinals")
    tv, fv = ctx.get_str("true.value", "1"), ctx.get_str("false.value", "0")
    ci = ctx.get_bool("case.insensitive", False)
    from .common import field_columns, field_modes
    rec = ctx.try_records(modes=field_modes({o: "d" for o in cat}), tail_mode="x")
    if rec is not None and rec.width() is not None:
        voc = [v.lower() for v in rec.vocab] if ci else rec.vocab
        rep = {}
        for o in cat:
            c = rec.field(o)
            u = ctx.cfg.get_list(f"fieldUniqueValues.{o}", None)
            if u is None:
                u = ctx.union(rec.strings(torch.unique(c[c >= 0])))
            u = [x.lower() for x in u] if ci else u
            ui = {x: i for i, x in enumerate(u)}
            lut = torch.tensor([ui.get(v, -1) for v in voc] or [-1], dtype=torch.long, device=rec.device)
            k = torch.where(c >= 0, lut[c.long().clamp_min(0)], torch.full_like(c.long(), -1))
            rep[o] = [("s", [fv, tv], (k == i).long()) for i in range(len(u))]
        ctx.emit_columns(field_columns(rec.line_spans(), rec.width(), ctx.native_delim(), rep), rec.n_lines)
        return
    rows = ctx.rows()
    uniq = {}
    for o in cat:
        u = ctx.cfg.get_list(f"fieldUniqueValues.{o}", None)
        if u is None:
            u = ctx.union(r[o] for r in rows)
        uniq[o] = [x.lower() for x in u] if ci else u
    d = ctx.delim_out
    out = []
    for r in rows:
        parts = []
        for i, v in enumerate(r):
            if i in uniq:
                vv = v.lower() if ci else v
                parts += [tv if vv == u else fv for u in uniq[i]]
            else:
                parts.append(v)
        out.append(d.join(parts))
    ctx.emit(out)


@job("linearMapper", "linear transform of numeric fields y = M x (S/util/LinearMapper.scala)")
def linear_mapper(args):
    """``trans.matrix.path`` rows of M (comma separated); output ``ids, y..., retained fields``;
    the transform of the whole shard is one GEMM on the device."""
    ctx = JobContext(args, app="linearMapper")
    ids = ctx.get_int_list("id.field.ordinals", [])
    q = ctx.get_int_list("quant.field.ordinals")
    ret = ctx.get_int_list("retained.field.ordinals", [])
    prec = ctx.get_int("output.precision", 3)
    M = torch.tensor([[float(x) for x in l.split(",")] for l in ctx.all_lines(ctx.path("trans.matrix.path"))],
                     dtype=torch.float64, device=ctx.device)
    X, src = ctx.numeric_matrix(q)
    if not isinstance(src, list):      # native: one GEMM, ids / retained fields from the raw bytes
        Y = X @ M.T
        spans, dl = src.line_spans(), ctx.native_delim()
        ctx.emit_columns([spans.column("rf", o, dl) for o in ids] + [("f", Y[:, j].contiguous(), prec)
                                                                     for j in range(Y.shape[1])]
                         + [spans.column("rf", o, dl) for o in ret], src.n_lines)
        return
    rows = src
    Y = (X @ M.T).cpu().tolist()
    d = ctx.delim_out
    ctx.emit([d.join([r[o] for o in ids] + [fmt(v, prec) for v in y] + [r[o] for o in ret]) for r, y in zip(rows, Y)])


@job("incrementalPrincipalComponent", "streaming PCA per key with persisted state (S/explore/IncrementalPrincipalComponent.scala)")
def incremental_pca(args):
    """Records ``id...,x1..xD`` grouped by key; the state file (``state.filePath``) of the previous
    run is loaded when it exists and written back (PrincipalCompState text blocks); all keys are
    updated together by the batched GHA recursion of ``analytics/pca.py``."""
    from pathlib import Path
    from ..analytics.pca import IncrementalPCA, PrincipalCompState
    ctx = JobContext(args, app="incrementalPrincipalComponent")
    ids = ctx.get_int_list("id.field.ordinals")
    q = ctx.get_int_list("quant.field.ordinals")
    prec = ctx.get_int("output.precision", 3)
    from .common import field_modes
    rec = ctx.try_records(modes=field_modes({**{o: "d" for o in ids}, **{o: "n" for o in q}}), tail_mode="x",
                          numeric=True)
    if rec is not None:
        keys, streams = _keyed_streams(ctx, rec, ids, q)
    else:
        groups = defaultdict(list)
        for r in ctx.rows(shard=False):
            groups[":".join(r[o] for o in ids)].append([float(r[o]) for o in q])
        keys = sorted(groups)
        if ctx.comm.is_distributed:
            from ..data.table import shard_range
            a, b = shard_range(len(keys), ctx.comm.rank, ctx.comm.world)
            keys = keys[a:b]
        streams = {k: torch.tensor(groups[k], dtype=torch.float64) for k in keys}
    ipca = IncrementalPCA(len(q), forget=ctx.get_float("forget.factor", 0.96),
                          low_energy=ctx.get_float("energy.lowThreshold", 0.95),
                          high_energy=ctx.get_float("energy.highThreshold", 0.98), device=ctx.device)
    sp = ctx.get_str("state.filePath", None)
    d = ctx.delim_out
    if sp and Path(sp).exists():
        blk = ctx.all_lines(sp)
        i = 0
        while i < len(blk):
            nh = int(blk[i].split(d)[2])
            st = PrincipalCompState.load(blk[i:i + 3 + nh], d)
            ipca.states[st.key] = st
            i += 3 + nh
    states = ipca.update(streams)
    lines = [l for k in keys for l in states[k].serialize(d, prec)]
    lines = ctx.gather_lines(lines)
    ctx.check()
    if sp and ctx.is_root:
        Path(sp).parent.mkdir(parents=True, exist_ok=True)
        Path(sp).write_text("\n".join(lines) + "\n")
    ctx.emit_root(lines)


def _keyed_streams(ctx, rec, key_ords, val_ords):
    """(this rank's keys in order, {key: [n_k, D] float64 rows in input order}) of a native table:
    byte-range shards, composite keys ranked in the reducer's order, rows shuffled to the rank that
    owns their key (one all-to-all), grouped by a stable device sort."""
    from ..data.records import owner_of, shuffle, sorted_key_tuples
    comm = ctx.comm
    kpos, G, ktab = sorted_key_tuples(rec, [rec.field(o) for o in key_ords], comm)
    gidx = rec.line_base + torch.arange(rec.n_lines, device=rec.device)
    vals = [rec.field(o, numeric=True).double() for o in val_ords]
    if comm.is_distributed:
        kpos, gidx, *vals = shuffle(comm, owner_of(kpos, G, comm.world), [kpos, gidx] + vals)
    o1 = torch.argsort(gidx, stable=True)
    o2 = torch.argsort(kpos[o1], stable=True)
    order = o1[o2]
    X = torch.stack(vals, 1)[order] if vals else torch.zeros((order.numel(), 0), dtype=torch.float64)
    ks = kpos[order]
    uk, cnt = torch.unique_consecutive(ks, return_counts=True)
    names = [":".join(rec.vocab[c] for c in row) for row in ktab[uk.cpu()].tolist()]
    parts = torch.split(X.cpu(), cnt.cpu().tolist())
    return names, dict(zip(names, parts))


@job("individualConditionalExpectation", "ICE curves by grid expansion + in-process batched model inference (S/interpret/IndividualConditionalExpectation.scala)")
def ice_job(args):
    """Input ``key...,x1..xD``; ``ice.feature.ordinal`` (feature index within x) is varied over
    ``ice.feature.values``; the reference HTTP-POSTs every grid batch to a prediction service, here
    the model (``--kind`` + ``--config``, the P/supv classifier drivers) scores the whole expanded
    grid in one batched call.  Output ``key...,value,prediction`` sorted by prediction per key
    (descending by default)."""
    from ..models import supervised as SV
    ctx = JobContext(args, app="individualConditionalExpectation")
    kl = ctx.get_int("data.keyLen")
    feat = ctx.get_int("feature.ordinal")
    vals = ctx.get_float_list("feature.values")
    desc = ctx.get_bool("prediction.sortDescending", True)
    prec = ctx.get_int("output.precision", 3)
    cls = {"rf": SV.RandomForest, "gbt": SV.GradientBoostedTrees, "svm": SV.SupportVectorMachine,
           "lr": SV.LogisticRegressionDiscriminant}[args.kind]
    model = cls(ctx.get_str("model.config", None) or args.model, device=args.device)
    model.train()
    rec = ctx.try_records(modes="x" * kl, tail_mode="n", numeric=True)
    if rec is not None and rec.width() is not None:
        n, V = rec.n_lines, len(vals)
        X = rec.nums.view(n, rec.width())[:, kl:].double().cpu()
        G = X.repeat_interleave(V, 0)
        G[:, feat] = torch.tensor(vals, dtype=torch.float64).repeat(n)
        p = torch.as_tensor(model.predictProb(G.numpy()))
        p = (p[:, -1] if p.dim() == 2 else p).double().view(n, V)
        order = torch.sort(p, 1, descending=desc, stable=True).indices
        rows_i = torch.arange(n).repeat_interleave(V)
        spans, dl = rec.line_spans().select(rows_i), ctx.native_delim()
        cols = [spans.column("rf", j, dl) for j in range(kl)]
        vt = torch.tensor(vals, dtype=torch.float64)
        cols += [("f", vt[order.reshape(-1)], -1), ("f", torch.gather(p, 1, order).reshape(-1), prec)]
        ctx.emit_columns(cols, n * V)
        return
    rows = ctx.rows()
    X = torch.tensor([[float(v) for v in r[kl:]] for r in rows], dtype=torch.float64)
    G = X.repeat_interleave(len(vals), 0)
    G[:, feat] = torch.tensor(vals, dtype=torch.float64).repeat(len(rows))
    p = model.predictProb(G.numpy())
    p = torch.as_tensor(p)
    p = p[:, -1] if p.dim() == 2 else p
    p = p.view(len(rows), len(vals))
    d = ctx.delim_out
    out = []
    for i, r in enumerate(rows):
        order = sorted(range(len(vals)), key=lambda j: float(p[i, j]), reverse=desc)
        out += [d.join(r[:kl] + [f"{vals[j]:g}", fmt(float(p[i, j]), prec)]) for j in order]
    ctx.emit(out)


# ================================================================================================
# discriminant analysis / SVM
# ================================================================================================
@job("fisherDiscriminant", "univariate Fisher discriminant per attribute, binary class (J/discriminant/FisherDiscriminant.java)")
def fisher(args):
    from ..models.linear import fisher_discriminant, fisher_lines
    ctx = JobContext(args, "fid.")
    t = ctx.table(raw_numeric=True)
    X = t.dense_features()
    r = fisher_discriminant(X, t.labels[: t.n].long(), comm=ctx.comm)
    ords = [f.ordinal for f in t.binned_fields] + [f.ordinal for f in t.numeric_fields]
    d = ctx.delim_out
    ctx.emit_root([d.join([str(o)] + l.split(",")[1:]) for o, l in zip(ords, fisher_lines(r.cpu()))])


@job("supportVectorMachine", "cascade SVM: per-rank SMO, all-gather of support vectors, final SMO (J/discriminant/SupportVectorMachine.java)")
def svm_job(args):
    """Output: one line per final support vector ``alpha,classValue,x...`` then ``bias,<b>``
    (decision f(x) = sum alpha_i y_i K(x_i, x) + b)."""
    from ..models.svm import CascadeSVM
    ctx = JobContext(args, "svm.")
    t = ctx.table(raw_numeric=True)
    X = t.dense_features().float()
    y = t.labels[: t.n].long()
    pos = ctx.get_str("positive.class.value", None)
    vals = t.class_field.cardinality
    pi = vals.index(pos) if pos in vals else 1
    yb = (y == pi).long()
    m = CascadeSVM(comm=ctx.comm, C=ctx.get_float("penalty.factor", 1.0), kernel=ctx.get_str("kernel.type", "linear"),
                   gamma=ctx.get_float("kernel.param", 1.0)).fit(X, yb)
    d = ctx.delim_out
    sv = m.model
    coef = sv.dual_coef[0].cpu().tolist()
    lines = [d.join([f"{abs(a):.6f}", vals[pi] if a > 0 else vals[1 - pi]] + [f"{v:.6f}" for v in x])
             for a, x in zip(coef, sv.sv_X.cpu().tolist())]
    lines.append(f"bias{d}{-float(sv.rho[0]):.6f}")
    ctx.emit_root(lines)
