"""External pipeline stages the reference's drivers call from chombo / sifarish:
``Normalizer``, ``Projection``, ``TemporalFilter``, ``Transformer`` (keyValueTrans),
``UniqueValueCounter``, ``TimeIntervalGenerator``, ``NumericalAttrDistrStats`` — plus the
histogram-file form of the KS drift job they feed (R/ovsa.sh, R/fit.sh, R/hica.sh, R/caen.sh,
R/dvg.sh, R/ks.sh).

chombo and sifarish are not part of the reference tree, so these are re-statements of the
behaviour the drivers and property files rely on (keys from resource/*.properties / *.conf);
their text layouts are documented per job and exercised end to end by tests/test_pipelines.py
(parity unpinned beyond what the reference's own consumers parse).
"""
from __future__ import annotations

import math
from collections import defaultdict
from pathlib import Path

import torch

from .common import JobContext, fmt, job


@job("normalizer", "numeric attribute normalisation zscore | minmax (chombo mr.Normalizer, nor.*)")
def normalizer(args):
    """``nor.num.attribute.ordinals``; global mean / std / min / max from one moments all-reduce;
    ``zscore`` (optionally ``force.unit.range``: then min-max scaled to [0, 1]) or ``minmax``."""
    ctx = JobContext(args, "nor.")
    ords = ctx.get_int_list("num.attribute.ordinals")
    strat = ctx.get_str("normalizing.strategy", "minmax")
    prec = ctx.get_int("floating.precision", 3)
    X, src = ctx.numeric_matrix(ords)
    nrow, dv = X.shape[0], X.device
    st = torch.stack([torch.full((len(ords),), float(nrow), dtype=torch.float64, device=dv), X.sum(0), (X * X).sum(0)])
    mn = X.min(0).values if nrow else torch.full((len(ords),), math.inf, dtype=torch.float64, device=dv)
    mx = X.max(0).values if nrow else torch.full((len(ords),), -math.inf, dtype=torch.float64, device=dv)
    ctx.all_reduce(st)
    if ctx.comm.is_distributed:
        ctx.comm.all_reduce(mn, "min")
        ctx.comm.all_reduce(mx, "max")
    n = st[0]
    mean = st[1] / n
    sd = ((st[2] / n - mean * mean).clamp_min(0) * n / (n - 1).clamp_min(1)).sqrt().clamp_min(1e-300)
    if strat == "zscore":
        Y = (X - mean) / sd
        if ctx.get_bool("force.unit.range", False):
            lo, hi = (mn - mean) / sd, (mx - mean) / sd
            Y = (Y - lo) / (hi - lo).clamp_min(1e-300)
    else:
        Y = (X - mn) / (mx - mn).clamp_min(1e-300)
    if not isinstance(src, list):         # native: the raw fields around the normalised values
        if _emit_replaced(ctx, src, {o: ("f", Y[:, j].contiguous(), prec) for j, o in enumerate(ords)}):
            return
        rows = ctx.rows()
    else:
        rows = src
    d = ctx.delim_out
    out = []
    for r, y in zip(rows, Y.tolist()):
        r = list(r)
        for o, v in zip(ords, y):
            r[o] = fmt(v, prec)
        out.append(d.join(r))
    ctx.emit(out)


@job("projection", "field projection with an optional row filter (chombo mr.Projection, pro.*)")
def projection(args):
    """``pro.projection.field`` ordinals in output order; ``pro.select.filter`` is a rule condition
    (``8 eq int:1``), evaluated column-wise (utils/rules.py)."""
    from ..utils.rules import RuleExpression
    ctx = JobContext(args, "pro.")
    fields = ctx.get_int_list("projection.field")
    flt = ctx.get_str("select.filter", None)
    rule = RuleExpression.from_condition(flt, ctx.get_str("cond.delim", " and ")) if flt else None
    from ..utils.rules import RecordColumns, rule_field_modes
    from .common import field_modes
    fm = rule_field_modes([rule] if rule else [])
    rec = ctx.try_records(modes=field_modes(fm), tail_mode="x", numeric=True, trim=True)
    if rec is not None:
        keep = rule.evaluate(RecordColumns(rec, [o for o, m in fm.items() if m == "n"])).cpu() if rule else \
            torch.ones(rec.n_lines, dtype=torch.bool)
        spans, dl = rec.line_spans().select(keep), ctx.native_delim()
        ctx.emit_columns([spans.column("rf", o, dl) for o in fields], len(spans))
        return
    rows = ctx.rows()
    keep = RuleExpression.from_condition(flt, ctx.get_str("cond.delim", " and ")).evaluate_rows(rows).tolist() \
        if flt else [True] * len(rows)
    d = ctx.delim_out
    ctx.emit([d.join(r[o] for o in fields) for r, k in zip(rows, keep) if k])


@job("temporalFilter", "keep records inside a time range (chombo mr.TemporalFilter, tef.*)")
def temporal_filter(args):
    ctx = JobContext(args, "tef.")
    to = ctx.get_int("time.stamp.field.ordinal")
    lo, hi = (float(x) for x in ctx.get_str("time.range").split(":"))
    mult = 1.0 if ctx.get_bool("time.stamp.in.mili", False) else 1000.0
    shift = ctx.get_float("time.zone.shift.hours", 0.0) * 3600.0
    t, src = ctx.numeric_matrix([to])
    t = t[:, 0].cpu()
    if mult == 1.0:
        t = t / 1000.0
    t = t + shift
    keep = (t >= lo) & (t <= hi)
    if not isinstance(src, list):
        spans = src.line_spans().select(keep)
        ctx.emit_columns([spans.column("r", delims=ctx.native_delim())], len(spans))
        return
    d = ctx.delim_out
    ctx.emit([d.join(r) for r, k in zip(src, keep.tolist()) if k])


@job("transformer", "attribute transformers from a schema (chombo mr.Transformer, tra.*): keyValueTrans lookup")
def transformer(args):
    """``tra.transformer.schema.file.path``: attributes with ``transformers`` and
    ``targetFieldOrdinals``; ``keyValueTrans`` replaces a value by the value of its key in the
    ``hdfsDataPath`` file of ``tra.transformer.config.file.path`` (lines ``key,value``, or the
    encoder's ``attr,key,value`` where the attribute ordinal must match)."""
    import json
    from ..utils.config import read_hocon
    ctx = JobContext(args, "tra.")
    sch = json.loads(Path(ctx.path("transformer.schema.file.path")).read_text())
    conf = read_hocon(ctx.path("transformer.config.file.path")).get("transformers", {})
    attrs = sch.get("attributes", sch.get("fields", []))
    luts: dict[int, dict[str, str]] = {}
    for a in attrs:
        for tname in a.get("transformers", []):
            if tname != "keyValueTrans":
                raise SystemExit(f"unsupported transformer {tname}")
            c = conf.get(tname, {})
            p = c.get("hdfsDataPath") or c.get("dataPath")
            fd = c.get("fieldDelim", ",")
            p = ctx.path(None, None, p) if not Path(p).exists() else p
            lut = {}
            for l in ctx.all_lines(p):
                q = l.split(fd)
                if len(q) >= 3:
                    if int(q[0]) == a["ordinal"]:
                        lut[q[1]] = q[2]
                else:
                    lut[q[0]] = q[1]
            luts[a["ordinal"]] = lut
    from .common import field_modes
    rec = ctx.try_records(modes=field_modes({a["ordinal"]: "d" for a in attrs}), tail_mode="x")
    if rec is not None and rec.width() is not None:
        # native: each attribute's lookup is one table over the dictionary; every target field is
        # a string-table column, the other fields the raw bytes
        rep_cols = {}
        for a in attrs:
            o = a["ordinal"]
            lut = luts.get(o, {})
            tab = [lut.get(w, w) for w in rec.vocab]
            for t in a.get("targetFieldOrdinals", [o]):
                rep_cols[t] = ("s", tab, rec.field(o))
        width = max([rec.width()] + [t + 1 for t in rep_cols])
        spans = rec.line_spans()
        cols = [rep_cols[j] if j in rep_cols else (spans.column("rf", j, ctx.native_delim()) if j < rec.width()
                                                  else ("c", "")) for j in range(width)]
        ctx.emit_columns(cols, rec.n_lines)
        return
    d = ctx.delim_out
    out = []
    for r in ctx.rows():
        o = list(r)
        for a in attrs:
            v = r[a["ordinal"]]
            if a["ordinal"] in luts:
                v = luts[a["ordinal"]].get(v, v)
            for t in a.get("targetFieldOrdinals", [a["ordinal"]]):
                while len(o) <= t:
                    o.append("")
                o[t] = v
        out.append(d.join(o))
    ctx.emit(out)


@job("uniqueValueCounter", "distinct values (and counts) of categorical fields (chombo spark.explore.UniqueValueCounter)")
def unique_value_counter(args):
    """Output per field ``ordinal,value[,count],...`` (``count.values``); the per-rank counters are
    merged over ranks."""
    from collections import Counter
    ctx = JobContext(args, app="uniqueValueCounter")
    ords = ctx.get_int_list("cat.field.ordinals", None) or ctx.get_int_list("cat.fieldOrdinals")
    ci = ctx.get_bool("case.insensitive", False)
    from .common import field_modes
    rec = ctx.try_records(modes=field_modes({o: "d" for o in ords}), tail_mode="x")
    if rec is not None:
        # native: per field one bincount over the (globally merged) dictionary, one all-reduce
        voc = [w.lower() for w in rec.vocab] if ci else rec.vocab
        uv = sorted(set(voc))
        ui = {w: i for i, w in enumerate(uv)}
        lut = torch.tensor([ui[w] for w in voc] or [0], dtype=torch.long, device=rec.device)
        U = max(1, len(uv))
        C = torch.stack([torch.bincount(lut[c[c >= 0].long()], minlength=U)[:U] for c in
                         (rec.field(o) for o in ords)]) if ords else torch.zeros((0, U), dtype=torch.long)
        ctx.all_reduce(C)
        with_counts = ctx.get_bool("count.values", False)
        d = ctx.delim_out
        out = []
        for j, o in enumerate(ords):
            parts = [str(o)]
            for i in torch.nonzero(C[j] > 0).view(-1).tolist():
                parts += [uv[i], str(int(C[j, i]))] if with_counts else [uv[i]]
            out.append(d.join(parts))
        ctx.emit_root(out)
        return
    cnt = Counter()
    for r in ctx.rows():
        for o in ords:
            cnt[(o, r[o].lower() if ci else r[o])] += 1
    cnt = ctx.sum_counts(cnt)
    with_counts = ctx.get_bool("count.values", False)
    d = ctx.delim_out
    out = []
    for o in ords:
        vals = sorted(v for (oo, v) in cnt if oo == o)
        parts = [str(o)]
        for v in vals:
            parts += [v, str(cnt[(o, v)])] if with_counts else [v]
        out.append(d.join(parts))
    ctx.emit_root(out)


@job("timeIntervalGenerator", "time since the previous record of the same id (chombo spark.explore.TimeIntervalGenerator)")
def time_interval(args):
    """Records grouped by ``id.fieldOrdinals`` and ordered by ``time.fieldOrdinal`` (device
    segmented sort); each record gets the interval to its predecessor (first record: 0) appended
    (``time.keepField=false`` replaces the time field by the interval)."""
    ctx = JobContext(args, app="timeIntervalGenerator")
    kords = ctx.get_int_list("id.fieldOrdinals")
    to = ctx.get_int("time.fieldOrdinal")
    keep = ctx.get_bool("time.keepField", True)
    from .common import field_modes
    rec = ctx.try_records(modes=field_modes({**{o: "d" for o in kords}, to: "n"}), tail_mode="x", numeric=True)
    if rec is not None:
        _time_interval_native(ctx, rec, kords, to, keep)
        return
    rows = ctx.rows(shard=False)
    keys = sorted({tuple(r[o] for o in kords) for r in rows})
    ki = {k: i for i, k in enumerate(keys)}
    k = torch.tensor([ki[tuple(r[o] for o in kords)] for r in rows], dtype=torch.long)
    t = torch.tensor([int(float(r[to])) for r in rows], dtype=torch.long)
    order = torch.argsort(t, stable=True)
    order = order[torch.argsort(k[order], stable=True)]
    ks, ts = k[order], t[order]
    dt = torch.zeros_like(ts)
    same = ks[1:] == ks[:-1]
    dt[1:] = torch.where(same, ts[1:] - ts[:-1], torch.zeros_like(ts[1:]))
    d = ctx.delim_out
    out = []
    for i, v in zip(order.tolist(), dt.tolist()):
        r = list(rows[i])
        if keep:
            r.append(str(v))
        else:
            r[to] = str(v)
        out.append(d.join(r))
    from ..data.table import shard_range
    a, b = shard_range(len(out), ctx.comm.rank, ctx.comm.world)
    ctx.emit(out[a:b])


def _time_interval_native(ctx, rec, kords, to, keep):
    """timeIntervalGenerator over byte-range shards: every record (with its line bytes) moves to the
    rank owning its key (keys in string order cut into contiguous blocks), one device sort by
    (key, time, input order) there, intervals by one shifted difference."""
    from ..data.records import owner_of, shuffle, shuffle_spans, sorted_key_tuples
    comm = ctx.comm
    kpos, G, _ = sorted_key_tuples(rec, [rec.field(o) for o in kords], comm)
    t = rec.field(to, numeric=True).long()
    gidx = rec.line_base + torch.arange(rec.n_lines, device=t.device)
    spans = rec.line_spans()
    if comm.is_distributed:
        owner = owner_of(kpos, G, comm.world)
        spans = shuffle_spans(comm, owner.cpu(), spans)
        kpos, t, gidx = shuffle(comm, owner, [kpos, t, gidx])
    o = torch.argsort(gidx, stable=True)
    o = o[torch.argsort(t[o], stable=True)]
    o = o[torch.argsort(kpos[o], stable=True)]
    ks, ts = kpos[o], t[o]
    dt = torch.zeros_like(ts)
    if ts.numel() > 1:
        dt[1:] = torch.where(ks[1:] == ks[:-1], ts[1:] - ts[:-1], torch.zeros_like(ts[1:]))
    sel = spans.select(o.cpu())
    dl = ctx.native_delim()
    if keep:
        cols = [sel.column("r", delims=dl), ("i", dt)]
    else:
        W = rec.width()
        if W is None:
            raise SystemExit("timeIntervalGenerator: records of differing field counts")
        from .common import field_columns
        cols = field_columns(sel, W, dl, {to: ("i", dt)})
    ctx.emit_columns(cols, len(sel))


def _emit_replaced(ctx, rec, replace: dict) -> bool:
    """Emit every record with fields ``replace`` swapped for format columns (fixed-width tables);
    False when the records differ in width (the caller takes its row path)."""
    from .common import field_columns
    W = rec.width()
    if W is None:
        return False
    ctx.emit_columns(field_columns(rec.line_spans(), W, ctx.native_delim(), replace), rec.n_lines)
    return True


@job("numericalAttrDistrStats", "per-key fixed-width histograms of numeric attributes (chombo spark.explore.NumericalAttrDistrStats)")
def num_distr_stats(args):
    """Per (id.fieldOrdinals key, attribute) a histogram of bin width ``attrBinWidth.<ord>``; one
    ``[G, A, B]`` scatter-add, all-reduced.  Line layout (read by kolmogorovSmirnovModelDrift):
    ``key..,attr,binWidth,count,mean,stdDev,bin,cnt,bin,cnt,...``."""
    ctx = JobContext(args, app="numericalAttrDistrStats")
    kords = ctx.get_int_list("id.fieldOrdinals", []) if ctx.has("id.fieldOrdinals") else []
    attrs = ctx.get_int_list("attr.ordinals")
    prec = ctx.get_int("output.precision", 3)
    from .common import field_modes
    rec = ctx.try_records(modes=field_modes({**{o: "d" for o in kords}, **{a: "n" for a in attrs}}), tail_mode="x",
                          numeric=True)
    if rec is not None:
        _num_distr_native(ctx, rec, kords, attrs, prec)
        return
    rows = ctx.rows()
    keys = ctx.union(tuple(r[o] for o in kords) for r in rows)
    ki = {k: i for i, k in enumerate(keys)}
    g = torch.tensor([ki[tuple(r[o] for o in kords)] for r in rows], dtype=torch.long)
    d = ctx.delim_out
    out = []
    for a in attrs:
        bw = float(ctx.cfg.values.get(f"attrBinWidth.{a}", ctx.get_float("bin.width", 1.0)))
        x = torch.tensor([float(r[a]) for r in rows], dtype=torch.float64)
        b = torch.floor(x / bw).long()
        lo = torch.tensor([int(b.min()) if len(rows) else 0])
        hi = torch.tensor([int(b.max()) if len(rows) else 0])
        if ctx.comm.is_distributed:
            ctx.comm.all_reduce(lo, "min")
            ctx.comm.all_reduce(hi, "max")
        B = int(hi - lo) + 1
        Hh = torch.zeros(len(keys) * B, dtype=torch.long).index_add_(0, g * B + (b - int(lo)), torch.ones_like(b)).view(len(keys), B)
        mom = torch.zeros((len(keys), 3), dtype=torch.float64)
        mom[:, 0].index_add_(0, g, torch.ones_like(x))
        mom[:, 1].index_add_(0, g, x)
        mom[:, 2].index_add_(0, g, x * x)
        ctx.all_reduce(Hh, mom)
        for i, k in enumerate(keys):
            n = float(mom[i, 0])
            if n == 0:
                continue
            mean = float(mom[i, 1]) / n
            sd = math.sqrt(max(float(mom[i, 2]) / n - mean * mean, 0.0))
            bins = [f"{(j + int(lo)) * bw:g}{d}{c}" for j, c in enumerate(Hh[i].tolist()) if c]
            out.append(d.join(list(k) + [str(a), f"{bw:g}", str(int(n)), fmt(mean, prec), fmt(sd, prec)] + bins))
    ctx.emit_root(out)


def _num_distr_native(ctx, rec, kords, attrs, prec):
    """numericalAttrDistrStats on a native token table: global key positions (string order), one
    [G, B] histogram scatter-add and one moments scatter per attribute, all-reduced."""
    from ..data.records import sorted_key_tuples
    g, G, ktab = sorted_key_tuples(rec, [rec.field(o) for o in kords], ctx.comm) if kords else \
        (torch.zeros(rec.n_lines, dtype=torch.long, device=rec.device), 1, torch.zeros((1, 0), dtype=torch.long))
    on_dev = rec.device.type == "cuda"
    if not on_dev:
        g = g.cpu()
    keys = [tuple(rec.vocab[c] for c in row) for row in ktab.tolist()]
    d = ctx.delim_out
    out = []
    for a in attrs:
        bw = float(ctx.cfg.values.get(f"attrBinWidth.{a}", ctx.get_float("bin.width", 1.0)))
        x = rec.field(a, numeric=True).double()
        if not on_dev:
            x = x.cpu()
        b = torch.floor(x / bw).long()
        n = x.numel()
        # bin range: one device reduction, one host read of both ends
        lo, hi = (torch.stack([b.min(), b.max()]).cpu() if n else torch.zeros(2, dtype=torch.long)).view(2, 1)
        if ctx.comm.is_distributed:
            ctx.comm.all_reduce(lo, "min")
            ctx.comm.all_reduce(hi, "max")
        B = int(hi - lo) + 1
        if on_dev and G * B < (1 << 20):
            # K23 LDS-privatised (code, value) sums (ops/encode_ops.loo_stats): the joint (key, bin)
            # counts and the per-key sums of x and x^2 as three passes over the device columns —
            # a global index_add onto G * B slots serialises on its atomics (the host index_add
            # was 13 ms of a 41 ms job at 2^21 records: profiles/r6_slow_jobs.jsonl)
            from ..ops.encode_ops import loo_stats
            gi = g.int().view(1, -1)
            kb = (g * B + (b - int(lo))).int().view(1, -1)
            _, kc = loo_stats(kb, n, torch.zeros(n, dtype=torch.float64, device=x.device), G * B + 1)
            s1, k1 = loo_stats(gi, n, x, G + 1)
            s2, _ = loo_stats(gi, n, x * x, G + 1)
            Hh = kc[0, :G * B].long().view(G, B)
            mom = torch.stack([k1[0, :G].double(), s1[0, :G], s2[0, :G]], 1)
        else:
            Hh = torch.zeros(G * B, dtype=torch.long, device=b.device).index_add_(
                0, g * B + (b - int(lo)), torch.ones_like(b)).view(G, B)
            mom = torch.zeros((G, 3), dtype=torch.float64, device=x.device)
            mom[:, 0].index_add_(0, g, torch.ones_like(x))
            mom[:, 1].index_add_(0, g, x)
            mom[:, 2].index_add_(0, g, x * x)
        ctx.all_reduce(Hh, mom)
        Hh, mom = Hh.cpu(), mom.cpu()
        for i, k in enumerate(keys):
            cnt = float(mom[i, 0])
            if cnt == 0:
                continue
            mean = float(mom[i, 1]) / cnt
            sd = math.sqrt(max(float(mom[i, 2]) / cnt - mean * mean, 0.0))
            bins = [f"{(j + int(lo)) * bw:g}{d}{c}" for j, c in enumerate(Hh[i].tolist()) if c]
            out.append(d.join(list(k) + [str(a), f"{bw:g}", str(int(cnt)), fmt(mean, prec), fmt(sd, prec)] + bins))
    ctx.emit_root(out)


def ks_from_distr(ctx: JobContext) -> None:
    """kolmogorovSmirnovModelDrift over histogram files (S/explore/KolmogorovSmirnovModelDrift.scala
    :57-76): lines of numericalAttrDistrStats, grouped by the first ``key.length`` fields; a key
    with exactly two histograms (reference, current) gets ``key..,ksStat,drifted`` with the critical
    value c * sqrt((n1+n2)/(n1 n2)), c = sqrt(-0.5 ln(significance.level))."""
    kl = ctx.get_int("key.length")
    sig = ctx.get_float("significance.level", 0.05)
    prec = ctx.get_int("output.precision", 3)
    c = math.sqrt(-0.5 * math.log(sig))
    groups = defaultdict(list)
    for r in ctx.rows(shard=False):
        groups[tuple(r[:kl])].append(r)
    d = ctx.delim_out
    out = []
    for k, hs in sorted(groups.items()):
        if len(hs) != 2:
            continue
        hists = []
        for r in hs:
            rest = r[kl:]
            tail = rest[4:]                      # binWidth count mean sd | bin cnt ...
            h = {float(tail[i]): float(tail[i + 1]) for i in range(0, len(tail), 2)}
            hists.append(h)
        bins = sorted(set(hists[0]) | set(hists[1]))
        a = torch.tensor([hists[0].get(b, 0.0) for b in bins], dtype=torch.float64)
        b = torch.tensor([hists[1].get(b, 0.0) for b in bins], dtype=torch.float64)
        n1, n2 = float(a.sum()), float(b.sum())
        ks = float((torch.cumsum(a, 0) / n1 - torch.cumsum(b, 0) / n2).abs().max())
        crit = c * math.sqrt((n1 + n2) / (n1 * n2))
        out.append(d.join(list(k) + [fmt(ks, prec), "true" if ks > crit else "false"]))
    ctx.emit_root(out)
