"""Markov / HMM / suffix-tree / sequence-mining / CTMC jobs (J/markov/*, J/sequence/*, S/markov/*,
S/sequence/*)."""
from __future__ import annotations

import math
from collections import defaultdict

import torch

from .common import JobContext, fmt, job


# ================================================================================================
# HMM estimation
# ================================================================================================
@job("hiddenMarkovModelBuilder", "supervised HMM estimation, fully or partially tagged (J/markov/HiddenMarkovModelBuilder.java, hmmb.*)")
def hmm_builder(args):
    """Fully tagged rows: ``id..,obs:state,obs:state,...`` after ``hmmb.skip.field.count`` fields.
    Partially tagged rows (``hmmb.partially.tagged``): state tokens embedded among the observations,
    emission weights spread left/right by ``hmmb.window.function`` (:174-260).  Counts of the three
    tables are all-reduced once; output: states, observations, S transition rows, S emission rows,
    the initial-state row (integer rows scaled by ``hmmb.trans.prob.scale``)."""
    from ..data.table import _literal
    from ..models.markov import HiddenMarkovModel, HiddenMarkovModelBuilder, normalize_rows
    ctx = JobContext(args, "hmmb.")
    states = ctx.get_list("model.states")
    observations = ctx.get_list("model.observations")
    scale = ctx.get_int("trans.prob.scale", 1000)
    b = HiddenMarkovModelBuilder(states, observations, comm=ctx.comm)
    lit = _literal(ctx.delim_in)
    native = lit is not None and len(lit) == 1
    if ctx.get_bool("partially.tagged", False):
        win = ctx.get_int_list("window.function")
        if native:   # every field of the row, states and observations by dictionary lookup
            rec = ctx.records()
            trans, emit, init = b.partially_tagged_counts_tokens(
                rec.off, rec.map_codes(rec.codes, states), rec.map_codes(rec.codes, observations), win)
        else:
            trans, emit, init = b.partially_tagged_counts(ctx.rows(), win)
    else:
        skip = ctx.get_int("skip.field.count", 0)
        sub = ctx.get_str("sub.field.delim", ":")
        if native and len(sub) == 1:
            # obs:state tokens split natively (code, sub code); rows with >= 2 tagged tokens
            rec = ctx.records(modes="x" * skip, sub_delim=sub)
            st_tok = (rec.map_codes(rec.sub, states) if rec.sub is not None
                      else torch.full_like(rec.codes, -1))
            obs, n = rec.padded(rec.map_codes(rec.codes, observations), start=skip)
            st, _ = rec.padded(st_tok, start=skip)
            keep = n >= 2
            if not bool(keep.all()):
                obs, st = obs[keep], st[keep]
        else:
            tagged = [r[skip:] for r in ctx.rows() if len(r) >= skip + 2]
            obs, st = b.encode(tagged, sub)
        trans, emit, init = b.counts(obs, st)
    ctx.all_reduce(trans, emit, init)
    A = normalize_rows(trans, scale)
    B = normalize_rows(emit, scale)
    pi = normalize_rows(init.view(1, -1), scale)[0]
    hmm = HiddenMarkovModel(states, observations, A.double(), B.double(), pi.double())
    d = ctx.delim_out
    ctx.emit_root([d.join(states), d.join(observations)] + [d.join(str(int(x)) for x in row) for row in A.cpu()]
                  + [d.join(str(int(x)) for x in row) for row in B.cpu()] + [d.join(str(int(x)) for x in pi.cpu())])
    return hmm


# ================================================================================================
# Markov chain classification
# ================================================================================================
@job("markovModelClassifier", "two-class Markov chain log-odds classifier (J/markov/MarkovModelClassifier.java, mmc.*)")
def mmc(args):
    """Rows ``id,[class],s1,s2,...``; log-odds = sum log(P_c0(s->s') / P_c1(s->s')) over the row
    with the class-conditional transition tables of ``mmc.mm.model.path`` (K15 gather-sum kernel,
    one thread per row); ``id,[actual],pred,logOdds`` per row (:127-150)."""
    from ..models.markov import MarkovModelClassifier, MarkovStateTransitionModel
    ctx = JobContext(args, "mmc.")
    states, mats = MarkovStateTransitionModel.load_matrices(ctx.path("mm.model.path", "model"), ",")
    labels = ctx.get_list("class.labels")
    skip = ctx.get_int("skip.field.count", 1)
    id_ord = ctx.get_int("id.field.ord", 0)
    val = ctx.get_bool("validation.mode", False)
    cls_ord = ctx.get_int("class.label.field.ord", -1)
    thr = ctx.get_float("log.odds.threshold", 0.0)
    clf = MarkovModelClassifier(mats[labels[0]], mats[labels[1]], labels, thr)
    rows = [r for r in ctx.rows() if len(r) >= skip + 2]
    si = {s: i for i, s in enumerate(states)}
    L = max([len(r) - skip for r in rows] + [1])
    X = torch.full((len(rows), L), -1, dtype=torch.int16)
    for i, r in enumerate(rows):
        toks = [v for j, v in enumerate(r[skip:], skip) if j != cls_ord] if cls_ord >= skip else r[skip:]
        X[i, : len(toks)] = torch.tensor([si.get(v, -1) for v in toks], dtype=torch.int16)
    lo = clf.log_odds(X.to(ctx.device)).double().cpu()
    d = ctx.delim_out
    out = []
    for r, v in zip(rows, lo.tolist()):
        pred = labels[0] if v > thr else labels[1]
        parts = [r[id_ord]] + ([r[cls_ord]] if val else []) + [pred, repr(v)]
        out.append(d.join(parts))
    ctx.emit(out)


# ================================================================================================
# probabilistic suffix tree counts
# ================================================================================================
@job("probabilisticSuffixTreeGenerator", "counts of all sub-sequences of length 2..L per partition/class (J/markov/ProbabilisticSuffixTreeGenerator.java, pstg.*)")
def pstg(args):
    """Each row's tokens (after ``pstg.skip.field.count``) are mapped to a shared vocabulary; every
    window of width 2..``pstg.max.seq.length`` is one row of an int64 key tensor (prefix id x
    token digits), counted by a device sort + unique; counts are merged across ranks; one line per
    distinct n-gram ``ids..,[class],tok..,count`` plus the ``$`` root count per prefix (:140-305).
    ``pstg.input.format.sequential=false`` reads one token per record (field ``pstg.data.field.ordinal``)
    with a sliding window per id."""
    ctx = JobContext(args, "pstg.")
    skip = ctx.get_int("skip.field.count", 0)
    cls_ord = ctx.get_int("class.label.field.ord", -1)
    L = ctx.get_int("max.seq.length", 5)
    root = ctx.get_str("tree.root.symbol", "$")
    id_ords = ctx.get_int_list("id.field.ordinals", [])
    seqs: list[tuple[tuple, list[str]]] = []
    if ctx.get_bool("input.format.sequential", True):
        for r in ctx.rows():
            if len(r) < skip + 2:
                continue
            pref = tuple(r[o] for o in id_ords) + ((r[cls_ord],) if cls_ord >= 0 else ())
            seqs.append((pref, r[skip:]))
    else:
        # streaming windows per id: a window of the last L tokens emits prefixes of width 2..L
        dfo = ctx.get_int("data.field.ordinal")
        wins = defaultdict(list)
        for r in ctx.rows(shard=False):
            pref = tuple(r[o] for o in id_ords) + ((r[cls_ord],) if cls_ord >= 0 else ())
            w = wins[pref]
            w.append(r[dfo])
            if len(w) > L:
                w.pop(0)
            if len(w) == L:
                seqs.append((pref, list(w[:L]) + ["\x00stream"]))
    counts = ngram_counts(ctx, seqs, L, streaming=not ctx.get_bool("input.format.sequential", True))
    d = ctx.delim_out
    ctx.emit_root([d.join(list(k) + [str(c)]) for k, c in sorted(counts.items())] if ctx.is_root else [])


def ngram_counts(ctx: JobContext, seqs, L: int, streaming: bool = False) -> dict[tuple, int]:
    """{(prefix.., tok..): count} and {(prefix.., '$'): root count} for all windows of width 2..L."""
    vocab = ctx.union({t for _, s in seqs for t in s if t != "\x00stream"})
    prefs = ctx.union({p for p, _ in seqs})
    ti = {t: i + 1 for i, t in enumerate(vocab)}      # 0 = padding
    pi = {p: i for i, p in enumerate(prefs)}
    V = len(vocab) + 1
    out: dict[tuple, int] = {}
    if not seqs:
        seqs = []
    maxlen = max([len(s) for _, s in seqs] + [2])
    T = torch.zeros((len(seqs), maxlen), dtype=torch.long)
    P = torch.tensor([pi[p] for p, _ in seqs], dtype=torch.long)
    for i, (_, s) in enumerate(seqs):
        toks = [ti[t] for t in s if t != "\x00stream"]
        T[i, : len(toks)] = torch.tensor(toks, dtype=torch.long)
    T = T.to(ctx.device)
    P = P.to(ctx.device)
    root = torch.zeros(len(prefs), dtype=torch.long, device=ctx.device)
    digits = max(1, math.ceil(math.log2(V + 1)))
    for w in range(2, L + 1):
        if T.shape[1] < w or T.shape[0] == 0:
            keys, cnt = torch.zeros(0, dtype=torch.long), torch.zeros(0, dtype=torch.long)
        else:
            win = T.unfold(1, w, 1)                                   # [n, nw, w]
            if streaming:
                win = win[:, :1]                                     # one prefix window per stream step
            ok = (win > 0).all(-1)
            key = P.view(-1, 1).expand_as(ok)
            for j in range(w):
                key = key * (1 << digits) + win[..., j]
            keys, cnt = torch.unique(key[ok], return_counts=True)
            root.index_add_(0, P.view(-1, 1).expand_as(ok)[ok], torch.ones_like(key[ok]))
        if ctx.comm.is_distributed:
            ks = ctx.comm.all_gather_v(keys.cpu())
            cs = ctx.comm.all_gather_v(cnt.cpu())
            keys, inv = torch.unique(ks, return_inverse=True)
            cnt = torch.zeros_like(keys).index_add_(0, inv, cs)
        for k, c in zip(keys.cpu().tolist(), cnt.cpu().tolist()):
            toks = []
            for _ in range(w):
                toks.append(vocab[(k & ((1 << digits) - 1)) - 1])
                k >>= digits
            out[tuple(prefs[k]) + tuple(reversed(toks))] = c
    ctx.all_reduce(root)
    for p, c in zip(prefs, root.cpu().tolist()):
        if c:
            out[tuple(p) + ("$",)] = c
    return out


# ================================================================================================
# GSP candidate generation / positional clusters
# ================================================================================================
@job("candidateGenerationWithSelfJoin", "GSP k+1 candidate sequences by self-join on the (k-1)-overlap (J/sequence/CandidateGenerationWithSelfJoin.java, cgs.*)")
def cgs(args):
    """Rows hold a frequent k-sequence in their first ``cgs.item.set.length`` fields.  The join is
    the device op of ``ops/sequence_ops.gsp_join`` (sort of the (k-1)-prefix ids + segmented
    expansion kernel, K18); with several ranks each joins its shard of left sequences against the
    full (all-gathered) right set, and the candidates are gathered to rank 0.  Every ordered pair
    (a, b) with a[1:] == b[:-1] yields a + b[-1] (incl. a == b), which fixes two reference bugs
    (pairs inside one hash bucket are never joined; the reverse join appends a token of the wrong
    sequence, :243-276)."""
    from ..models.markov import gsp_candidates_device
    ctx = JobContext(args, "cgs.")
    k = ctx.get_int("item.set.length")
    seqs = [tuple(r[:k]) for r in ctx.rows(shard=False) if len(r) >= k]
    cands = gsp_candidates_device(seqs, device=ctx.device, comm=ctx.comm)
    d = ctx.delim_out
    ctx.emit_root([d.join(c) for c in cands])


@job("sequencePositionalCluster", "time-bounded event locality score over a sliding window (J/sequence/SequencePositionalCluster.java)")
def spc(args):
    """Rows carry a quantity (``quant.field.ordinal``) and a time stamp (``seq.num..field.ordinal``);
    a record meets the condition ``cond.expression`` (predicates on the quantity, ``$0`` or the
    field ordinal as operand, joined by ' and '); the locality score of a record is the fraction of
    condition-meeting events among the events in the trailing ``window.time.span`` (hoidla's
    analyzer is outside the reference tree: score definition documented, parity unpinned); records
    with score > ``score.threshold`` are written as ``seq,quant,score``."""
    ctx = JobContext(args, "")
    from ..utils.rules import RuleExpression
    q = ctx.get_int("quant.field.ordinal")
    so = ctx.get_int("seq.num..field.ordinal", None)
    so = ctx.get_int("seq.num.field.ordinal") if so is None else so
    span = ctx.get_float("window.time.span")
    thr = ctx.get_float("score.threshold")
    expr = ctx.get_str("cond.expression").replace("$0", str(q))
    rule = RuleExpression.from_condition(expr)
    rows = ctx.rows(shard=False)
    t = torch.tensor([float(r[so]) for r in rows], dtype=torch.float64)
    met = rule.evaluate_rows(rows).double()
    order = torch.argsort(t, stable=True)
    ts, ms = t[order], met[order]
    cm = torch.cumsum(ms, 0)
    lo = torch.searchsorted(ts, ts - span, right=False)
    idx = torch.arange(len(ts))
    n_in = (idx - lo + 1).double()
    met_in = cm - torch.where(lo > 0, cm[(lo - 1).clamp_min(0)], torch.zeros_like(cm))
    score = torch.zeros_like(t)
    score[order] = met_in / n_in
    d = ctx.delim_out
    ctx.emit_root([f"{r[so]}{d}{r[q]}{d}{fmt(s)}" for r, s in zip(rows, score.tolist()) if s > thr])


# ================================================================================================
# continuous-time Markov chains
# ================================================================================================
_MS = {"week": 7 * 86400_000, "day": 86400_000, "hour": 3600_000, "minute": 60_000, "sec": 1000}


@job("stateTransitionRate", "CTMC rate matrix per key from time-stamped states (S/markov/StateTransitionRate.scala)")
def state_transition_rate(args):
    """``(key,q00,q01,...)`` per key; transition counts and dwell times of all keys come from one
    segmented pass (sort by (key, time), bigram + dwell scatter-add over ``[G, S, S]``)."""
    from ..models.markov import StateTransitionRate
    ctx = JobContext(args, app="stateTransitionRate")
    kords = ctx.get_int_list("key.field.ordinals")
    to, so = ctx.get_int("time.field.ordinal"), ctx.get_int("state.field.ordinal")
    states = ctx.get_list("state.values")
    unit = ctx.get_str("rate.time.unit", "hour")
    in_unit = ctx.get_str("input.time.unit", "ms")
    prec = ctx.get_int("trans.rate.output.precision", 6)
    from ..data.table import _literal
    lit = _literal(ctx.delim_in)
    if lit is not None and len(lit) == 1 and 1 <= len(kords) <= 2 and to not in kords and so not in kords:
        return _state_transition_rate_native(ctx, kords, to, so, states, unit, in_unit, prec)
    rows = ctx.rows(shard=False)
    keys = sorted({tuple(r[o] for o in kords) for r in rows})
    ki = {k: i for i, k in enumerate(keys)}
    si = {s: i for i, s in enumerate(states)}
    ent = torch.tensor([ki[tuple(r[o] for o in kords)] for r in rows])
    mult = 1000 if in_unit == "sec" else 1
    tm = torch.tensor([int(float(r[to])) * mult for r in rows], dtype=torch.long)
    st = torch.tensor([si[r[so]] for r in rows])
    Q = StateTransitionRate(len(states)).fit_grouped(ent, tm, st, len(keys), _MS[unit])
    d = ctx.delim_out
    out = []
    for i, k in enumerate(keys):
        out.append("(" + d.join(list(k) + [f"{v:.{prec}f}" for v in Q[i].reshape(-1).tolist()]) + ")")
    ctx.emit_root(out)


def _state_transition_rate_native(ctx, kords, to, so, states, unit, in_unit, prec):
    """stateTransitionRate on the native record table: events shuffled to the rank owning their
    key (keys in string order, contiguous blocks per rank), then one segmented device pass per
    rank (StateTransitionRate.fit_grouped) and the native formatter for ``(key,q00,q01,...)``."""
    import numpy as np
    from ..data.records import format_lines, owner_of, shuffle
    from ..data.table import shard_range
    from ..models.markov import StateTransitionRate
    comm = ctx.comm
    top = max(list(kords) + [to, so]) + 1
    modes = "".join("n" if i == to else ("d" if (i in kords or i == so) else "x") for i in range(top))
    rec = ctx.records(modes=modes, tail_mode="x", numeric=True)
    dev = rec.device
    V = max(1, len(rec.vocab))
    kc = [rec.field(o).long() for o in kords]
    tm_raw = rec.field(to, numeric=True)
    st = rec.map_codes(rec.field(so), states).long()
    ok = (st >= 0) & ~torch.isnan(tm_raw)
    for c in kc:
        ok &= c >= 0
    comp = kc[0] if len(kc) == 1 else kc[0] * V + kc[1]
    comp, st = comp[ok], st[ok]
    mult = 1000 if in_unit == "sec" else 1
    tm = torch.trunc(tm_raw[ok]).long() * mult
    if len(kc) == 1:
        return _str_single_key(ctx, rec, comp, tm, st, states, unit, prec)
    # global key set in string-tuple order
    loc = torch.unique(comp)
    allk = comm.all_gather_v(loc) if comm.is_distributed else loc
    allk = torch.unique(allk).cpu()
    parts = [allk] if len(kc) == 1 else [allk // V, allk % V]
    strs = [np.array([rec.vocab[i] for i in p.tolist()]) for p in parts]
    order = (np.lexsort(tuple(reversed(strs))) if allk.numel() else np.zeros(0, np.int64)).astype(np.int64)
    order_t = torch.from_numpy(order)
    G = allk.numel()
    rank_of = torch.empty(G, dtype=torch.long)
    rank_of[order_t] = torch.arange(G)
    kpos = rank_of.to(dev)[torch.searchsorted(allk.to(dev), comp)] if comp.numel() else comp
    owner = owner_of(kpos, G, comm.world) if comm.is_distributed else torch.zeros_like(kpos)
    kpos, tm, st = shuffle(comm, owner, [kpos, tm, st])
    a, b = shard_range(G, comm.rank, comm.world) if comm.is_distributed else (0, G)
    Q = StateTransitionRate(len(states)).fit_grouped(kpos - a, tm, st, b - a, _MS[unit])
    skeys = allk[order_t][a:b]
    key_parts = [skeys] if len(kc) == 1 else [skeys // V, skeys % V]
    cols = [("g", "(")] + [("s", rec.vocab, p.int()) for p in key_parts]
    Qc = Q.reshape(b - a, -1).double().cpu()
    cols += [("f", Qc[:, j].contiguous(), prec) for j in range(Qc.shape[1])] + [("g", ")")]
    ctx.emit_text(format_lines(cols, b - a, ctx.delim_out))


def _str_single_key(ctx, rec, key, tm, st, states, unit, prec):
    """One key field: keys in string order by the device packed-key sort (data/records.sorted_keys)."""
    from ..data.records import format_lines, owner_of, shuffle, sorted_keys
    from ..data.table import shard_range
    from ..models.markov import StateTransitionRate
    comm = ctx.comm
    keys, pos = sorted_keys(rec, key, comm)
    G = keys.numel()
    kpos = pos[key]
    owner = owner_of(kpos, G, comm.world) if comm.is_distributed else torch.zeros_like(kpos)
    kpos, tm, st = shuffle(comm, owner, [kpos, tm, st])
    a, b = shard_range(G, comm.rank, comm.world) if comm.is_distributed else (0, G)
    Q = StateTransitionRate(len(states)).fit_grouped(kpos - a, tm, st, b - a, _MS[unit])
    Qc = Q.reshape(b - a, -1).double().cpu()
    cols = [("g", "("), ("s", rec.vocab, keys[a:b].int().cpu())]
    cols += [("f", Qc[:, j].contiguous(), prec) for j in range(Qc.shape[1])] + [("g", ")")]
    ctx.emit_text(format_lines(cols, b - a, ctx.delim_out))


@job("contTimeStateTransitionStats", "CTMC statistics by uniformisation: stateDwellTime | StateTransitionCount | futureStateProb (S/markov/ContTimeStateTransitionStats.scala)")
def cont_time_stats(args):
    """Rate matrices from ``state.trans.file.path`` (stateTransitionRate output); input rows
    ``key..,initState[,endState]``; the matrix-power chains of all keys are one batched device
    launch (K16).  Output ``(key,stat)``.  The reference's stateDwellTime weights ``t/(i+1)`` per
    Poisson term; here the exact uniformisation integral (tail-probability weights / lambda) is
    used for dwell time, and ``StateTransitionCount`` is dwell-time(i) x q_ij."""
    from ..models.markov import ContTimeStateTransitionStats
    ctx = JobContext(args, app="contTimeStateTransitionStats")
    kl = ctx.get_int("key.field.len")
    states = ctx.get_list("state.values")
    S = len(states)
    horizon = ctx.get_float("time.horizon")
    stat = ctx.get_str("state.trans.stat")
    targets = ctx.get_list("target.states", None)
    d = ctx.delim_out
    rates = {}
    for l in ctx.all_lines(ctx.path("state.trans.file.path")):
        p = l.strip()[1:-1].split(d)
        rates[tuple(p[:kl])] = torch.tensor([float(x) for x in p[kl:kl + S * S]], dtype=torch.float64).view(S, S)
    si = {s: i for i, s in enumerate(states)}
    out = []
    cache = {}
    for r in ctx.rows():
        key = tuple(r[:kl])
        if key not in cache:
            cs = ContTimeStateTransitionStats(rates[key].to(ctx.device))
            A, B = cs.sums([horizon])
            cache[key] = (cs, A[0].cpu(), B[0].cpu())
        cs, P, Dw = cache[key]
        i0 = si[r[kl]]
        end = si[r[kl + 1]] if len(r) > kl + 1 and r[kl + 1] else -1
        if stat == "futureStateProb":
            if end < 0:
                raise SystemExit("futureStateProb needs an end state")
            v = float(P[i0, end])
        elif stat == "stateDwellTime":
            v = float(Dw[i0, si[targets[0]]])
        elif stat == "StateTransitionCount":
            a, b = si[targets[0]], si[targets[1]]
            v = float(Dw[i0, a]) * float(cs.Q[a, b])
        else:
            raise SystemExit(f"invalid state transition stats {stat}")
        out.append("(" + d.join(list(key) + [repr(v)]) + ")")
    ctx.emit(out)


# ================================================================================================
# sequence analytics
# ================================================================================================
@job("dotMatrixMatching", "all-pairs dot-matrix window-match similarity of sequences (S/sequence/DotMatrixMatching.scala)")
def dot_matrix(args):
    """Rows ``id,tok,tok,...``; every pair (i < j) gets the window-match score of the K dot-matrix
    kernel (sequences vs sequences, no bucket-pair replication); output ``id1,id2,score``."""
    from ..models.markov import dot_matrix_similarity
    ctx = JobContext(args, app="dotMatrixMatching")
    skip = ctx.get_int("skip.field.count", 1)
    w = ctx.get_int("window.size", 3)
    prec = ctx.get_int("output.precision", 3)
    rows = ctx.rows(shard=False)
    vocab = {}
    L = max([len(r) - skip for r in rows] + [w])
    X = torch.full((len(rows), L), -1, dtype=torch.long)
    for i, r in enumerate(rows):
        X[i, : len(r) - skip] = torch.tensor([vocab.setdefault(t, len(vocab)) for t in r[skip:]], dtype=torch.long)
    # each rank scores its block of query rows against all rows
    from ..data.table import shard_range
    a, b = shard_range(len(rows), ctx.comm.rank, ctx.comm.world)
    Sm = dot_matrix_similarity(X[a:b].to(ctx.device), X.to(ctx.device), w).cpu()
    d = ctx.delim_out
    out = [f"{rows[a + i][0]}{d}{rows[j][0]}{d}{fmt(float(Sm[i, j]), prec)}"
           for i in range(b - a) for j in range(a + i + 1, len(rows))]
    ctx.emit(out)


@job("eventTimeDistribution", "per-key histogram of event hour-of-day / day-of-week (S/sequence/EventTimeDistribution.scala)")
def event_time(args):
    """Epoch-millisecond time stamps; ``hour.granularity`` bins hours; counts of all keys are one
    ``[G, B]`` scatter-add, all-reduced; output ``key..,bin:count,...``.  Day of week is
    ((t / day) + 4) mod 7 with 0 = Sunday (the reference divides by a week first, which maps every
    time stamp to bin 0)."""
    ctx = JobContext(args, app="eventTimeDistribution")
    kords = ctx.get_int_list("id.field.ordinals")
    to = ctx.get_int("time.field.ordinal")
    res = ctx.get_str("time.resolution", "hourOfDay")
    gr = ctx.get_int("hour.granularity", 1)
    rows = ctx.rows()
    keys = ctx.union(tuple(r[o] for o in kords) for r in rows)
    ki = {k: i for i, k in enumerate(keys)}
    t = torch.tensor([int(float(r[to])) for r in rows], dtype=torch.long)
    if res == "hourOfDay":
        b = (t % 86400_000) // 3600_000 // gr
        B = (24 + gr - 1) // gr
    else:
        b = ((t // 86400_000) + 4) % 7
        B = 7
    g = torch.tensor([ki[tuple(r[o] for o in kords)] for r in rows], dtype=torch.long)
    H = torch.zeros(len(keys) * B, dtype=torch.long).index_add_(0, g * B + b, torch.ones_like(b)).view(len(keys), B)
    ctx.all_reduce(H)
    d = ctx.delim_out
    ctx.emit_root([d.join(list(k) + [f"{j}:{int(c)}" for j, c in enumerate(H[i].tolist()) if c])
                   for i, k in enumerate(keys)])


@job("sequenceGenerator", "group records by key, ordered by a sequence field (S/sequence/SequenceGenerator.scala)")
def seq_gen(args):
    """Output ``key..,v..,v..,...`` (the value fields of every record of the key in sequence
    order); the ordering is the device segmented sort of ``models/markov.sequence_generator``."""
    from ..models.markov import sequence_generator
    ctx = JobContext(args, app="sequenceGenerator")
    kords = ctx.get_int_list("id.field.ordinals")
    vords = ctx.get_int_list("val.field.ordinals")
    sf = ctx.get_int("seq.field")
    rows = ctx.rows(shard=False)
    keys = sorted({tuple(r[o] for o in kords) for r in rows})
    ki = {k: i for i, k in enumerate(keys)}
    kk = torch.tensor([ki[tuple(r[o] for o in kords)] for r in rows])
    sv = torch.tensor([int(float(r[sf])) for r in rows])
    ks, order, starts = sequence_generator(kk, sv, torch.arange(len(rows)))
    d = ctx.delim_out
    bounds = starts.tolist() + [len(rows)]
    out = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        k = keys[int(ks[a])]
        vals = [v for i in order[a:b].tolist() for v in (rows[i][o] for o in vords)]
        out.append(d.join(list(k) + vals))
    from ..data.table import shard_range
    a, b = shard_range(len(out), ctx.comm.rank, ctx.comm.world)
    ctx.emit(out[a:b])


@job("timeDelayEmbeddingModel", "histogram of symbol windows per key (S/sequence/TimeDelayEmbeddingModel.scala, appName markovChainPredictor)",
     aliases=("markovChainPredictor",))
def time_delay(args):
    """Per key, records ordered by ``seq.fieldOrd``; every full window of ``window.size`` symbols of
    ``attr.ordinal`` is counted (device n-gram count); output ``key..,w1:w2:w3,count,...``."""
    ctx = JobContext(args, app="markovChainPredictor")
    kords = ctx.get_int_list("id.fieldOrdinals", [])
    ao = ctx.get_int("attr.ordinal")
    so = ctx.get_int("seq.fieldOrd")
    w = ctx.get_int("window.size", 3)
    g = defaultdict(list)
    for r in ctx.rows(shard=False):
        g[tuple(r[o] for o in kords)].append((float(r[so]), r[ao]))
    seqs = [(k, [s for _, s in sorted(v)]) for k, v in sorted(g.items())]
    if ctx.comm.is_distributed:
        from ..data.table import shard_range
        a, b = shard_range(len(seqs), ctx.comm.rank, ctx.comm.world)
        seqs = seqs[a:b]
    d = ctx.delim_out
    out = []
    for k, s in seqs:
        c: dict[str, int] = defaultdict(int)
        if len(s) >= w:
            vocab = {t: i for i, t in enumerate(sorted(set(s)))}
            inv = sorted(vocab, key=vocab.get)
            T = torch.tensor([vocab[t] for t in s], dtype=torch.long, device=ctx.device)
            win = T.unfold(0, w, 1)
            key = torch.zeros(win.shape[0], dtype=torch.long, device=ctx.device)
            for j in range(w):
                key = key * len(vocab) + win[:, j]
            u, cnt = torch.unique(key, return_counts=True)
            for kk, cc in zip(u.cpu().tolist(), cnt.cpu().tolist()):
                toks = []
                for _ in range(w):
                    toks.append(inv[kk % len(vocab)])
                    kk //= len(vocab)
                c[":".join(reversed(toks))] = cc
        out.append(d.join(list(k) + [f"{x}{d}{c[x]}" for x in sorted(c)]))
    ctx.emit(out)
