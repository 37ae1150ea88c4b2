"""Markov / HMM / suffix-tree / sequence-mining / CTMC jobs (J/markov/*, J/sequence/*, S/markov/*,
S/sequence/*)."""
from __future__ import annotations

import math
from collections import defaultdict

import torch
from ..ops.encode_ops import unique_rows

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
    from ..data.table import _literal
    lit = _literal(ctx.delim_in)
    if lit is None or len(lit) != 1:
        return _mmc_rows(ctx, clf, states, labels, skip, id_ord, val, cls_ord, thr)
    from ..data.records import format_lines
    # native path: state tokens by dictionary lookup, the padded [N, L] state matrix on the device
    # (class field dropped when it sits among the states), the K15 gather-sum kernel, and the
    # output from the raw id / class fields and the device results
    rec = ctx.records(modes="x" * skip)
    keep = rec.lens() >= skip + 2
    X, _ = rec.padded(rec.map_codes(rec.codes, states), start=skip, drop=(cls_ord,) if cls_ord >= skip else (),
                      min_len=1)
    X = X[keep]
    lo = clf.log_odds(X.to(ctx.device)).double()
    pred = (lo <= thr).int()             # 0 -> labels[0] (log-odds above the threshold)
    spans = rec.line_spans().select(keep.cpu())
    cols = [spans.column("rf", id_ord, lit)]
    if val:
        cols.append(spans.column("rf", cls_ord, lit))
    cols += [("s", list(labels[:2]), pred), ("f", lo, -2)]     # device repr when the lines have a device twin
    ctx.emit_columns(cols, int(keep.sum()))


def _mmc_rows(ctx, clf, states, labels, skip, id_ord, val, cls_ord, thr):
    """Regex delimiters: the split-row path."""
    rows = [r for r in ctx.rows() if len(r) >= skip + 2]
    si = {s: i for i, s in enumerate(states)}
    toks = [[v for j, v in enumerate(r[skip:], skip) if j != cls_ord] if cls_ord >= skip else r[skip:] for r in rows]
    L = max([len(t) for t in toks] + [1])
    X = torch.tensor([[si.get(v, -1) for v in t] + [-1] * (L - len(t)) for t in toks], dtype=torch.int16).view(-1, L)
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
    """Counts of every window of width 2..``pstg.max.seq.length`` of the token fields, per prefix
    (``pstg.id.field.ordinals`` fields + the ``pstg.class.label.field.ord`` label), plus the
    ``<root symbol>`` count per prefix (the number of windows), one line each:
    ``ids..,[class],tok..,count`` in key order (:140-305).  As in the reference the class field adds
    one to ``pstg.skip.field.count`` (:118-122).  ``pstg.input.format.sequential=false`` reads one
    token per record (``pstg.data.field.ordinal``) and slides a window of the last L tokens per
    prefix over the records in input order.

    Native path (one-character delimiter): the rank's byte range is tokenized once; the K5 hash
    count kernel (``ops/sequence_ops.ngram_counts``, LDS-privatised open addressing) counts all
    widths of all rows in one pass with the prefix as the group id; the decoded (prefix, n-gram,
    count) rows of all ranks are merged on rank 0, ordered by string ranks and formatted natively."""
    from ..data.table import _literal
    ctx = JobContext(args, "pstg.")
    skip = ctx.get_int("skip.field.count", 0)
    cls_ord = ctx.get_int("class.label.field.ord", -1)
    if cls_ord >= 0:
        skip += 1
    L = ctx.get_int("max.seq.length", 5)
    root = ctx.get_str("tree.root.symbol", "$")
    id_ords = ctx.get_int_list("id.field.ordinals", [])
    pref_ords = list(id_ords) + ([cls_ord] if cls_ord >= 0 else [])
    sequential = ctx.get_bool("input.format.sequential", True)
    lit = _literal(ctx.delim_in)
    if lit is None or len(lit) != 1:
        return _pstg_rows(ctx, skip, cls_ord, L, root, id_ords, sequential)
    if sequential:
        rec = ctx.records(modes="".join("d" if i in pref_ords else "x" for i in range(skip)))
        keep = rec.lens() >= skip + 2
        T, _ = rec.padded(start=skip, dtype=torch.int32)
        T = T[keep]
        P = (torch.stack([rec.field(o) for o in pref_ords], 1)[keep] if pref_ords
             else torch.zeros((T.shape[0], 0), dtype=torch.int32, device=T.device))
    else:
        dfo = ctx.get_int("data.field.ordinal")
        top = max(pref_ords + [dfo]) + 1
        rec = ctx.records(modes="".join("d" if (i in pref_ords or i == dfo) else "x" for i in range(top)),
                          tail_mode="x")
        T, P = _stream_windows(ctx, rec, pref_ords, dfo, L)
    rows = _ngram_rows(T, P, L, streaming=not sequential)
    _emit_pst(ctx, rec, rows, len(pref_ords), L, root)


def _stream_windows(ctx, rec, pref_ords, dfo, L):
    """Non-sequential input: every record adds its token to the window of its prefix; each full
    window (the last L tokens) is one row of ``T`` [W, L] whose prefixes of width 2..L are
    counted.  Records are shuffled to the rank owning their prefix (all-to-all, input order kept:
    rows arrive in source-rank order, each source's rows in file order), then grouped by a stable
    sort on the device."""
    from ..data.records import segment_rank, shuffle
    dev = rec.device
    tok = rec.field(dfo).long()
    P = (torch.stack([rec.field(o) for o in pref_ords], 1).long() if pref_ords
         else torch.zeros((rec.n_lines, 0), dtype=torch.long, device=dev))
    ok = (tok >= 0) & ((P >= 0).all(1) if pref_ords else torch.ones_like(tok, dtype=torch.bool))
    tok, P = tok[ok], P[ok]
    comm = ctx.comm
    if comm.is_distributed:
        h = torch.zeros_like(tok)
        for j in range(P.shape[1]):
            h = (h * 1000003 + P[:, j]) % (1 << 40)
        cols = shuffle(comm, h % comm.world, [tok] + [P[:, j] for j in range(P.shape[1])])
        tok = cols[0]
        P = torch.stack(cols[1:], 1) if P.shape[1] else torch.zeros((tok.numel(), 0), dtype=torch.long, device=dev)
    if tok.numel() == 0:
        return torch.zeros((0, L), dtype=torch.int32, device=dev), P[:0]
    if P.shape[1]:
        _, g = unique_rows(P, True)
    else:
        g = torch.zeros_like(tok)
    order = torch.argsort(g, stable=True)
    gs, ts = g[order], tok[order]
    first = torch.ones_like(gs, dtype=torch.bool)
    first[1:] = gs[1:] != gs[:-1]
    pos = segment_rank(first)
    n_g = torch.bincount(gs)
    # a window is complete at every record with pos >= L - 1; it starts at that record - (L - 1)
    end = torch.nonzero(pos >= L - 1).view(-1)
    start = end - (L - 1)
    T = ts[start.view(-1, 1) + torch.arange(L, device=dev).view(1, -1)].int()
    Pw = P[order][start].int()
    del n_g
    return T, Pw


def _ngram_rows(T: torch.Tensor, P: torch.Tensor, L: int, streaming: bool) -> torch.Tensor:
    """int64 [U, k + L + 2] rows ``prefix codes.., token codes.. (-1 padded), is_root, count`` of
    this rank: the windows of width 2..L of every row of ``T`` (dictionary codes, -1 padding;
    with ``streaming`` only the windows starting at column 0) counted per prefix row of ``P``."""
    from ..ops import sequence_ops as SO
    dev = T.device
    k = P.shape[1]
    N = T.shape[0]
    empty = torch.zeros((0, k + L + 2), dtype=torch.long, device=dev)
    if N == 0:
        return empty
    valid = T >= 0
    uv = torch.unique(T[valid])                          # the token codes in use -> dense 0..S-1
    S = uv.numel()
    dense = torch.where(valid, torch.searchsorted(uv, T.clamp_min(0)), torch.full_like(T, -1)).int()
    if k:
        gk, ginv = unique_rows(P.long(), True)
    else:
        gk, ginv = torch.zeros((1, 0), dtype=torch.long, device=dev), torch.zeros(N, dtype=torch.long, device=dev)
    base = S + 1
    out = []
    if streaming:
        counts = {}
        for w in range(2, min(L, T.shape[1]) + 1):
            win = dense[:, :w].long()
            okw = (win >= 0).all(1)
            key = ginv.clone()
            for j in range(w):
                key = key * base + win[:, j].clamp_min(0)
            keys, cnt = torch.unique(key[okw], return_counts=True)
            counts[w] = (keys % (base ** w), keys // (base ** w), cnt)
    else:
        gmul = base ** L
        if gmul * max(1, gk.shape[0]) >= (1 << 58):
            raise SystemExit("probabilisticSuffixTreeGenerator: (tokens + 1)^max.seq.length x prefixes exceeds the "
                             "2^58 n-gram key space")
        res = SO.ngram_counts(dense, S, 2, L, group=ginv if k else None)
        counts = {w: (kk % gmul, kk // gmul, cc) for w, (kk, cc) in res.items()}
    for w, (packed, grp, cnt) in counts.items():
        toks = torch.full((packed.numel(), L), -1, dtype=torch.long, device=dev)
        rem = packed.clone()
        for j in range(w - 1, -1, -1):
            toks[:, j] = uv[(rem % base)]
            rem = rem // base
        out.append(torch.cat([gk[grp], toks, torch.zeros_like(cnt).view(-1, 1), cnt.long().view(-1, 1)], 1))
    if not out:
        return empty
    rows = torch.cat(out, 0)
    # the root line of every prefix: the number of its windows
    g_all = torch.cat([grp for _, grp, _ in counts.values()])
    c_all = torch.cat([cnt.long() for _, _, cnt in counts.values()])
    rc = torch.zeros(gk.shape[0], dtype=torch.long, device=dev).index_add_(0, g_all, c_all)
    live = rc > 0
    rroot = torch.cat([gk[live], torch.full((int(live.sum()), L), -1, dtype=torch.long, device=dev),
                       torch.ones((int(live.sum()), 1), dtype=torch.long, device=dev), rc[live].view(-1, 1)], 1)
    return torch.cat([rows, rroot], 0)


def _emit_pst(ctx, rec, rows: torch.Tensor, k: int, L: int, root: str) -> None:
    """Merge every rank's (prefix, n-gram, count) rows on rank 0 (sum per distinct key), order them
    as the reference's sorted Tuple keys (string order field by field, a shorter key first, the
    root symbol compared as a string) and write them with the native formatter."""
    import bisect

    import numpy as np
    from ..data.records import format_lines, sorted_keys
    comm = ctx.comm
    if comm.is_distributed:
        dev = comm.device if comm.backend == "nccl" else torch.device("cpu")
        rows = comm.all_gather_v(rows.to(dev))
    if not ctx.is_root:
        return
    rows = rows.cpu()
    if rows.numel() == 0:
        ctx.emit_root_text(b"")
        return
    key, inv = unique_rows(rows[:, :-1], True)
    cnt = torch.zeros(key.shape[0], dtype=torch.long).index_add_(0, inv, rows[:, -1])
    codes = key[:, : k + L]
    is_root = key[:, k + L].bool()
    used = torch.unique(codes[codes >= 0])
    keys_sorted, pos = sorted_keys(rec, used.to(rec.device) if rec.device.type != "cpu" else used)
    keys_sorted, pos = keys_sorted.cpu(), pos.cpu()
    vocab = rec.vocab
    # rank of the root symbol among the used strings (it only meets tokens, at the first token slot)
    nless = bisect.bisect_left(range(keys_sorted.numel()), root, key=lambda i: vocab[int(keys_sorted[i])])
    rk = torch.where(codes >= 0, 2 * pos[codes.clamp_min(0)] + 2, torch.zeros_like(codes))
    rk[is_root, k] = 2 * nless + 1
    order = np.lexsort(tuple(rk[:, j].numpy() for j in range(k + L - 1, -1, -1)))
    order = torch.from_numpy(order.astype(np.int64))
    codes, is_root, cnt = codes[order], is_root[order], cnt[order]
    # compact string table of the used codes (+ the root symbol)
    tab = [vocab[int(c)] for c in keys_sorted.tolist()] + [root]
    lut = torch.full((len(vocab) + 1,), -1, dtype=torch.int32)
    lut[keys_sorted] = torch.arange(keys_sorted.numel(), dtype=torch.int32)
    ci = torch.where(codes >= 0, lut[codes.clamp_min(0)], torch.full_like(codes, -1, dtype=torch.int32).int()).int()
    tk = ci[:, k:].clone()
    tk[is_root, 0] = len(tab) - 1
    n_tok = (tk >= 0).sum(1)
    off = torch.cat([torch.zeros(1, dtype=torch.long), torch.cumsum(n_tok, 0)])
    cols = [("s", tab, ci[:, j].contiguous()) for j in range(k)]
    cols += [("l", tab, tk[tk >= 0].contiguous(), off), ("i", cnt)]
    ctx.emit_root_columns(cols, int(cnt.numel()))


def _pstg_rows(ctx, skip, cls_ord, L, root, id_ords, sequential):
    """Regex delimiters: split rows, then the same counting as the native path."""
    seqs: list[tuple[tuple, list[str]]] = []
    if sequential:
        for r in ctx.rows():
            if len(r) < skip + 2:
                continue
            pref = tuple(r[o] for o in id_ords) + ((r[cls_ord],) if cls_ord >= 0 else ())
            seqs.append((pref, r[skip:]))
    else:
        dfo = ctx.get_int("data.field.ordinal")
        wins = defaultdict(list)
        for r in ctx.rows(shard=False):
            pref = tuple(r[o] for o in id_ords) + ((r[cls_ord],) if cls_ord >= 0 else ())
            w = wins[pref]
            w.append(r[dfo])
            if len(w) > L:
                w.pop(0)
            if len(w) == L:
                seqs.append((pref, list(w)))
        if ctx.comm.rank != 0:
            seqs = []
    counts = ngram_counts(ctx, seqs, L, streaming=not sequential, root=root)
    d = ctx.delim_out
    ctx.emit_root([d.join(list(k) + [str(c)]) for k, c in sorted(counts.items())] if ctx.is_root else [])


def ngram_counts(ctx: JobContext, seqs, L: int, streaming: bool = False, root: str = "$") -> dict[tuple, int]:
    """{(prefix.., tok..): count} and {(prefix.., root): root count} for all windows of width 2..L
    (split-row path; ``streaming``: only the windows at the start of each row)."""
    vocab = ctx.union({t for _, s in seqs for t in s})
    prefs = ctx.union({p for p, _ in seqs})
    ti = {t: i for i, t in enumerate(vocab)}
    pi = {p: i for i, p in enumerate(prefs)}
    out: dict[tuple, int] = {}
    maxlen = max([len(s) for _, s in seqs] + [2])
    T = torch.tensor([[ti[t] for t in s] + [-1] * (maxlen - len(s)) for _, s in seqs], dtype=torch.int32)
    T = T.view(len(seqs), maxlen)
    P = torch.tensor([pi[p] for p, _ in seqs], dtype=torch.int32).view(-1, 1)
    rows = _ngram_rows(T.to(ctx.device), P.to(ctx.device), L, streaming)
    if ctx.comm.is_distributed:
        dev = ctx.comm.device if ctx.comm.backend == "nccl" else torch.device("cpu")
        rows = ctx.comm.all_gather_v(rows.to(dev))
    for r in rows.cpu().tolist():
        key = prefs[r[0]] + ((root,) if r[1 + L] else tuple(vocab[t] for t in r[1:1 + L] if t >= 0))
        out[key] = out.get(key, 0) + r[-1]
    return out


# ================================================================================================
# GSP candidate generation / positional clusters
# ================================================================================================
@job("candidateGenerationWithSelfJoin", "GSP k+1 candidate sequences by self-join on the (k-1)-overlap (J/sequence/CandidateGenerationWithSelfJoin.java, cgs.*)")
def cgs(args):
    """Rows hold a frequent k-sequence in their first ``cgs.item.set.length`` fields.  Every ordered
    pair (a, b) with a[1:] == b[:-1] yields a + b[-1] (incl. a == b), which fixes two reference bugs
    (pairs inside one hash bucket are never joined; the reverse join appends a token of the wrong
    sequence, :243-276).  Native path: each rank reads its byte range; the (small) set of distinct
    k-sequences is all-gathered as dictionary codes, ordered by the tokens' string ranks, and every
    rank joins its block of left sequences against all of them on the device (``SO.gsp_join``,
    K18); rank 0 writes the sorted union."""
    from ..data.table import _literal
    ctx = JobContext(args, "cgs.")
    k = ctx.get_int("item.set.length")
    lit = _literal(ctx.delim_in)
    if lit is None or len(lit) != 1:
        from ..models.markov import gsp_candidates_device
        seqs = [tuple(r[:k]) for r in ctx.rows(shard=False) if len(r) >= k]
        cands = gsp_candidates_device(seqs, device=ctx.device, comm=ctx.comm)
        ctx.emit_root([ctx.delim_out.join(c) for c in cands])
        return
    from ..data.records import format_lines, sorted_keys
    from ..data.table import shard_range
    from ..ops import sequence_ops as SO
    comm = ctx.comm
    rec = ctx.records(modes="d" * k, tail_mode="x")
    ok = rec.lens() >= k
    S = torch.stack([rec.field(j)[ok].long() for j in range(k)], 1) if k else torch.zeros((0, 0), dtype=torch.long)
    S = unique_rows(S) if S.shape[0] else S
    if comm.is_distributed:
        cdev = comm.device if comm.pg_backend == "nccl" else torch.device("cpu")
        S = comm.all_gather_v(S.to(cdev)).to(rec.device)
        S = unique_rows(S) if S.shape[0] else S
    if S.shape[0] == 0:
        ctx.emit_root_text(b"")
        return
    keys, pos = sorted_keys(rec, S.reshape(-1))          # token code -> string rank (every rank alike)
    R = pos[S].int()
    R = unique_rows(R)                           # lexicographic = tuple-of-strings order
    lo, hi = shard_range(R.shape[0], comm.rank, comm.world) if comm.is_distributed else (0, R.shape[0])
    C = SO.gsp_join(R.to(ctx.device).contiguous(), lo, hi)
    if comm.is_distributed:
        cdev = comm.device if comm.pg_backend == "nccl" else torch.device("cpu")
        C = comm.all_gather_v(C.to(cdev))
    if not ctx.is_root:
        return
    # the union's sort on the device (a host unique of the candidates was ~20 ms of the 78 ms job
    # at 800 k sequences: profiles/r6_slow_jobs.jsonl); only the code columns come back
    C = C.to(rec.device).long()
    C = unique_rows(C) if C.numel() else C.view(0, k + 1)
    kc = keys.to(C.device)
    cols = [("s", rec.vocab, kc[C[:, j]].int().cpu().contiguous()) for j in range(k + 1)]
    ctx.emit_root_columns(cols, int(C.shape[0]))


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
    from ..utils.rules import RecordColumns, rule_field_modes
    from .common import field_modes
    fm = rule_field_modes([rule], {so: "n"})
    rec = ctx.try_records(modes=field_modes(fm), tail_mode="x", numeric=True, trim=True)
    if rec is not None:
        # native: each rank tokenizes its byte range; the (time, condition) pairs of all ranks are
        # one all-gather (16 bytes a record), every rank scores the global time order and writes
        # the records of its own range
        t_l = rec.field(so, numeric=True).double()
        met_l = rule.evaluate(RecordColumns(rec, [o for o, m in fm.items() if m == "n"])).double()
        comm = ctx.comm
        pair = torch.stack([t_l, met_l], 1)
        allp = comm.all_gather_v(pair) if comm.is_distributed else pair     # scored on the job's device
        score = _locality_scores(allp[:, 0], allp[:, 1], span)
        base = rec.line_base
        sc = score[base: base + rec.n_lines]
        keep = sc > thr
        spans, dl = rec.line_spans().select(keep), ctx.native_delim()
        ctx.emit_columns([spans.column("rf", so, dl), spans.column("rf", q, dl), ("f", sc[keep], 3)], len(spans))
        return
    rows = ctx.rows(shard=False)
    t = torch.tensor([float(r[so]) for r in rows], dtype=torch.float64)
    met = rule.evaluate_rows(rows).double()
    score = _locality_scores(t, met, span)
    d = ctx.delim_out
    ctx.emit_root([f"{r[so]}{d}{r[q]}{d}{fmt(s)}" for r, s in zip(rows, score.tolist()) if s > thr])


def _locality_scores(t: torch.Tensor, met: torch.Tensor, span: float) -> torch.Tensor:
    """Fraction of condition-meeting events among the events of the trailing ``span`` (time
    order, ties in input order) of every event."""
    order = torch.argsort(t, stable=True)
    ts, ms = t[order], met[order]
    cm = torch.cumsum(ms, 0)
    lo = torch.searchsorted(ts, ts - span, right=False)
    idx = torch.arange(len(ts), device=t.device)
    n_in = (idx - lo + 1).double()
    met_in = cm - torch.where(lo > 0, cm[(lo - 1).clamp_min(0)], torch.zeros_like(cm))
    score = torch.zeros_like(t)
    score[order] = met_in / n_in
    return score


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
    # an event with an unknown state or an unparsable time stamp is an error, as in the row path
    # and the reference (DoubleTable.add fails): dropping it would splice its neighbours into a
    # transition that never happened.  Counted over all ranks so every rank stops together.
    bad = torch.tensor([int((~ok).sum())], dtype=torch.long, device=dev)
    ctx.all_reduce(bad)
    if int(bad):
        raise SystemExit(f"stateTransitionRate: {int(bad)} event(s) with a state outside state.values, "
                         f"a missing key or an unparsable time stamp")
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
    ctx.emit_columns(cols, b - a)


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
    ctx.emit_columns(cols, b - a)


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
    from .common import field_modes
    rec = ctx.try_records(modes="d" * (kl + 2), tail_mode="x")
    if rec is not None:
        _cont_time_native(ctx, rec, rates, kl, states, horizon, stat, targets)
        return
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


def _cont_time_native(ctx, rec, rates, kl, states, horizon, stat, targets):
    """contTimeStateTransitionStats over a native token table: the stats of every distinct key
    once (key level), every record's value one gather, output through the native formatter."""
    from ..models.markov import ContTimeStateTransitionStats
    S = len(states)
    n = rec.n_lines
    kc = torch.stack([rec.field(j).long() for j in range(kl)], 1) if kl else torch.zeros((n, 0), dtype=torch.long)
    uk, inv = unique_rows(kc, True) if n else (torch.zeros((0, kl), dtype=torch.long),
                                                                      torch.zeros(0, dtype=torch.long))
    P = torch.zeros((uk.shape[0], S, S), dtype=torch.float64)
    Dw = torch.zeros((uk.shape[0], S, S), dtype=torch.float64)
    Q = torch.zeros((uk.shape[0], S, S), dtype=torch.float64)
    for u, codes in enumerate(uk.tolist()):
        key = tuple(rec.vocab[c] for c in codes)
        if key not in rates:
            raise SystemExit(f"contTimeStateTransitionStats: no rate matrix for key {key}")
        cs = ContTimeStateTransitionStats(rates[key].to(ctx.device))
        A, B = cs.sums([horizon])
        P[u], Dw[u], Q[u] = A[0].cpu(), B[0].cpu(), cs.Q.cpu()
    i0 = rec.map_codes(rec.field(kl), states).long().cpu()
    if bool((i0 < 0).any()):
        raise SystemExit("contTimeStateTransitionStats: unknown initial state")
    inv = inv.cpu()
    if stat == "futureStateProb":
        end = rec.map_codes(rec.field(kl + 1), states).long().cpu()
        if bool((end < 0).any()):
            raise SystemExit("futureStateProb needs an end state")
        v = P[inv, i0, end]
    elif stat == "stateDwellTime":
        v = Dw[inv, i0, states.index(targets[0])]
    elif stat == "StateTransitionCount":
        a, b = states.index(targets[0]), states.index(targets[1])
        v = Dw[inv, i0, a] * Q[inv, a, b]
    else:
        raise SystemExit(f"invalid state transition stats {stat}")
    spans, dl = rec.line_spans(), ctx.native_delim()
    ctx.emit_columns([("g", "(")] + [spans.column("rf", j, dl) for j in range(kl)] + [("f", v, -2), ("g", ")")], n)


# ================================================================================================
# sequence analytics
# ================================================================================================
@job("dotMatrixMatching", "all-pairs dot-matrix window-match similarity of sequences (S/sequence/DotMatrixMatching.scala)")
def dot_matrix(args):
    """Rows ``id,tok,tok,...``; every pair (i < j) gets the window-match score of the K19
    dot-matrix kernel; output ``id1,id2,score`` in (i, j) order.  Native path: each rank reads its
    byte range; its sequences stay put while the other ranks' blocks (padded token-code rows + id
    codes + global row base) travel around the ring (``Comm.ring_iter``, the next transfer posted
    before the current block's kernel runs) — instead of the reference's bucket-pair replication
    (S/sequence/DotMatrixMatching.scala:76-100)."""
    from ..data.table import _literal
    ctx = JobContext(args, app="dotMatrixMatching")
    skip = ctx.get_int("skip.field.count", 1)
    w = ctx.get_int("window.size", 3)
    prec = ctx.get_int("output.precision", 3)
    lit = _literal(ctx.delim_in)
    if lit is None or len(lit) != 1:
        return _dot_matrix_rows(ctx, skip, w, prec)
    from ..data.records import format_lines
    from ..models.markov import dot_matrix_similarity
    comm = ctx.comm
    rec = ctx.records(modes="d" + "x" * max(0, skip - 1))
    X, _ = rec.padded(start=skip, dtype=torch.long, min_len=w)
    Lm = torch.tensor([X.shape[1]], dtype=torch.long)
    if comm.is_distributed:
        comm.all_reduce(Lm, "max")
    L = int(Lm)
    if X.shape[1] < L:
        X = torch.cat([X, torch.full((X.shape[0], L - X.shape[1]), -1, dtype=X.dtype, device=X.device)], 1)
    ids = rec.field(0).long()
    base = rec.line_base
    cdev = comm.device if (comm.is_distributed and comm.pg_backend == "nccl") else torch.device("cpu")
    payload = [X.to(cdev), ids.to(cdev), torch.tensor([base], dtype=torch.long, device=cdev)]
    dev = ctx.device
    A = X.to(dev)
    I, J, Sv, Jid = [], [], [], []
    for _owner, (Bx, bid, bb) in comm.ring_iter(payload):
        b0 = int(bb.cpu()[0]) if bb.numel() else 0
        if Bx.shape[0] == 0 or A.shape[0] == 0:
            continue
        Sm = dot_matrix_similarity(A, Bx.to(dev), w)
        keep = (torch.arange(b0, b0 + Bx.shape[0], device=Sm.device).view(1, -1)
                > torch.arange(base, base + A.shape[0], device=Sm.device).view(-1, 1))
        qi, jj = torch.nonzero(keep, as_tuple=True)
        I.append(qi)
        J.append(jj + b0)
        Sv.append(Sm[qi, jj])
        Jid.append(bid.to(Sm.device)[jj])
    if I:
        I, J, Sv, Jid = torch.cat(I), torch.cat(J), torch.cat(Sv), torch.cat(Jid)
        o = torch.argsort(I * (1 << 40) + J)
        I, Sv, Jid = I[o], Sv[o], Jid[o]
    else:
        I = Jid = torch.zeros(0, dtype=torch.long)
        Sv = torch.zeros(0, dtype=torch.float64)
    cols = [("s", rec.vocab, ids.to(I.device)[I].int().cpu()), ("s", rec.vocab, Jid.int().cpu()),
            ("f", Sv.double().cpu(), prec)]
    ctx.emit_columns(cols, int(I.numel()))


def _dot_matrix_rows(ctx, skip, w, prec):
    """Regex delimiters: the split-row path (every rank reads the input, scores a block of rows)."""
    from ..models.markov import dot_matrix_similarity
    rows = ctx.rows(shard=False)
    vocab = {}
    L = max([len(r) - skip for r in rows] + [w])
    X = torch.tensor([[vocab.setdefault(t, len(vocab)) for t in r[skip:]] + [-1] * (L - len(r) + skip) for r in rows],
                     dtype=torch.long).view(len(rows), L)
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
    from .common import field_modes
    rec = ctx.try_records(modes=field_modes({**{o: "d" for o in kords}, to: "n"}), tail_mode="x", numeric=True)
    if rec is not None:
        from ..data.records import sorted_key_tuples
        kpos, G, ktab = sorted_key_tuples(rec, [rec.field(o) for o in kords], ctx.comm)
        t = rec.field(to, numeric=True).long()
        if res == "hourOfDay":
            b, B = (t % 86400_000) // 3600_000 // gr, (24 + gr - 1) // gr
        else:
            b, B = ((t // 86400_000) + 4) % 7, 7
        H = torch.zeros(G * B, dtype=torch.long, device=rec.device).index_add_(0, kpos * B + b, torch.ones_like(b))
        ctx.all_reduce(H)
        d = ctx.delim_out
        ctx.emit_root([d.join([rec.vocab[c] for c in k] + [f"{j}:{int(c)}" for j, c in enumerate(h) if c])
                       for k, h in zip(ktab.tolist(), H.view(G, B).tolist())])
        return
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
    order, ties in input order), keys in string order.  Native path: each rank reads its byte
    range; records move to the rank owning their key (one all-to-all; keys in string order cut
    into contiguous blocks, so the rank-ordered part files are the global order); one device sort
    by (key, sequence) per rank and the native formatter."""
    from ..data.table import _literal
    ctx = JobContext(args, app="sequenceGenerator")
    kords = ctx.get_int_list("id.field.ordinals")
    vords = ctx.get_int_list("val.field.ordinals")
    sf = ctx.get_int("seq.field")
    lit = _literal(ctx.delim_in)
    if lit is None or len(lit) != 1:
        return _seq_gen_rows(ctx, kords, vords, sf)
    from ..data.records import format_lines, owner_of, shuffle, sorted_key_tuples
    from ..data.table import shard_range
    comm = ctx.comm
    top = max(list(kords) + list(vords) + [sf]) + 1
    modes = "".join("n" if i == sf else ("d" if (i in kords or i in vords) else "x") for i in range(top))
    # the sequence field doubles as a value field: its number AND its dictionary string
    rec = ctx.records(modes=modes, tail_mode="x", numeric=True)
    if sf in vords:
        rec2 = ctx.records(modes="".join("d" if i == sf else "x" for i in range(top)), tail_mode="x")
        vcols = [rec2.field(o).long() if o == sf else rec.field(o).long() for o in vords]
    else:
        vcols = [rec.field(o).long() for o in vords]
    kpos, G, ktab = sorted_key_tuples(rec, [rec.field(o) for o in kords], comm)
    seqv = torch.trunc(rec.field(sf, numeric=True)).long()
    owner = owner_of(kpos, G, comm.world) if comm.is_distributed else torch.zeros_like(kpos)
    cols = shuffle(comm, owner, [kpos, seqv] + vcols)
    kp, sv, V = cols[0], cols[1], torch.stack(cols[2:], 1) if vcols else None
    o = torch.argsort(sv, stable=True)
    o = o[torch.argsort(kp[o], stable=True)]
    kp = kp[o]
    a, b = shard_range(G, comm.rank, comm.world) if comm.is_distributed else (0, G)
    cnt = torch.bincount(kp - a, minlength=b - a) * len(vords) if b > a else torch.zeros(0, dtype=torch.long)
    off = torch.cat([torch.zeros(1, dtype=torch.long, device=cnt.device), torch.cumsum(cnt, 0)]).cpu()
    vals = V[o].reshape(-1).int().cpu() if V is not None else torch.zeros(0, dtype=torch.int32)
    out = [("s", rec.vocab, ktab[a:b, j].int().contiguous()) for j in range(len(kords))]
    out.append(("l", rec.vocab, vals, off))
    ctx.emit_columns(out, b - a)


def _seq_gen_rows(ctx, kords, vords, sf):
    """Regex delimiters: the split-row path."""
    from ..models.markov import sequence_generator
    rows = ctx.rows(shard=False)
    keys = sorted({tuple(r[o] for o in kords) for r in rows})
    ki = {k: i for i, k in enumerate(keys)}
    kk = torch.tensor([ki[tuple(r[o] for o in kords)] for r in rows], dtype=torch.long)
    sv = torch.tensor([int(float(r[sf])) for r in rows], dtype=torch.long)
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
    """Per key, records ordered by ``seq.fieldOrd`` (ties in input order); every full window of
    ``window.size`` symbols of ``attr.ordinal`` is counted; output ``key..,w1:w2:w3,count,...``
    (windows in string order), keys in string order.  Native path: byte-range reads, one
    all-to-all to the key owners, windows gathered from the device sort and counted by one unique
    over (key, window) codes."""
    from ..data.table import _literal
    ctx = JobContext(args, app="markovChainPredictor")
    kords = ctx.get_int_list("id.fieldOrdinals", [])
    ao = ctx.get_int("attr.ordinal")
    so = ctx.get_int("seq.fieldOrd")
    w = ctx.get_int("window.size", 3)
    lit = _literal(ctx.delim_in)
    if lit is None or len(lit) != 1:
        return _time_delay_rows(ctx, kords, ao, so, w)
    from ..data.records import format_lines, owner_of, segment_rank, shuffle, sorted_key_tuples
    from ..data.table import shard_range
    comm = ctx.comm
    top = max(list(kords) + [ao, so]) + 1
    modes = "".join("n" if i == so else ("d" if (i in kords or i == ao) else "x") for i in range(top))
    rec = ctx.records(modes=modes, tail_mode="x", numeric=True)
    kpos, G, ktab = sorted_key_tuples(rec, [rec.field(o) for o in kords], comm)
    owner = owner_of(kpos, G, comm.world) if comm.is_distributed else torch.zeros_like(kpos)
    kp, sq, sym = shuffle(comm, owner, [kpos, rec.field(so, numeric=True), rec.field(ao).long()])
    o = torch.argsort(sq, stable=True)
    o = o[torch.argsort(kp[o], stable=True)]
    kp, sym = kp[o], sym[o]
    first = torch.ones_like(kp, dtype=torch.bool)
    first[1:] = kp[1:] != kp[:-1]
    end = torch.nonzero(segment_rank(first) >= w - 1).view(-1)
    win = sym[end.view(-1, 1) - (w - 1) + torch.arange(w, device=sym.device).view(1, -1)]   # [n_win, w]
    a, b = shard_range(G, comm.rank, comm.world) if comm.is_distributed else (0, G)
    uwin, winv = unique_rows(win, True) if win.numel() else (win, win[:, 0])
    # window strings (few distinct): their string order decides the output order inside a key
    wstr = [":".join(rec.vocab[c] for c in row) for row in uwin.cpu().tolist()]
    wrank = torch.empty(len(wstr), dtype=torch.long)
    wrank[torch.tensor(sorted(range(len(wstr)), key=wstr.__getitem__), dtype=torch.long)] = \
        torch.arange(len(wstr), dtype=torch.long)
    wr = wrank.to(win.device)[winv] if win.numel() else winv
    key = (kp[end] - a) * max(1, len(wstr)) + wr
    uk, cnt = torch.unique(key, return_counts=True)
    kk, ww = uk // max(1, len(wstr)), uk % max(1, len(wstr))
    per = torch.bincount(kk, minlength=b - a) if b > a else torch.zeros(0, dtype=torch.long)
    off = torch.cat([torch.zeros(1, dtype=torch.long, device=per.device), torch.cumsum(per, 0)]).cpu()
    wtab = sorted(wstr)
    out = [("s", rec.vocab, ktab[a:b, j].int().contiguous()) for j in range(len(kords))]
    out.append(("lp", wtab, ww.int().cpu(), cnt.long().cpu(), off))
    ctx.emit_columns(out, b - a)


def _time_delay_rows(ctx, kords, ao, so, w):
    """Regex delimiters: the split-row path."""
    g = defaultdict(list)
    for r in ctx.rows(shard=False):
        g[tuple(r[o] for o in kords)].append((float(r[so]), r[ao]))
    seqs = [(k, [s for _, s in sorted(v, key=lambda e: e[0])]) for k, v in sorted(g.items())]
    if ctx.comm.is_distributed:
        from ..data.table import shard_range
        a, b = shard_range(len(seqs), ctx.comm.rank, ctx.comm.world)
        seqs = seqs[a:b]
    d = ctx.delim_out
    out = []
    for k, s in seqs:
        c: dict[str, int] = defaultdict(int)
        for i in range(len(s) - w + 1):
            c[":".join(s[i:i + w])] += 1
        out.append(d.join(list(k) + [f"{x}{d}{c[x]}" for x in sorted(c)]))
    ctx.emit(out)
