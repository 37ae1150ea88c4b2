"""Sequence ops (K14/K15 Viterbi / log-odds, K5 n-grams, K16 uniformisation, K19 dot matrix):
GPU -> HIP kernels; CPU -> PyTorch references."""
from __future__ import annotations

import numpy as np
import torch
from .encode_ops import unique_rows

from .. import _native
from ..utils.tracing import traced


@traced("viterbi", nbytes=lambda obs, *a, **k: obs.numel() * obs.element_size(), device=lambda obs, *a, **k: obs.device)
def viterbi(obs: torch.Tensor, logA: torch.Tensor, logB: torch.Tensor, logpi: torch.Tensor,
            forward: bool = False) -> tuple[torch.Tensor | None, torch.Tensor]:
    """Batched log-space Viterbi (path int16 [N, T], -1 padded; score [N]) or, with ``forward``,
    the forward log-likelihood [N].  ``obs`` int16 [N, T], negative = end of sequence."""
    obs = obs.to(torch.int16).contiguous()
    if obs.is_cuda:
        path, score = _native.C().viterbi(obs, logA.float().contiguous(), logB.float().contiguous(),
                                          logpi.float().contiguous(), 1 if forward else 0)
        return (None if forward else path), score
    N, T = obs.shape
    S = logA.shape[0]
    lA, lB, lp = logA.double(), logB.double(), logpi.double()
    ob = obs.long()
    valid = (ob >= 0) & (ob < lB.shape[1])      # an out-of-range observation ends the sequence too
    lens = torch.where(valid.all(1), torch.full((N,), T), (~valid).int().argmax(1))
    ob = torch.where(valid, ob, torch.zeros_like(ob))
    o0 = ob[:, 0].clamp_min(0)
    delta = lp.view(1, S) + lB[:, o0].T
    bps = []
    for t in range(1, T):
        ot = ob[:, t].clamp_min(0)
        cand = delta.unsqueeze(2) + lA.unsqueeze(0)            # [N, S_i, S_j]
        if forward:
            nd = torch.logsumexp(cand, 1) + lB[:, ot].T
            bp = None
        else:
            mx, bp = cand.max(1)
            nd = mx + lB[:, ot].T
        act = (t < lens).view(N, 1)
        delta = torch.where(act, nd, delta)
        bps.append(bp)
    empty = lens == 0                              # an invalid first observation: no path, score -inf
    if forward:
        ll = torch.logsumexp(delta, 1)
        return None, torch.where(empty, torch.full_like(ll, float("-inf")), ll).float()
    score, s = delta.max(1)
    score = torch.where(empty, torch.full_like(score, float("-inf")), score)
    # backtrack all rows at once: path[L-1] = argmax, path[t] = bp_{t+1}[path[t+1]] for t < L-1
    path = torch.full((N, T), -1, dtype=torch.int16)
    rows = torch.arange(N)
    nxt = s.clone()
    for t in range(T - 1, -1, -1):
        st = s if t == T - 1 else torch.where(t == lens - 1, s, bps[t][rows, nxt])
        st = torch.where(t < lens, st, torch.full_like(st, -1))
        path[:, t] = st.to(torch.int16)
        nxt = st.clamp_min(0)
    return path, score.float()


# ------------------------------------------------------------------------------------------------
# long-sequence Viterbi: chunked max-plus scan, sequence-parallel across ranks
# ------------------------------------------------------------------------------------------------
def _viterbi_rows_cpu(ob, lA, lB, start, want_bp):
    """CPU oracle of the chunk kernel: Viterbi over rows ``ob`` [R, L] from per-row start vectors
    ``start`` [R, S] (delta at position 0 = start + logB[:, o_0]).  Returns (back-pointers
    [R, L, S] or None, final delta [R, S])."""
    R, L = ob.shape
    S = lA.shape[0]
    o = ob.long()
    valid = o >= 0
    lens = torch.where(valid.all(1), torch.full((R,), L), (~valid).int().argmax(1))
    delta = start + lB[:, o[:, 0].clamp_min(0)].T
    delta = torch.where((lens > 0).view(R, 1), delta, torch.full_like(delta, float("-inf")))
    bp = torch.zeros((R, L, S), dtype=torch.long) if want_bp else None
    for t in range(1, L):
        mx, arg = (delta.unsqueeze(2) + lA.unsqueeze(0)).max(1)
        delta = torch.where((t < lens).view(R, 1), mx + lB[:, o[:, t].clamp_min(0)].T, delta)
        if bp is not None:
            bp[:, t] = arg
    return bp, delta


def _run_chunks(ob, lA, lB, start, n, obs_div, want_bp):
    """n independent Viterbi runs: run k decodes observation row k // obs_div from start row
    k % len(start).  GPU: the K14 kernel, one wavefront per run."""
    if ob.is_cuda:
        bp = (torch.empty((n, ob.shape[1], lA.shape[0]), dtype=torch.int16, device=ob.device)
              if want_bp else None)
        return bp, _native.C().viterbi_chunks(ob, lA, lB, start, n, obs_div, bp)
    k = torch.arange(n)
    return _viterbi_rows_cpu(ob[k // obs_div], lA, lB, start[k % start.shape[0]], want_bp)


def _backtrack(bp, lens, ends, first: bool):
    """Follow chunk c's back-pointers from state ends[c, k] at its last position to position 0:
    the states reached ([P, K], ``first``) or the path of track 0 ([P, L])."""
    P, K = ends.shape
    if bp.is_cuda:
        e = ends.to(torch.int32).contiguous().view(-1)
        if first:
            out = torch.empty(P * K, dtype=torch.int32, device=bp.device)
            _native.C().viterbi_backtrack(bp, lens, e, K, out, None)
            return out.view(P, K).long()
        path = torch.empty((P, bp.shape[1]), dtype=torch.int16, device=bp.device)
        _native.C().viterbi_backtrack(bp, lens, e, 1, None, path)
        return path
    L = bp.shape[1]
    s = ends.long().clone()
    ln = lens.long()
    path = torch.full((P, L), -1, dtype=torch.int16)
    has = ln > 0
    path[has, ln[has] - 1] = s[has, 0].to(torch.int16)
    for t in range(L - 1, 0, -1):
        act = (t <= ln - 1).view(P, 1)
        s = torch.where(act, torch.gather(bp[:, t], 1, s), s)
        path[:, t - 1] = torch.where(act[:, 0], s[:, 0].to(torch.int16), path[:, t - 1])
    return s if first else path


def _maxplus_prefix(X):
    """Inclusive prefix max-plus products X[0] (x) ... (x) X[c] of [n, S, S]: Hillis-Steele,
    ceil(log2 n) batched steps, temporaries bounded to ~2^25 elements."""
    n, S = X.shape[0], X.shape[-1]
    blk = max(1, (1 << 25) // S ** 3)
    d = 1
    while d < n:
        nxt = X.clone()
        for a in range(d, n, blk):
            b = min(n, a + blk)
            nxt[a:b] = (X[a - d:b - d].unsqueeze(3) + X[a:b].unsqueeze(1)).amax(2)
        X = nxt
        d *= 2
    return X


def _stitch(D, F, lA, f_next):
    """Chunk end states of the best path for each candidate first state of the NEXT segment
    (-1: none, end in the best final state).  D [P, S] chunk-end deltas, F [P, S] end -> start
    state maps.  The boundary argmaxes are one batched device op; only a chain of P table
    lookups stays sequential (host).  Returns (ends [K, P], first states [K])."""
    P = D.shape[0]
    lA = lA.to(D.dtype)
    fn = torch.as_tensor(list(f_next), dtype=torch.long, device=D.device)
    add = torch.where(fn.view(-1, 1) < 0, torch.zeros_like(D[P - 1]).unsqueeze(0), lA[:, fn.clamp_min(0)].T)
    e = (D[P - 1].unsqueeze(0) + add).argmax(1).cpu().numpy()
    Fh = F.cpu().numpy()
    ends = np.empty((len(e), P), dtype=np.int64)
    ends[:, P - 1] = e
    f = Fh[P - 1, e]
    if P > 1:
        E = (D[:-1].unsqueeze(2) + lA.unsqueeze(0)).argmax(1)   # best end of chunk c-1 entering state f
        Hm = torch.gather(F[:-1], 1, E)                          # ... and the first state of chunk c-1
        Eh, Hh = E.cpu().numpy(), Hm.cpu().numpy()
        for c in range(P - 1, 0, -1):
            ends[:, c - 1] = Eh[c - 1, f]
            f = Hh[c - 1, f]
    return ends, f


def viterbi_long(obs: torch.Tensor, logA: torch.Tensor, logB: torch.Tensor, logpi: torch.Tensor,
                 chunk: int = 1024, comm=None) -> tuple[torch.Tensor, float]:
    """Viterbi decoding of ONE long observation sequence as a chunked max-plus scan (SURVEY.md
    §5.7; the reference decodes every sequence in one sequential loop,
    J/markov/ViterbiDecoder.java:53-143):

    1. chunk products M_c[i, j] = best score through chunk c ending in j when entered from state
       i: the P x S (chunk, entry state) pairs are independent Viterbi runs, one wavefront each;
    2. scan: the score vector at every chunk end is a prefix max-plus product of the M_c
       (ceil(log2 P) batched steps); across ranks each rank's total is all-gathered;
    3. every chunk is re-decoded from its exact entry vector with back-pointers; the end -> start
       state map of each chunk (S back-tracks per chunk, in parallel) lets the chunk boundaries be
       stitched with one batched argmax and a chain of P lookups, then all chunks back-track in
       parallel.

    ``obs``: this rank's contiguous segment (1-D, a negative value ends it); with a distributed
    ``comm`` the segments of ranks 0..W-1 form the sequence in rank order and every rank gets
    the path of its own segment.  Returns (path int16 [len(obs)], -1 past the end; best score)."""
    from ..parallel.comm import get_comm
    comm = comm or get_comm()
    dist = comm.is_distributed
    rank, world = (comm.rank, comm.world) if dist else (0, 1)
    ob1 = obs.reshape(-1).to(torch.int16)
    dev = ob1.device
    neg = (ob1 < 0).nonzero()
    T = int(neg[0, 0]) if neg.numel() else int(ob1.numel())
    if T == 0:
        raise ValueError("viterbi_long: empty observation segment")
    S = int(logA.shape[0])
    dt = torch.float32 if dev.type == "cuda" else torch.float64
    lA = logA.to(dev, dt).contiguous()
    lB = logB.to(dev, dt).contiguous()
    lp = logpi.to(dev, dt).reshape(1, S).contiguous()
    L = max(2, int(chunk))
    P = (T + L - 1) // L
    ob = torch.full((P * L,), -1, dtype=torch.int16, device=dev)
    ob[:T] = ob1[:T]
    ob = ob.view(P, L)
    lens = (T - torch.arange(P, device=dev) * L).clamp(max=L).to(torch.int32)
    # 1. chunk products
    _, M = _run_chunks(ob, lA, lB, lA, P * S, S, False)
    M = M.view(P, S, S)
    if rank == 0:  # the sequence start: every row of M[0] is the delta from logpi
        _, v0 = _run_chunks(ob, lA, lB, lp, 1, 1, False)
        M[0] = v0.view(1, S).expand(S, S)
    # 2. scan (u: score vector entering this segment)
    pre = _maxplus_prefix(M)
    u = torch.zeros(S, dtype=dt, device=dev)
    if dist:
        tot = comm.all_gather(pre[-1].contiguous())
        if rank > 0:
            u = tot[0, 0].clone()
            for q in range(1, rank):
                u = (u.view(S, 1) + tot[q]).amax(0)
    v = (u.view(1, S, 1) + pre).amax(1)
    entry = torch.cat([u.view(1, S), v[:-1]], 0)
    start = (entry.unsqueeze(2) + lA.unsqueeze(0)).amax(1)
    if rank == 0:
        start[0] = lp[0]
    # 3. exact re-decode with back-pointers, end -> start maps, stitching, parallel back-track
    bp, D = _run_chunks(ob, lA, lB, start.contiguous(), P, 1, True)
    F = _backtrack(bp, lens, torch.arange(S, device=dev).repeat(P, 1), first=True)
    f_next = -1
    if dist:
        _, g = _stitch(D, F, lA, range(-1, S))
        G = comm.all_gather(torch.as_tensor(g, dtype=torch.long, device=dev)).cpu().numpy()
        for q in range(world - 1, rank, -1):
            f_next = int(G[q][f_next + 1])
    ends, _ = _stitch(D, F, lA, [f_next])
    path = _backtrack(bp, lens, torch.as_tensor(ends[0], device=dev).view(P, 1), first=False)
    out = torch.full((ob1.numel(),), -1, dtype=torch.int16, device=dev)
    out[:T] = path.reshape(-1)[:T]
    score = float(D[P - 1].max())
    if dist:
        score = float(comm.all_gather(torch.tensor([score], dtype=torch.float64, device=dev))[world - 1, 0])
    return out, score


def markov_logodds(states: torch.Tensor, log_ratio: torch.Tensor) -> torch.Tensor:
    """Sum of log(A0/A1) over each sequence's transitions (stops at the first negative state)."""
    st = states.to(torch.int16).contiguous()
    if st.is_cuda:
        return _native.C().markov_logodds(st, log_ratio.float().contiguous())
    N, L = st.shape
    S = log_ratio.shape[0]
    s = st.long()
    a, b = s[:, :-1], s[:, 1:]
    ok = (a >= 0) & (b >= 0) & (a < S) & (b < S)
    ok = torch.cumprod(ok.int(), 1).bool()  # stop at first invalid transition
    v = log_ratio.float()[a.clamp(0, S - 1), b.clamp(0, S - 1)]
    return (v * ok).sum(1)


def ngram_counts(states: torch.Tensor, n_states: int, min_len: int = 2, max_len: int = 5,
                 group: torch.Tensor | None = None) -> dict[int, tuple[torch.Tensor, torch.Tensor]]:
    """Count every contiguous sub-sequence of length min_len..max_len (ProbabilisticSuffixTree
    counting, J/markov/ProbabilisticSuffixTreeGenerator.java:140-194).  n-grams are packed into
    int64 keys (base n_states + 1, group id in the high bits).  GPU: one pass of the K5 hash-count
    kernel for all lengths (LDS-privatised table, global open addressing); CPU: per-length device
    sort (torch.unique; also on a GPU when the states do not fit the kernel's int16).  Returns
    {length: (sorted keys, counts)}."""
    N, L = states.shape
    base = n_states + 1
    gmul = base ** max_len
    if group is not None:
        gmax = int(group.max()) + 1 if group.numel() else 1
        if gmul * gmax >= (1 << 58):
            raise ValueError("n-gram key space (groups x (S+1)^max_len) exceeds 2^58")
    elif gmul >= (1 << 58):
        raise ValueError("n-gram key space (S+1)^max_len exceeds 2^58")
    if states.is_cuda and n_states < 32767:
        st = states.to(torch.int16).contiguous()
        g = group.to(torch.int32).contiguous() if group is not None else None
        windows = sum(max(0, L - k + 1) for k in range(min_len, max_len + 1)) * N
        space = sum(base ** k for k in range(min_len, max_len + 1)) * (gmax if group is not None else 1)
        cap = 1 << max(10, int(2 * min(windows, space) + 1).bit_length())
        keys, counts = _native.C().ngram_count(st, n_states, min_len, max_len, g, gmul, min(cap, 1 << 30))
        keys, order = torch.sort(keys)
        counts = counts[order]
        ln = keys >> 58
        keys = keys & ((1 << 58) - 1)
        out = {}
        for k in range(min_len, max_len + 1):
            if k > L:
                break
            m = ln == k
            out[k] = (keys[m], counts[m])
        return out
    s = states.long()
    out = {}
    for k in range(min_len, max_len + 1):
        if k > L:
            break
        key = torch.zeros((N, L - k + 1), dtype=torch.long, device=s.device)
        ok = torch.ones_like(key, dtype=torch.bool)
        for j in range(k):
            col = s[:, j: L - k + 1 + j]
            ok &= (col >= 0) & (col < n_states)
            key = key * base + col.clamp_min(0)
        if group is not None:
            key = key + group.long().view(-1, 1) * gmul
        keys, counts = torch.unique(key[ok], return_counts=True)
        out[k] = (keys, counts)
    return out


def uniformization_sums(P: torch.Tensor, w1: torch.Tensor, w2: torch.Tensor,
                        steps: list[int]) -> tuple[torch.Tensor, torch.Tensor]:
    """A_b = sum_{k<=steps[b]} w1[b,k] P^k and B_b = sum w2[b,k] P^k for B problems sharing one
    S x S matrix (S <= 64): the K16 power-chain kernel on GPU (P^k never leaves LDS), repeated
    fp64 matmuls on CPU.  w1, w2 [B, ldw] with ldw > max(steps)."""
    P = P.double().contiguous()
    w1 = w1.double().contiguous()
    w2 = w2.double().contiguous()
    if P.is_cuda:
        st = torch.tensor(steps, dtype=torch.int32, device=P.device)
        out = _native.C().uniformization(P, w1, w2, st, [int(s) for s in steps])
        return out[:, 0], out[:, 1]
    S = P.shape[0]
    A = torch.zeros((len(steps), S, S), dtype=torch.float64)
    B = torch.zeros_like(A)
    for b, L in enumerate(steps):
        cur = torch.eye(S, dtype=torch.float64)
        for k in range(L + 1):
            if k:
                cur = cur @ P
            A[b] += w1[b, k] * cur
            B[b] += w2[b, k] * cur
    return A, B


def dot_matrix_hits(ida: torch.Tensor, idb: torch.Tensor) -> torch.Tensor:
    """hits[i, j] = #{(p, q): ida[i, p] == idb[j, q] >= 0} (K19 on GPU).  Inputs are int32 window
    ids (negative = invalid window)."""
    if ida.is_cuda:
        return _native.C().dot_matrix(ida.to(torch.int32).contiguous(), idb.to(torch.int32).contiguous())
    a = ida.long()
    b = torch.where(idb.long() < 0, torch.full_like(idb.long(), -2), idb.long())
    eq = a.unsqueeze(1).unsqueeze(3) == b.unsqueeze(0).unsqueeze(2)
    return eq.sum((2, 3)).to(torch.int32)


def gsp_join(X: torch.Tensor, lo: int = 0, hi: int | None = None) -> torch.Tensor:
    """GSP candidate self-join (K18): X int [N, k] token-id rows; left rows [lo, hi) of the
    lexicographically sorted unique rows are joined with every row b whose b[:-1] equals their
    a[1:], giving a ++ b[-1].  Returns int32 [M, k+1] (left-row order, partners in sorted order)."""
    X = unique_rows(X.to(torch.int32)) if X.numel() else X.to(torch.int32)
    N, k = X.shape
    hi = N if hi is None else hi
    if X.is_cuda:
        return _native.C().gsp_join(X.contiguous(), int(lo), int(hi))
    if N == 0 or hi <= lo:
        return torch.zeros((0, k + 1), dtype=torch.int32)
    # oracle: dense ids of the (k-1)-grams, partners found by searchsorted over sorted prefix ids
    both = torch.cat([X[:, :-1], X[:, 1:]])
    _, inv = unique_rows(both, True)
    pid, sid = inv[:N], inv[N:]
    order = torch.argsort(pid, stable=True)
    ps = pid[order]
    a = torch.arange(lo, hi)
    s = torch.searchsorted(ps, sid[a], right=False)
    e = torch.searchsorted(ps, sid[a], right=True)
    cnt = e - s
    left = torch.repeat_interleave(a, cnt)
    base = torch.repeat_interleave(s - torch.cumsum(cnt, 0) + cnt, cnt)
    right = order[base + torch.arange(int(cnt.sum()))]
    return torch.cat([X[left], X[right, -1:]], 1)


def decode_ngram(key: int, k: int, n_states: int, max_len: int | None = None) -> tuple[int, list[int]]:
    base = n_states + 1
    grp = 0
    if max_len is not None:
        grp, key = divmod(key, base ** max_len)
    seq = []
    for _ in range(k):
        key, r = divmod(key, base)
        seq.append(r)
    return grp, seq[::-1]
