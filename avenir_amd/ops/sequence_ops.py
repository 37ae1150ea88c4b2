"""Sequence ops (K14/K15 Viterbi / log-odds, K5 n-grams, K16 uniformisation, K19 dot matrix):
GPU -> HIP kernels; CPU -> PyTorch references."""
from __future__ import annotations

import torch

from .. import _native


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
    valid = ob >= 0
    lens = torch.where(valid.all(1), torch.full((N,), T), (~valid).int().argmax(1))
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
    if forward:
        return None, torch.logsumexp(delta, 1).float()
    score, s = delta.max(1)
    path = torch.full((N, T), -1, dtype=torch.int16)
    for r in range(N):
        L = int(lens[r])
        if L == 0:
            continue
        st = int(s[r])
        path[r, L - 1] = st
        for t in range(L - 1, 0, -1):
            st = int(bps[t - 1][r, st])
            path[r, t - 1] = st
    return path, score.float()


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
    sort (torch.unique).  Returns {length: (sorted keys, counts)}."""
    N, L = states.shape
    base = n_states + 1
    gmul = base ** max_len
    if group is not None:
        gmax = int(group.max()) + 1 if group.numel() else 1
        if gmul * gmax >= (1 << 58):
            raise ValueError("n-gram key space (groups x (S+1)^max_len) exceeds 2^58")
    elif gmul >= (1 << 58):
        raise ValueError("n-gram key space (S+1)^max_len exceeds 2^58")
    if states.is_cuda:
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
