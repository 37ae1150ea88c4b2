"""Markov chains, HMMs, Viterbi, suffix statistics, continuous-time Markov chains and sequence
mining (``J/markov``, ``J/sequence``, ``S/markov``, ``S/sequence``).

* ``MarkovStateTransitionModel`` — first-order transition counts (K4 bigram kernel, one pass, one
  all-reduce), Laplace correction on rows containing a zero, integer-scaled or float rows
  (``J/markov/MarkovStateTransitionModel.java``, ``J/util/StateTransitionProbability.java:87-117``).
* ``MarkovModelClassifier`` — cumulative log-odds of two class models vs a threshold (K15 kernel).
* ``HiddenMarkovModelBuilder`` / ``HiddenMarkovModel`` / ``ViterbiDecoder`` — supervised estimation
  from ``obs:state`` tokens and batched log-space decoding (K14 kernel).
* ``ProbabilisticSuffixTree`` — counts of every sub-sequence of length 2..L (device radix-sort
  counting) assembled into a suffix tree.
* ``StateTransitionRate`` / ``ContTimeStateTransitionStats`` — CTMC rate matrix from timestamped
  state sequences and uniformisation statistics (``S/markov/*.scala``).
* ``SequenceGenerator``, ``TimeDelayEmbedding``, ``gsp_candidates`` (GSP self-join),
  ``dot_matrix_similarity``, ``positional_event_clusters``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from pathlib import Path

import torch
from ..ops.encode_ops import unique_rows

from ..ops import histogram as H
from ..ops import sequence_ops as SO
from ..parallel.comm import Comm, get_comm


# ================================================================================================
# transition probability tables
# ================================================================================================
def normalize_rows(counts: torch.Tensor, scale: int = 1, laplace: bool = True) -> torch.Tensor:
    """StateTransitionProbability.normalizeRows: add 1 to every cell of a row that has a zero, then
    divide by the row sum (integer division x scale when scale > 1)."""
    c = counts.long().clone()
    if laplace:
        zero_row = (c == 0).any(-1, keepdim=True)
        c = c + zero_row.long()
    rs = c.sum(-1, keepdim=True).clamp_min(1)
    if scale > 1:
        return (c * scale) // rs
    return c.double() / rs


class MarkovStateTransitionModel:
    def __init__(self, states: list[str], class_labels: list[str] | None = None, scale: int = 1000,
                 laplace: bool = True, comm: Comm | None = None):
        self.states = list(states)
        self.class_labels = class_labels
        self.scale = scale
        self.laplace = laplace
        self.comm = comm
        self.counts: torch.Tensor | None = None

    @property
    def n_states(self) -> int:
        return len(self.states)

    def encode(self, seqs: list[list[str]], length: int | None = None) -> torch.Tensor:
        idx = {s: i for i, s in enumerate(self.states)}
        L = length or max((len(s) for s in seqs), default=0)
        out = torch.full((len(seqs), L), -1, dtype=torch.int16)
        for r, s in enumerate(seqs):
            for j, v in enumerate(s[:L]):
                out[r, j] = idx.get(v, -1)
        return out

    def fit(self, states: torch.Tensor, labels: torch.Tensor | None = None) -> "MarkovStateTransitionModel":
        C = len(self.class_labels) if (labels is not None and self.class_labels) else 1
        cnt = H.bigram_histogram(states, self.n_states, labels if C > 1 else None, C)
        comm = self.comm or get_comm()
        if comm.is_distributed:
            comm.all_reduce(cnt)
        self.counts = cnt
        return self

    def probabilities(self, scaled: bool = False) -> torch.Tensor:
        """[C, S, S]: float rows (default) or integer rows scaled by ``scale``."""
        if scaled:
            return normalize_rows(self.counts, self.scale, self.laplace)
        return normalize_rows(self.counts, 1, self.laplace)

    def model_lines(self, delim: str = ",") -> list[str]:
        lines = [delim.join(self.states)]
        P = self.probabilities(scaled=self.scale > 1).cpu()
        for c in range(P.shape[0]):
            if self.class_labels and P.shape[0] > 1:
                lines.append(f"classLabel:{self.class_labels[c]}")
            for r in range(P.shape[1]):
                lines.append(delim.join(str(int(x)) if self.scale > 1 else f"{float(x):.6f}" for x in P[c, r]))
        return lines

    def save(self, path: str | Path, delim: str = ",") -> None:
        Path(path).write_text("\n".join(self.model_lines(delim)) + "\n")

    @staticmethod
    def load_matrices(path: str | Path, delim: str = ",") -> tuple[list[str], dict[str, torch.Tensor]]:
        """Read the model file (MarkovModel): states line, then optional ``classLabel:X`` blocks of S
        rows.  Returns (states, {label or "": [S, S] float probabilities})."""
        lines = [ln for ln in Path(path).read_text().splitlines() if ln.strip()]
        states = lines[0].split(delim)
        S = len(states)
        mats, cur, rows = {}, "", []
        for ln in lines[1:]:
            if ln.startswith("classLabel:"):
                if rows:
                    mats[cur] = torch.tensor(rows, dtype=torch.float64)
                cur, rows = ln.split(":", 1)[1], []
            else:
                rows.append([float(x) for x in ln.split(delim)])
        if rows:
            mats[cur] = torch.tensor(rows, dtype=torch.float64)
        for k, m in mats.items():
            if m.shape != (S, S):
                raise ValueError(f"bad matrix shape {tuple(m.shape)} for {k!r}")
            rs = m.sum(1, keepdim=True)
            mats[k] = m / rs.clamp_min(1e-300)
        return states, mats


class MarkovModelClassifier:
    """log-odds = sum log(P0(s->s') / P1(s->s')); predict class0 when log-odds > threshold."""

    def __init__(self, P0: torch.Tensor, P1: torch.Tensor, class_labels: list[str], threshold: float = 0.0):
        self.lr = (torch.log(P0.double().clamp_min(1e-300)) - torch.log(P1.double().clamp_min(1e-300))).float()
        self.labels = class_labels
        self.threshold = threshold

    def log_odds(self, states: torch.Tensor) -> torch.Tensor:
        return SO.markov_logodds(states, self.lr.to(states.device))

    def predict(self, states: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        lo = self.log_odds(states)
        return (lo <= self.threshold).long(), lo   # 0 -> class_labels[0]


# ================================================================================================
# hidden Markov models
# ================================================================================================
@dataclass
class HiddenMarkovModel:
    states: list[str]
    observations: list[str]
    A: torch.Tensor          # [S, S]
    B: torch.Tensor          # [S, O]
    pi: torch.Tensor         # [S]

    def log_params(self, device=None):
        dev = device or self.A.device
        f = lambda x: torch.log(x.double().clamp_min(1e-300)).float().to(dev)
        return f(self.A), f(self.B), f(self.pi)

    def to_lines(self, delim: str = ",", scale: int = 1) -> list[str]:
        """HiddenMarkovModelBuilder output: states, observations, S transition rows, S emission
        rows, 1 initial-state row."""
        fmt = (lambda x: str(int(round(float(x) * scale)))) if scale > 1 else (lambda x: f"{float(x):.6f}")
        lines = [delim.join(self.states), delim.join(self.observations)]
        lines += [delim.join(fmt(x) for x in row) for row in self.A.cpu()]
        lines += [delim.join(fmt(x) for x in row) for row in self.B.cpu()]
        lines.append(delim.join(fmt(x) for x in self.pi.cpu()))
        return lines

    @classmethod
    def from_lines(cls, lines: list[str], delim: str = ",") -> "HiddenMarkovModel":
        lines = [ln for ln in lines if ln.strip()]
        st, ob = lines[0].split(delim), lines[1].split(delim)
        S = len(st)
        num = lambda ln: [float(x) for x in ln.split(delim)]
        A = torch.tensor([num(x) for x in lines[2:2 + S]], dtype=torch.float64)
        B = torch.tensor([num(x) for x in lines[2 + S:2 + 2 * S]], dtype=torch.float64)
        pi = torch.tensor(num(lines[2 + 2 * S]), dtype=torch.float64)
        norm = lambda m: m / m.sum(-1, keepdim=True).clamp_min(1e-300)
        return cls(st, ob, norm(A), norm(B), norm(pi))


class HiddenMarkovModelBuilder:
    """Supervised HMM estimation from fully tagged ``obs:state`` sequences."""

    def __init__(self, states: list[str], observations: list[str], laplace: bool = True,
                 comm: Comm | None = None):
        self.states, self.observations = states, observations
        self.laplace = laplace
        self.comm = comm

    def encode(self, tagged: list[list[str]], sub_delim: str = ":") -> tuple[torch.Tensor, torch.Tensor]:
        si = {s: i for i, s in enumerate(self.states)}
        oi = {o: i for i, o in enumerate(self.observations)}
        L = max((len(x) for x in tagged), default=0)
        obs = torch.full((len(tagged), L), -1, dtype=torch.int16)
        st = torch.full((len(tagged), L), -1, dtype=torch.int16)
        for r, seq in enumerate(tagged):
            for j, tok in enumerate(seq):
                o, s = tok.split(sub_delim)
                obs[r, j], st[r, j] = oi.get(o, -1), si.get(s, -1)
        return obs, st

    def counts(self, obs: torch.Tensor, st: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """This rank's (transition [S, S], emission [S, O], initial [S]) counts (int64)."""
        S, O = len(self.states), len(self.observations)
        trans = H.bigram_histogram(st, S)[0]
        s, o = st.long(), obs.long()
        ok = (s >= 0) & (o >= 0) & (s < S) & (o < O)
        emit = torch.bincount((s[ok] * O + o[ok]), minlength=S * O)[: S * O].view(S, O)
        first = s[:, 0] if s.shape[1] else s.new_zeros(0)
        init = torch.bincount(first[(first >= 0) & (first < S)], minlength=S)[:S]
        return trans.long(), emit.long().to(trans.device), init.long().to(trans.device)

    def partially_tagged_counts(self, rows: list[list[str]], window: list[int]):
        """Partially tagged sequences (HiddenMarkovModelBuilder.java:174-260): state tokens sit
        among the observations; each state's emission counts are spread over the observations to
        its left and right within a boundary, weighted by ``window[k]`` at distance k+1 (last
        weight repeated).  Boundaries reproduce the reference's integer arithmetic exactly,
        including its operator precedence (``s_i - s_{i-1} / 2``).  The (state, obs, weight)
        triples of all rows become one scatter-add."""
        S, O = len(self.states), len(self.observations)
        si = {s: i for i, s in enumerate(self.states)}
        oi = {o: i for i, o in enumerate(self.observations)}
        ts, to, tw, tr_a, tr_b, init = [], [], [], [], [], []
        wl = len(window)
        for items in rows:
            idx = [i for i, tok in enumerate(items) if tok in si]
            if not idx:
                continue
            init.append(si[items[idx[0]]])
            n = len(items)
            for i, p in enumerate(idx):
                lw = rw = 0
                if i > 0:
                    lw = p - idx[i - 1] // 2
                    lb = p - lw
                else:
                    lb = -1
                if i < len(idx) - 1:
                    rw = idx[i + 1] - p // 2
                    rb = p + rw
                else:
                    rb = -1
                if lb == -1 and rb != -1:
                    lb = max(p - rw, 0)
                elif rb == -1 and lb != -1:
                    rb = min(p + lw, n - 1)
                elif lb == -1 and rb == -1:
                    lb = p // 2
                    rb = p + (n - 1 - p) // 2
                st = si[items[p]]
                for k, j in enumerate(range(p - 1, lb - 1, -1)):
                    if j < 0 or j >= n:
                        continue
                    if items[j] in oi:
                        ts.append(st), to.append(oi[items[j]]), tw.append(window[min(k, wl - 1)])
                for k, j in enumerate(range(p + 1, rb + 1)):
                    if j < 0 or j >= n:
                        continue
                    if items[j] in oi:
                        ts.append(st), to.append(oi[items[j]]), tw.append(window[min(k, wl - 1)])
            for a, b in zip(idx[:-1], idx[1:]):
                tr_a.append(si[items[a]]), tr_b.append(si[items[b]])
        emit = torch.zeros(S * O, dtype=torch.long).index_add_(
            0, torch.tensor(ts, dtype=torch.long) * O + torch.tensor(to, dtype=torch.long),
            torch.tensor(tw, dtype=torch.long)).view(S, O)
        trans = torch.bincount(torch.tensor(tr_a, dtype=torch.long) * S + torch.tensor(tr_b, dtype=torch.long),
                               minlength=S * S)[: S * S].view(S, S)
        ini = torch.bincount(torch.tensor(init, dtype=torch.long), minlength=S)[:S]
        return trans, emit, ini

    def partially_tagged_counts_tokens(self, off: torch.Tensor, st_tok: torch.Tensor, ob_tok: torch.Tensor,
                                       window: list[int]):
        """:meth:`partially_tagged_counts` over a CSR token table on its device: ``off`` [L+1]
        line offsets, ``st_tok`` / ``ob_tok`` [T] state / observation index of every token (-1
        when the token is not one).  The per-state left / right emission windows are expanded
        into (state, observation, weight) triples with one ``repeat_interleave`` and scattered
        once; no per-line Python loop (same integer boundary arithmetic as the list version)."""
        S, O = len(self.states), len(self.observations)
        dev = st_tok.device
        L = off.numel() - 1
        lens = off[1:] - off[:-1]
        tl = torch.repeat_interleave(torch.arange(L, device=dev), lens)
        pos = torch.arange(st_tok.numel(), device=dev) - off[:-1][tl]
        ks = torch.nonzero(st_tok >= 0).view(-1)
        z = torch.zeros(0, dtype=torch.long, device=dev)
        if ks.numel() == 0:
            return (torch.zeros((S, S), dtype=torch.long, device=dev), torch.zeros((S, O), dtype=torch.long, device=dev),
                    torch.zeros(S, dtype=torch.long, device=dev))
        ln, p, sv = tl[ks], pos[ks], st_tok[ks].long()
        nn = lens[ln]
        f = torch.zeros(1, dtype=torch.bool, device=dev)
        prev_same = torch.cat([f, ln[1:] == ln[:-1]])
        next_same = torch.cat([ln[1:] == ln[:-1], f])
        p_prev = torch.cat([z.new_zeros(1), p[:-1]])
        p_next = torch.cat([p[1:], z.new_zeros(1)])
        neg = torch.full_like(p, -1)
        lw = torch.where(prev_same, p - torch.div(p_prev, 2, rounding_mode="floor"), torch.zeros_like(p))
        lb = torch.where(prev_same, p - lw, neg)
        rw = torch.where(next_same, p_next - torch.div(p, 2, rounding_mode="floor"), torch.zeros_like(p))
        rb = torch.where(next_same, p + rw, neg)
        c1 = (lb == -1) & (rb != -1)
        c2 = (rb == -1) & (lb != -1)
        c3 = (lb == -1) & (rb == -1)
        lb = torch.where(c1, (p - rw).clamp_min(0), lb)
        rb = torch.where(c2, torch.minimum(p + lw, nn - 1), rb)
        lb = torch.where(c3, torch.div(p, 2, rounding_mode="floor"), lb)
        rb = torch.where(c3, p + torch.div(nn - 1 - p, 2, rounding_mode="floor"), rb)
        n_left = (p - lb.clamp_min(0)).clamp_min(0)
        n_right = (torch.minimum(rb, nn - 1) - p).clamp_min(0)
        tot = n_left + n_right
        rep = torch.repeat_interleave(torch.arange(ks.numel(), device=dev), tot)
        start = torch.cumsum(tot, 0) - tot
        t = torch.arange(rep.numel(), device=dev) - start[rep]
        left = t < n_left[rep]
        j = torch.where(left, p[rep] - 1 - t, p[rep] + 1 + (t - n_left[rep]))
        k = torch.where(left, t, t - n_left[rep])
        w = torch.tensor(window, dtype=torch.long, device=dev)[k.clamp_max(len(window) - 1)]
        ob = ob_tok[off[:-1][ln[rep]] + j].long()
        ok = ob >= 0
        emit = torch.zeros(S * O, dtype=torch.long, device=dev).index_add_(0, sv[rep][ok] * O + ob[ok], w[ok]).view(S, O)
        a, b = sv[:-1][prev_same[1:]], sv[1:][prev_same[1:]]
        trans = torch.bincount(a * S + b, minlength=S * S)[: S * S].view(S, S)
        ini = torch.bincount(sv[~prev_same], minlength=S)[:S]
        return trans, emit, ini

    def fit(self, obs: torch.Tensor, st: torch.Tensor) -> HiddenMarkovModel:
        trans, emit, init = self.counts(obs, st)
        comm = self.comm or get_comm()
        if comm.is_distributed:
            for x in (trans, emit, init):
                comm.all_reduce(x)
        A = normalize_rows(trans, 1, self.laplace)
        B = normalize_rows(emit, 1, self.laplace)
        pi = normalize_rows(init.view(1, -1), 1, self.laplace)[0]
        return HiddenMarkovModel(self.states, self.observations, A, B, pi)


class ViterbiDecoder:
    def __init__(self, hmm: HiddenMarkovModel):
        self.hmm = hmm

    def decode(self, obs: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        lA, lB, lp = self.hmm.log_params(obs.device)
        return SO.viterbi(obs, lA, lB, lp)

    def decode_long(self, obs: torch.Tensor, chunk: int = 1024, comm=None) -> tuple[torch.Tensor, float]:
        """One long sequence (this rank's segment of it when distributed) by the chunked
        max-plus scan of ``sequence_ops.viterbi_long``: (path, best log score)."""
        lA, lB, lp = self.hmm.log_params(obs.device)
        return SO.viterbi_long(obs, lA, lB, lp, chunk=chunk, comm=comm)

    def log_likelihood(self, obs: torch.Tensor) -> torch.Tensor:
        lA, lB, lp = self.hmm.log_params(obs.device)
        return SO.viterbi(obs, lA, lB, lp, forward=True)[1]

    def decode_labels(self, obs: torch.Tensor) -> list[list[str]]:
        path, _ = self.decode(obs)
        return [[self.hmm.states[int(s)] for s in row if int(s) >= 0] for row in path.cpu()]


# ================================================================================================
# probabilistic suffix tree
# ================================================================================================
@dataclass
class SuffixTreeNode:
    token: int
    count: int = 0
    children: dict = field(default_factory=dict)


class ProbabilisticSuffixTree:
    def __init__(self, n_states: int, max_len: int = 5):
        self.n_states, self.max_len = n_states, max_len
        self.root = SuffixTreeNode(-1)

    def fit(self, states: torch.Tensor, comm: Comm | None = None) -> "ProbabilisticSuffixTree":
        counts = SO.ngram_counts(states, self.n_states, 2, self.max_len)
        comm = comm or get_comm()
        for k, (keys, cnt) in counts.items():
            if comm.is_distributed:  # sparse keys: gather every rank's (key, count) and merge
                keys = comm.all_gather_v(keys)
                cnt = comm.all_gather_v(cnt)
                keys, inv = torch.unique(keys, return_inverse=True)
                cnt = torch.zeros_like(keys).index_add_(0, inv, cnt)
            for key, c in zip(keys.cpu().tolist(), cnt.cpu().tolist()):
                _, seq = SO.decode_ngram(key, k, self.n_states)
                node = self.root
                for tok in seq:
                    node = node.children.setdefault(tok, SuffixTreeNode(tok))
                node.count += c
        self._propagate(self.root)
        self.root.count = sum(ch.count for ch in self.root.children.values())
        return self

    def _propagate(self, node: SuffixTreeNode) -> int:
        # counts of longer n-grams flow up to their prefixes only when the prefix itself was unseen
        for ch in node.children.values():
            sub = self._propagate(ch)
            if ch.count == 0:
                ch.count = sub
        return node.count

    def find(self, seq: list[int]) -> SuffixTreeNode | None:
        node = self.root
        for tok in seq:
            node = node.children.get(tok)
            if node is None:
                return None
        return node

    def next_prob(self, context: list[int]) -> torch.Tensor:
        node = self.find(context)
        p = torch.zeros(self.n_states, dtype=torch.float64)
        if node is None or not node.children:
            return p
        for tok, ch in node.children.items():
            p[tok] = ch.count
        return p / p.sum()


# ================================================================================================
# continuous-time Markov chains
# ================================================================================================
class StateTransitionRate:
    """CTMC rate matrix from (entity, time, state) events: transition counts and dwell times per
    state, q_ij = n_ij / T_i (S/markov/StateTransitionRate.scala:91-167)."""

    def __init__(self, n_states: int):
        self.S = n_states

    def fit(self, entity: torch.Tensor, time: torch.Tensor, state: torch.Tensor) -> torch.Tensor:
        order = torch.argsort(entity.long() * (1 << 40) + time.long() - time.long().min(), stable=True)
        e, t, s = entity[order].long(), time[order].double(), state[order].long()
        same = e[1:] == e[:-1]
        a, b = s[:-1][same], s[1:][same]
        dt = (t[1:] - t[:-1])[same]
        S = self.S
        n = torch.bincount(a * S + b, minlength=S * S)[: S * S].view(S, S).double()
        dwell = torch.zeros(S, dtype=torch.float64, device=s.device).index_add_(0, a, dt)
        Q = n / dwell.clamp_min(1e-300).view(-1, 1)
        Q.fill_diagonal_(0)
        Q -= torch.diag(Q.sum(1))
        self.Q = Q
        return Q

    def fit_grouped(self, key: torch.Tensor, time_ms: torch.Tensor, state: torch.Tensor, n_keys: int,
                    unit_ms: float = 3600_000.0) -> torch.Tensor:
        """One rate matrix per key ``[G, S, S]`` (StateTransitionRate.scala:91-167): sort by
        (key, time), transitions between consecutive events of a key, dwell time of the source
        state in ``unit_ms`` units; off-diagonal q_ij = n_ij / T_i, q_ii = -sum_j q_ij (rows of
        unvisited states stay zero)."""
        k, t, s = key.long(), time_ms.long(), state.long()
        order = torch.argsort(t, stable=True)
        order = order[torch.argsort(k[order], stable=True)]
        k, t, s = k[order], t[order].double(), s[order]
        same = k[1:] == k[:-1]
        g, a, b = k[:-1][same], s[:-1][same], s[1:][same]
        dt = (t[1:] - t[:-1])[same] / unit_ms
        S, G = self.S, n_keys
        n = torch.zeros(G * S * S, dtype=torch.float64, device=s.device).index_add_(
            0, (g * S + a) * S + b, torch.ones_like(dt)).view(G, S, S)
        dwell = torch.zeros(G * S, dtype=torch.float64, device=s.device).index_add_(0, g * S + a, dt).view(G, S)
        Q = torch.where(dwell.unsqueeze(2) > 0, n / dwell.clamp_min(1e-300).unsqueeze(2), torch.zeros_like(n))
        eye = torch.eye(S, dtype=torch.bool, device=s.device)
        off = Q.masked_fill(eye, 0.0).sum(2)
        Q = torch.where(eye, -off.unsqueeze(2).expand_as(Q), Q)
        self.Q = Q
        return Q


class ContTimeStateTransitionStats:
    """Uniformisation: P = I + Q/lambda, powers P^0..P^L with L = 4 + 6 sqrt(lambda t) + lambda t
    (S/markov/ContTimeStateTransitionStats.scala:96-236)."""

    def __init__(self, Q: torch.Tensor):
        self.Q = Q.double()
        self.lam = float((-torch.diagonal(self.Q)).max())
        S = Q.shape[0]
        self.P = torch.eye(S, dtype=torch.float64, device=Q.device) + self.Q / max(self.lam, 1e-300)

    def _weights(self, t: float) -> tuple[int, torch.Tensor, torch.Tensor]:
        """Truncation L = 4 + 6 sqrt(lt) + lt and the Poisson weights w_k and tails P(N > k)."""
        lt = self.lam * t
        L = int(4 + 6 * math.sqrt(lt) + lt)
        k = torch.arange(L + 1, dtype=torch.float64)
        w = torch.exp(-lt + k * math.log(max(lt, 1e-300)) - torch.lgamma(k + 1))
        tail = (1.0 - torch.cumsum(w, 0)).clamp_min(0)
        return L, w, tail

    def sums(self, times: list[float]) -> tuple[torch.Tensor, torch.Tensor]:
        """For every t: (future-state probabilities [S, S], expected dwell times [S, S]) from ONE
        batched power-chain launch (K16); P^k is never materialised in HBM."""
        ws = [self._weights(t) for t in times]
        ldw = max(L for L, _, _ in ws) + 1
        w1 = torch.zeros((len(times), ldw), dtype=torch.float64)
        w2 = torch.zeros_like(w1)
        for b, (L, w, tail) in enumerate(ws):
            w1[b, : L + 1] = w
            w2[b, : L + 1] = tail
        dev = self.P.device
        A, B = SO.uniformization_sums(self.P, w1.to(dev), w2.to(dev), [L for L, _, _ in ws])
        return A, B / self.lam

    def future_state_prob(self, t: float) -> torch.Tensor:
        """[S, S]: P(X(t) = j | X(0) = i) = sum_k Poisson(k; lt) (P^k)_ij."""
        return self.sums([t])[0][0]

    def state_dwell_time(self, t: float) -> torch.Tensor:
        """[S, S]: expected time spent in j over [0, t] starting in i
        = (1/lambda) sum_k P(N > k) (P^k)_ij, N ~ Poisson(lt)."""
        return self.sums([t])[1][0]

    def transition_count(self, t: float) -> torch.Tensor:
        """[S, S, S]: expected number of i->j transitions over [0, t] from start state s
        (dwell time in i x q_ij)."""
        dw = self.state_dwell_time(t)          # [s, i]
        Qo = self.Q.clone()
        Qo.fill_diagonal_(0)
        return dw.unsqueeze(2) * Qo.unsqueeze(0)


# ================================================================================================
# sequence mining
# ================================================================================================
def sequence_generator(key: torch.Tensor, seq_field: torch.Tensor, value: torch.Tensor):
    """Group records by key and order them by the sequence field (S/sequence/SequenceGenerator):
    returns (sorted keys, sorted values, group boundaries)."""
    k = key.long()
    order = torch.argsort(seq_field.long(), stable=True)
    order = order[torch.argsort(k[order], stable=True)]
    ks = k[order]
    starts = torch.nonzero(torch.cat([torch.ones(1, dtype=torch.bool, device=ks.device), ks[1:] != ks[:-1]])).squeeze(1)
    return ks, value[order], starts


class TimeDelayEmbedding:
    """Histogram of length-w symbol windows per key (S/sequence/TimeDelayEmbeddingModel)."""

    def __init__(self, n_symbols: int, window: int):
        self.S, self.w = n_symbols, window

    def fit(self, states: torch.Tensor, group: torch.Tensor | None = None):
        return SO.ngram_counts(states, self.S, self.w, self.w, group)[self.w]


def gsp_candidates(freq: list[tuple[int, ...]]) -> list[tuple[int, ...]]:
    """GSP k+1 candidates: join a and b when a[1:] == b[:-1] (J/sequence/CandidateGenerationWithSelfJoin
    :243-276).  Hash join on the (k-1)-overlap instead of bucket-pair replication."""
    by_prefix: dict[tuple, list[tuple]] = {}
    for s in freq:
        by_prefix.setdefault(s[:-1], []).append(s)
    out = set()
    for a in freq:
        for b in by_prefix.get(a[1:], []):
            out.add(a + (b[-1],))
    return sorted(out)


def gsp_candidates_device(seqs: list[tuple[str, ...]], device="cpu", comm: Comm | None = None) -> list[tuple[str, ...]]:
    """GSP k+1 candidates of a set of frequent k-sequences of string tokens, on the device
    (``SO.gsp_join``); distributed: each rank joins its shard of left sequences against all of
    them and rank 0 receives the union (sorted, unique)."""
    comm = comm or get_comm()
    seqs = sorted(set(seqs))
    if not seqs:
        return []
    k = len(seqs[0])
    vocab = sorted({t for s in seqs for t in s})
    ti = {t: i for i, t in enumerate(vocab)}
    X = torch.tensor([[ti[t] for t in s] for s in seqs], dtype=torch.int32, device=device)
    lo, hi = 0, X.shape[0]
    if comm.is_distributed:
        from ..data.table import shard_range
        lo, hi = shard_range(X.shape[0], comm.rank, comm.world)
    C = SO.gsp_join(X, lo, hi)
    if comm.is_distributed:
        C = comm.all_gather_v(C.cpu() if comm.backend == "gloo" else C)
    C = unique_rows(C.cpu()) if C.numel() else C.cpu().view(0, k + 1)
    return [tuple(vocab[i] for i in row) for row in C.tolist()]


def dot_matrix_similarity(A: torch.Tensor, B: torch.Tensor, window: int = 3) -> torch.Tensor:
    """Dot-matrix window matching score for every pair of sequences (S/sequence/DotMatrixMatching
    :176-252): number of (i, j) positions where the length-``window`` sub-sequences match, normalised
    by the number of windows.  A [n, L], B [m, L'] int (negative = padding)."""
    wa = A.long().unfold(1, window, 1)      # [n, La, w]
    wb = B.long().unfold(1, window, 1)      # [m, Lb, w]
    va = (wa >= 0).all(-1)
    vb = (wb >= 0).all(-1)
    # dense window ids shared by both sides (exact: no hashing), -1 for windows with padding
    allw = torch.cat([wa.reshape(-1, window), wb.reshape(-1, window)])
    _, inv = unique_rows(allw, True)
    ida = torch.where(va, inv[: wa.shape[0] * wa.shape[1]].view(va.shape), torch.full_like(va, -1, dtype=torch.long))
    idb = torch.where(vb, inv[wa.shape[0] * wa.shape[1]:].view(vb.shape), torch.full_like(vb, -1, dtype=torch.long))
    hits = SO.dot_matrix_hits(ida.to(torch.int32), idb.to(torch.int32)).double()
    denom = (va.sum(1).view(-1, 1) * vb.sum(1).view(1, -1)).clamp_min(1).double().sqrt()
    return hits / denom


def positional_event_clusters(times: torch.Tensor, flags: torch.Tensor, window: float, min_count: int) -> torch.Tensor:
    """Time-bounded event locality (J/sequence/SequencePositionalCluster): for each event, number of
    condition-matching events within +-window; returns a boolean "in cluster" mask."""
    t = times.double()
    order = torch.argsort(t)
    ts, fs = t[order], flags[order].long()
    cs = torch.cumsum(fs, 0)
    lo = torch.searchsorted(ts, ts - window, right=False)
    hi = torch.searchsorted(ts, ts + window, right=True) - 1
    cnt = cs[hi] - torch.where(lo > 0, cs[(lo - 1).clamp_min(0)], torch.zeros_like(lo))
    out = torch.zeros_like(flags, dtype=torch.bool)
    out[order] = cnt >= min_count
    return out
