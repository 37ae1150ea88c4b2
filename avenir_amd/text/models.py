"""Text models: extractive summarisers, LDA topics, word / document vectors, NB text classifier.

Reference: P/text/summ.py:41-619 (TermFreqSumm, SumBasicSumm, LatentSemSumm via gensim LSI,
NonNegMatFactSumm via sklearn NMF, TextRankSumm via networkx pagerank, EmbeddingTextRankSumm,
MaxMarginalRelevance), P/text/lda.py:35-306 (gensim LDA), P/text/wv.py + dv.py (gensim word2vec /
doc2vec), P/text/process.py:33-76 (nltk NaiveBayes text classifier).

MI355X design: every summariser works on the device sentence-term matrix: LSA = one SVD, NMF =
multiplicative updates (2 GEMMs per step), TextRank = cosine-similarity GEMM + power-iteration
pagerank, MMR = similarity GEMM + greedy selection; LDA is batch variational Bayes whose E and M
steps are GEMMs over the doc-term matrix; word2vec is skip-gram with negative sampling trained
in large device batches.
"""
from __future__ import annotations

import math
from collections import Counter
from typing import Sequence

import torch

from .preprocess import DocSentences, TfIdf, Vocabulary, clean_tokens, cosine_similarity_matrix, doc_term_matrix


# ================================================================================================
# summarisers
# ================================================================================================
def _sent_matrix(tokens: Sequence[Sequence[str]], device="cpu", normalized: bool = True) -> torch.Tensor:
    vocab = Vocabulary(tokens)
    X = doc_term_matrix(tokens, vocab, device).to_dense()
    if normalized:
        X = X / X.sum(1, keepdim=True).clamp_min(1e-12)
    return X


def max_marginal_relevance(vecs: torch.Tensor, scores: torch.Tensor, k: int, reg: float = 0.7,
                           aggr: str = "average") -> list[tuple[int, float]]:
    """Greedy MMR (summ.py:565-619): score' = reg * score/max + (1 - reg) * aggr(cosine distance to
    already selected).  Returns [(index, mmr score)] in document order."""
    s = scores.double() / scores.max().clamp_min(1e-300)
    dist = 1 - cosine_similarity_matrix(vecs.double())
    chosen: list[tuple[int, float]] = []
    avail = torch.ones(len(s), dtype=torch.bool, device=s.device)
    for _ in range(min(k, len(s))):
        if chosen:
            d = dist[:, [c for c, _ in chosen]]
            div = {"max": d.max(1).values, "min": d.min(1).values, "average": d.mean(1)}[aggr]
        else:
            div = torch.zeros_like(s)
        sc = torch.where(avail, reg * s + (1 - reg) * div, torch.full_like(s, -1e300))
        j = int(sc.argmax())
        chosen.append((j, float(sc[j])))
        avail[j] = False
    return sorted(chosen)


class Summarizer:
    """Common front end: ``summarize(text or path) -> [(sentence, score)]`` in document order.
    ``size`` sentences (``by_count``) or ``size`` percent of the sentences."""

    def __init__(self, size: int = 5, by_count: bool = True, min_sentence_length: int = 5, device="cpu",
                 diversify: bool = False, reg: float = 0.7, aggr: str = "average"):
        self.size, self.by_count, self.min_len, self.device = size, by_count, min_sentence_length, device
        self.diversify, self.reg, self.aggr = diversify, reg, aggr

    def _prepare(self, path=None, text=None):
        ds = DocSentences(path, self.min_len, False, text)
        sents, toks = ds.getSentences(), ds.getSentencesAsTokens()
        k = self.size if self.by_count else max(1, int(len(sents) * self.size / 100))
        return sents, toks, k

    def scores(self, toks) -> torch.Tensor:
        raise NotImplementedError

    def summarize(self, path=None, text=None) -> list[tuple[str, float]]:
        sents, toks, k = self._prepare(path, text)
        if len(sents) <= k:
            return [(s, 1.0) for s in sents]
        sc = self.scores(toks)
        if self.diversify:
            sel = max_marginal_relevance(_sent_matrix(toks, self.device), sc, k, self.reg, self.aggr)
            return [(sents[i], v) for i, v in sel]
        top = torch.argsort(sc, descending=True)[:k].tolist()
        return [(sents[i], float(sc[i])) for i in sorted(top)]

    getSummary = summarize


class TermFreqSumm(Summarizer):
    """Sentence score = sum of corpus term counts of its words / length ("linear") or
    count * 1/(1 + ln(len/minlen)) ("log")."""

    def __init__(self, normalizer: str = "linear", **kw):
        super().__init__(**kw)
        self.normalizer = normalizer

    def scores(self, toks):
        X = _sent_matrix(toks, self.device, normalized=False)
        counts = X.sum(0)
        tot = X @ counts
        lens = torch.tensor([len(t) for t in toks], dtype=torch.float32, device=X.device)
        if self.normalizer == "linear":
            return tot / lens
        if self.normalizer == "log":
            return torch.floor(tot * (1.0 / (1.0 + torch.log(lens / lens.min()))))
        return tot


class SumBasicSumm(Summarizer):
    """SumBasic: repeatedly take the sentence with the highest mean word probability, then square
    the probabilities of its words."""

    def summarize(self, path=None, text=None):
        sents, toks, k = self._prepare(path, text)
        if len(sents) <= k:
            return [(s, 1.0) for s in sents]
        X = _sent_matrix(toks, self.device, normalized=False)
        p = X.sum(0) / X.sum()
        lens = (X.sum(1)).clamp_min(1)
        avail = torch.ones(len(sents), dtype=torch.bool, device=X.device)
        out = []
        for _ in range(k):
            sc = torch.where(avail, (X @ p) / lens, torch.full_like(lens, -1.0))
            j = int(sc.argmax())
            out.append((j, float(sc[j])))
            avail[j] = False
            used = X[j] > 0
            p = torch.where(used, p * p, p)
        return [(sents[i], v) for i, v in sorted(out)]

    getSummary = summarize


class LatentSemSumm(Summarizer):
    """LSA: SVD of the sentence-term matrix; for summary slot i take, topic by topic, the sentence
    with the i-th largest |loading| not yet chosen (selTopSents, summ.py:106-121)."""

    def __init__(self, num_topics: int = 5, **kw):
        super().__init__(**kw)
        self.num_topics = num_topics

    def _loadings(self, X):
        U, S, Vh = torch.linalg.svd(X, full_matrices=False)
        return (U[:, : self.num_topics] * S[: self.num_topics]).abs()          # [n_sent, T]

    def summarize(self, path=None, text=None):
        sents, toks, k = self._prepare(path, text)
        if len(sents) <= k:
            return [(s, 1.0) for s in sents]
        L = self._loadings(_sent_matrix(toks, self.device, normalized=False))
        T = L.shape[1]
        order = torch.argsort(L, 0, descending=True)
        chosen: dict[int, float] = {}
        for i in range(L.shape[0]):
            for t in range(T):
                s = int(order[i, t])
                if s not in chosen:
                    chosen[s] = float(L[s, t])
                    if len(chosen) == k:
                        return [(sents[j], chosen[j]) for j in sorted(chosen)]
        return [(sents[j], chosen[j]) for j in sorted(chosen)]

    getSummary = summarize


def nmf(X: torch.Tensor, k: int, iters: int = 200, seed: int = 0, eps: float = 1e-10):
    """Lee-Seung multiplicative-update NMF, X ~ W H (Frobenius loss), all GEMMs on X's device."""
    g = torch.Generator(device=X.device).manual_seed(seed)
    n, m = X.shape
    scale = math.sqrt(float(X.mean()) / k) if float(X.mean()) > 0 else 1.0
    W = torch.rand((n, k), device=X.device, generator=g) * scale
    H = torch.rand((k, m), device=X.device, generator=g) * scale
    for _ in range(iters):
        H *= (W.T @ X) / (W.T @ W @ H + eps)
        W *= (X @ H.T) / (W @ (H @ H.T) + eps)
    return W, H


class NonNegMatFactSumm(LatentSemSumm):
    def __init__(self, num_topics: int = 5, iters: int = 200, **kw):
        super().__init__(num_topics, **kw)
        self.iters = iters

    def _loadings(self, X):
        W, _ = nmf(X, self.num_topics, self.iters)
        return W


# one persistent workgroup sweeps P per iteration below this size; above it the multi-workgroup
# kernels win (MI355X: 0.07 vs 0.25 ms at n = 256, 0.67 vs 0.24 ms at 1024, 2.6 vs 0.29 ms at 2048)
PAGERANK_KERNEL_MAX_N = 768


def pagerank(S: torch.Tensor, d: float = 0.85, iters: int = 100, tol: float = 1e-10) -> torch.Tensor:
    """Weighted pagerank by power iteration on a similarity matrix (dangling rows -> uniform).
    GPU, n <= 768: the whole iteration in one persistent kernel (text.hip pagerank_kernel, no host
    synchronisation per iteration); larger n: the multi-workgroup kernels (pagerank_multi); CPU:
    tensor GEMVs."""
    n = S.shape[0]
    out = S.sum(1, keepdim=True)
    P = torch.where(out > 0, S / out.clamp_min(1e-300), torch.full_like(S, 1.0 / n))
    if S.is_cuda and 0 < n <= PAGERANK_KERNEL_MAX_N:
        from .. import _native
        r, _ = _native.C().pagerank(P.double().contiguous(), float(d), int(iters), float(tol))
        return r.to(S.dtype)
    if S.is_cuda and n > 0:
        # larger graphs: several workgroups per iteration, every iteration enqueued up front with a
        # device-side convergence flag (one host read at the end)
        from .. import _native
        r, _ = _native.C().pagerank_multi(P.double().contiguous(), float(d), int(iters), float(tol))
        return r.to(S.dtype)
    r = torch.full((n,), 1.0 / n, dtype=S.dtype, device=S.device)
    for _ in range(iters):
        nr = (1 - d) / n + d * (P.T @ r)
        if float((nr - r).abs().sum()) < tol:
            r = nr
            break
        r = nr
    return r


class TextRankSumm(Summarizer):
    def scores(self, toks):
        X = _sent_matrix(toks, self.device)
        S = cosine_similarity_matrix(X.double())
        S.fill_diagonal_(0)
        return pagerank(S).float()


class EmbeddingTextRankSumm(Summarizer):
    """TextRank over sentence embeddings = mean of word vectors (``embeddings`` dict or a
    :class:`Word2Vec` model)."""

    def __init__(self, embeddings, **kw):
        super().__init__(**kw)
        self.emb = embeddings

    def _vec(self, w):
        if isinstance(self.emb, Word2Vec):
            return self.emb.vector(w)
        v = self.emb.get(w)
        return None if v is None else torch.as_tensor(v, dtype=torch.float32)

    def scores(self, toks):
        vecs = []
        for t in toks:
            vs = [v for v in (self._vec(w) for w in t) if v is not None]
            vecs.append(torch.stack(vs).mean(0) if vs else None)
        dim = next(v.shape[0] for v in vecs if v is not None)
        E = torch.stack([v if v is not None else torch.zeros(dim) for v in vecs]).double()
        S = cosine_similarity_matrix(E).clamp_min(0)
        S.fill_diagonal_(0)
        return pagerank(S).float()


# ================================================================================================
# LDA (batch variational Bayes, GEMM form)
# ================================================================================================
class LatentDirichletAllocation:
    def __init__(self, num_topics: int = 10, alpha: float | None = None, eta: float | None = None, iters: int = 50,
                 e_steps: int = 20, seed: int = 0, device="cpu"):
        self.K, self.iters, self.e_steps, self.seed, self.device = num_topics, iters, e_steps, seed, device
        self.alpha = alpha if alpha is not None else 1.0 / num_topics
        self.eta = eta if eta is not None else 1.0 / num_topics
        self.vocab: Vocabulary | None = None

    def fit(self, docs: Sequence[Sequence[str]], min_count: int = 1) -> "LatentDirichletAllocation":
        self.vocab = Vocabulary(docs, min_count)
        X = doc_term_matrix(docs, self.vocab, self.device).to_dense().double()
        D, V = X.shape
        g = torch.Generator(device=X.device).manual_seed(self.seed)
        # near-Gamma(100, 1/100) initialisation (Hoffman et al. 2010): 1 + N(0, 0.1)
        lam = (1.0 + 0.1 * torch.randn((self.K, V), dtype=torch.float64, device=X.device, generator=g)).clamp_min(0.5)
        gamma = torch.ones((D, self.K), dtype=torch.float64, device=X.device)
        for _ in range(self.iters):
            Elogbeta = torch.digamma(lam) - torch.digamma(lam.sum(1, keepdim=True))
            expElogbeta = Elogbeta.exp()
            for _ in range(self.e_steps):
                Elogtheta = torch.digamma(gamma) - torch.digamma(gamma.sum(1, keepdim=True))
                expElogtheta = Elogtheta.exp()
                phinorm = expElogtheta @ expElogbeta + 1e-100
                gamma = self.alpha + expElogtheta * ((X / phinorm) @ expElogbeta.T)
            Elogtheta = torch.digamma(gamma) - torch.digamma(gamma.sum(1, keepdim=True))
            expElogtheta = Elogtheta.exp()
            phinorm = expElogtheta @ expElogbeta + 1e-100
            lam = self.eta + expElogbeta * (expElogtheta.T @ (X / phinorm))
        self.lam, self.gamma = lam, gamma
        return self

    def topic_term(self) -> torch.Tensor:
        return self.lam / self.lam.sum(1, keepdim=True)

    def doc_topic(self) -> torch.Tensor:
        return self.gamma / self.gamma.sum(1, keepdim=True)

    def top_terms(self, topic: int, n: int = 10) -> list[tuple[str, float]]:
        tt = self.topic_term()[topic]
        words = self.vocab.words
        idx = torch.argsort(tt, descending=True)[:n].tolist()
        return [(words[i], float(tt[i])) for i in idx]

    def transform(self, docs: Sequence[Sequence[str]], e_steps: int = 50) -> torch.Tensor:
        X = doc_term_matrix(docs, self.vocab, self.device).to_dense().double()
        Elogbeta = torch.digamma(self.lam) - torch.digamma(self.lam.sum(1, keepdim=True))
        expElogbeta = Elogbeta.exp()
        gamma = torch.ones((X.shape[0], self.K), dtype=torch.float64, device=X.device)
        for _ in range(e_steps):
            expElogtheta = (torch.digamma(gamma) - torch.digamma(gamma.sum(1, keepdim=True))).exp()
            gamma = self.alpha + expElogtheta * ((X / (expElogtheta @ expElogbeta + 1e-100)) @ expElogbeta.T)
        return gamma / gamma.sum(1, keepdim=True)


# ================================================================================================
# word2vec (skip-gram, negative sampling) and doc2vec (PV-DBOW)
# ================================================================================================
def _row_mean_add(M: torch.Tensor, rows: torch.Tensor, upd: torch.Tensor, mean: bool = True) -> None:
    """M[r] += mean of the batch updates addressed to row r: a large device batch touches a
    frequent word many times, and summing those SGD steps (what sequential Hogwild would apply
    with fresh gradients) diverges; averaging keeps the step size independent of batch size."""
    if not mean:
        M.index_add_(0, rows, upd)
        return
    acc = torch.zeros_like(M).index_add_(0, rows, upd)
    cnt = torch.bincount(rows, minlength=M.shape[0]).clamp_min(1).to(M.dtype)
    M += acc / cnt.unsqueeze(1)


def _alias_table(p: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Vose's alias table of a discrete distribution (host, O(V)): (prob f32 [V], alias i32 [V])."""
    import numpy as np
    q = (p.double().cpu().numpy() * p.numel()).astype(np.float64)
    V = q.size
    prob, alias = np.ones(V), np.arange(V, dtype=np.int64)
    small = [i for i in range(V) if q[i] < 1.0]
    large = [i for i in range(V) if q[i] >= 1.0]
    while small and large:
        s, l = small.pop(), large.pop()
        prob[s], alias[s] = q[s], l
        q[l] -= 1.0 - q[s]
        (small if q[l] < 1.0 else large).append(l)
    return torch.tensor(prob, dtype=torch.float32), torch.tensor(alias, dtype=torch.int32)


def _sgns_dim(d: int) -> int:
    for p in (64, 128, 192, 256):
        if d <= p:
            return p
    return 0


class Word2Vec:
    """Skip-gram with negative sampling, mini-batch SGD with per-row averaged updates (rate
    ``lr``, linear decay).  GPU with dim <= 256: per batch one ``sgns_step`` (text.hip: a
    wavefront per pair, device negatives from an alias table, gradient accumulation + mean apply);
    CPU: the same batches as tensor ops."""

    def __init__(self, dim: int = 100, window: int = 5, negative: int = 5, min_count: int = 1, epochs: int = 5,
                 lr: float = 0.5, batch: int = 4096, seed: int = 0, device="cpu"):
        self.dim, self.window, self.negative, self.min_count = dim, window, negative, min_count
        self.epochs, self.lr, self.batch, self.seed, self.device = epochs, lr, batch, seed, torch.device(device)

    def _pairs(self, ids: list[list[int]]):
        """(centre, context) of every in-sentence window pair, vectorised over the flat corpus."""
        flat = torch.tensor([w for s in ids for w in s], dtype=torch.long)
        sent = torch.tensor([k for k, s in enumerate(ids) for _ in s], dtype=torch.long)
        cen, ctx = [], []
        for off in range(1, self.window + 1):
            ok = sent[off:] == sent[:-off] if flat.numel() > off else torch.zeros(0, dtype=torch.bool)
            a, b = flat[:-off][ok], flat[off:][ok]
            cen += [a, b]
            ctx += [b, a]
        if not cen:
            return torch.zeros(0, dtype=torch.long), torch.zeros(0, dtype=torch.long)
        return torch.cat(cen), torch.cat(ctx)

    def _use_kernel(self) -> bool:
        return self.device.type == "cuda" and _sgns_dim(self.dim) > 0

    def _fit_kernel(self, Win: torch.Tensor, Wout: torch.Tensor, cen: torch.Tensor, ctx: torch.Tensor,
                    mean_in: bool = True, decay_per_batch: bool = True) -> None:
        """Epochs of device SGNS mini-batches (the tensor path's batches, rate and averaged
        updates): Win [R, dp] / Wout [V, dp] zero-padded beyond ``dim`` (padding coordinates stay
        zero: their gradients are products with zeros)."""
        from .. import _native
        V = Wout.shape[0]
        aprob, alias = _alias_table(self.noise)
        aprob, alias = aprob.to(self.device), alias.to(self.device)
        g = torch.Generator(device=self.device).manual_seed(self.seed)
        n = cen.numel()
        if n:   # ids index the tables: checked once per fit
            assert int(cen.min()) >= 0 and int(cen.max()) < Win.shape[0] and int(ctx.min()) >= 0 and int(ctx.max()) < V
        cen, ctx = cen.to(self.device).int(), ctx.to(self.device).int()
        gIn, gOut = torch.zeros_like(Win), torch.zeros_like(Wout)
        # hot rows (sgns kernels): the H most probable noise words accumulate into R replicas
        R = _native.C().sgns_hot_replicas()
        H = min(V, 256)
        hot = torch.full((V,), -1, dtype=torch.int32, device=self.device)
        hot[torch.topk(self.noise, H).indices] = torch.arange(H, dtype=torch.int32, device=self.device)
        words_in = mean_in and Win.shape[0] == V        # word2vec: the centre table is over word ids
        gOutHot = torch.zeros((R, H, Wout.shape[1]), device=self.device)
        gInHot = torch.zeros_like(gOutHot) if words_in else None
        # ping-pong count buffers: a batch's apply pass clears the other pair for the next batch
        cIns = [torch.zeros(Win.shape[0] + (R * H if words_in else 0), device=self.device) for _ in range(2)]
        cOuts = [torch.zeros(V + R * H, device=self.device) for _ in range(2)]
        nb = max(1, (n + self.batch - 1) // self.batch)
        total, step = self.epochs * nb, 0
        C = _native.C()
        for ep in range(self.epochs):
            perm = torch.randperm(n, device=self.device, generator=g)
            c_ep, o_ep = cen[perm].contiguous(), ctx[perm].contiguous()
            lr_ep = self.lr * (1 - ep / self.epochs)
            for b in range(0, n, self.batch):
                lr = self.lr * max(1e-4, 1 - step / total) if decay_per_batch else lr_ep
                cur, nxt = step & 1, (step + 1) & 1
                C.sgns_step(Win, Wout, gIn, gOut, cIns[cur], cOuts[cur], c_ep[b:b + self.batch],
                            o_ep[b:b + self.batch], aprob, alias, int(self.negative), float(lr), bool(mean_in),
                            int(self.seed), step, hot=hot, gOutHot=gOutHot, gInHot=gInHot, cIn_next=cIns[nxt],
                            cOut_next=cOuts[nxt])
                step += 1

    def fit(self, sentences: Sequence[Sequence[str]]) -> "Word2Vec":
        self.vocab = Vocabulary(sentences, self.min_count)
        V = len(self.vocab)
        ids = [[self.vocab.index[w] for w in s if w in self.vocab.index] for s in sentences]
        cen, ctx = self._pairs(ids)
        cnt = torch.bincount(torch.tensor([w for s in ids for w in s], dtype=torch.long), minlength=V).double()
        self.noise = (cnt ** 0.75 / (cnt ** 0.75).sum()).float().to(self.device)
        g = torch.Generator(device=self.device).manual_seed(self.seed)
        self.W = ((torch.rand((V, self.dim), device=self.device, generator=g) - 0.5) / self.dim)
        self.C = torch.zeros((V, self.dim), device=self.device)
        if self._use_kernel():
            dp = _sgns_dim(self.dim)
            Win = torch.zeros((V, dp), device=self.device)
            Win[:, : self.dim] = self.W
            Wout = torch.zeros((V, dp), device=self.device)
            self._fit_kernel(Win, Wout, cen, ctx)
            self.W, self.C = Win[:, : self.dim].contiguous(), Wout[:, : self.dim].contiguous()
            return self
        cen, ctx = cen.to(self.device), ctx.to(self.device)
        n = cen.numel()
        total = self.epochs * max(1, (n + self.batch - 1) // self.batch)
        step = 0
        for _ in range(self.epochs):
            perm = torch.randperm(n, device=self.device, generator=g)
            for b in range(0, n, self.batch):
                idx = perm[b:b + self.batch]
                c, o = cen[idx], ctx[idx]
                negs = torch.multinomial(self.noise, idx.numel() * self.negative, True, generator=g).view(-1, self.negative)
                lr = self.lr * max(1e-4, 1 - step / total)
                wc = self.W[c]                                                      # [B, d]
                tgt = torch.cat([o.view(-1, 1), negs], 1)                           # [B, 1+neg]
                ct = self.C[tgt]                                                    # [B, 1+neg, d]
                lab = torch.zeros(tgt.shape, device=self.device)
                lab[:, 0] = 1
                gsc = (lab - torch.sigmoid((ct * wc.unsqueeze(1)).sum(2))) * lr     # [B, 1+neg]
                _row_mean_add(self.W, c, (gsc.unsqueeze(2) * ct).sum(1))
                _row_mean_add(self.C, tgt.reshape(-1), (gsc.unsqueeze(2) * wc.unsqueeze(1)).reshape(-1, self.dim))
                step += 1
        return self

    def vector(self, word: str):
        i = self.vocab.index.get(word)
        return None if i is None else self.W[i]

    def most_similar(self, word: str, topn: int = 5) -> list[tuple[str, float]]:
        v = self.vector(word)
        if v is None:
            return []
        sims = cosine_similarity_matrix(v.view(1, -1), self.W)[0]
        sims[self.vocab.index[word]] = -2
        idx = torch.argsort(sims, descending=True)[:topn].tolist()
        words = self.vocab.words
        return [(words[i], float(sims[i])) for i in idx]

    def save(self, path):
        from safetensors.torch import save_file
        save_file({"W": self.W.cpu().contiguous()}, str(path), metadata={"words": "\n".join(self.vocab.words)})

    @classmethod
    def load(cls, path, device="cpu"):
        from safetensors import safe_open
        m = cls(device=device)
        with safe_open(str(path), "pt") as f:
            m.W = f.get_tensor("W").to(device)
            words = f.metadata()["words"].split("\n")
        m.vocab = Vocabulary()
        m.vocab.index = {w: i for i, w in enumerate(words)}
        m.dim = m.W.shape[1]
        return m


class Doc2Vec(Word2Vec):
    """PV-DBOW: a document vector predicts the document's words (negative sampling); word
    vectors are not trained."""

    def fit(self, docs: Sequence[Sequence[str]]) -> "Doc2Vec":
        self.vocab = Vocabulary(docs, self.min_count)
        V, D = len(self.vocab), len(docs)
        ids = [[self.vocab.index[w] for w in d if w in self.vocab.index] for d in docs]
        doc = torch.tensor([i for i, s in enumerate(ids) for _ in s], dtype=torch.long, device=self.device)
        word = torch.tensor([w for s in ids for w in s], dtype=torch.long, device=self.device)
        cnt = torch.bincount(word.cpu(), minlength=V).double()
        self.noise = (cnt ** 0.75 / (cnt ** 0.75).sum()).float().to(self.device)
        g = torch.Generator(device=self.device).manual_seed(self.seed)
        self.D = ((torch.rand((D, self.dim), device=self.device, generator=g) - 0.5) / self.dim)
        self.C = torch.zeros((V, self.dim), device=self.device)
        if self._use_kernel():      # PV-DBOW = SGNS with the document table as the centre table
            dp = _sgns_dim(self.dim)
            Din = torch.zeros((D, dp), device=self.device)
            Din[:, : self.dim] = self.D
            Wout = torch.zeros((V, dp), device=self.device)
            self._fit_kernel(Din, Wout, doc, word, mean_in=False, decay_per_batch=False)
            self.D, self.C = Din[:, : self.dim].contiguous(), Wout[:, : self.dim].contiguous()
            self.W = self.C
            return self
        n = doc.numel()
        for ep in range(self.epochs):
            perm = torch.randperm(n, device=self.device, generator=g)
            lr = self.lr * (1 - ep / self.epochs)
            for b in range(0, n, self.batch):
                idx = perm[b:b + self.batch]
                d, o = doc[idx], word[idx]
                negs = torch.multinomial(self.noise, idx.numel() * self.negative, True, generator=g).view(-1, self.negative)
                tgt = torch.cat([o.view(-1, 1), negs], 1)
                dv, ct = self.D[d], self.C[tgt]
                lab = torch.zeros(tgt.shape, device=self.device)
                lab[:, 0] = 1
                gsc = (lab - torch.sigmoid((ct * dv.unsqueeze(1)).sum(2))) * lr
                _row_mean_add(self.D, d, (gsc.unsqueeze(2) * ct).sum(1), mean=False)   # few rows per doc
                _row_mean_add(self.C, tgt.reshape(-1), (gsc.unsqueeze(2) * dv.unsqueeze(1)).reshape(-1, self.dim))
        self.W = self.C
        return self

    def doc_vectors(self) -> torch.Tensor:
        return self.D


# ================================================================================================
# text classifier (P/text/process.py: nltk NaiveBayes over bag-of-words features)
# ================================================================================================
class TextNaiveBayes:
    """Multinomial NB over the device doc-term matrix: training = one sparse GEMM (class one-hot^T
    x counts), prediction = one GEMM with the log-probability table."""

    def __init__(self, alpha: float = 1.0, device="cpu"):
        self.alpha, self.device = alpha, device

    def fit(self, docs: Sequence[Sequence[str]], labels: Sequence) -> "TextNaiveBayes":
        self.classes = sorted(set(labels))
        self.vocab = Vocabulary(docs)
        X = doc_term_matrix(docs, self.vocab, self.device).to_dense()
        y = torch.tensor([self.classes.index(l) for l in labels], device=X.device)
        Y = torch.nn.functional.one_hot(y, len(self.classes)).float()
        cnt = Y.T @ X + self.alpha
        self.logp = torch.log(cnt / cnt.sum(1, keepdim=True))
        self.logprior = torch.log(Y.sum(0) / Y.shape[0])
        return self

    def predict_log_proba(self, docs):
        X = doc_term_matrix(docs, self.vocab, self.device).to_dense()
        s = X @ self.logp.T + self.logprior
        return s - torch.logsumexp(s, 1, keepdim=True)

    def predict(self, docs):
        return [self.classes[i] for i in self.predict_log_proba(docs).argmax(1).tolist()]

    def accuracy(self, docs, labels) -> float:
        return sum(int(p == l) for p, l in zip(self.predict(docs), labels)) / max(len(labels), 1)

    def most_informative(self, n: int = 10) -> list[tuple[str, float]]:
        if len(self.classes) != 2:
            raise ValueError("binary only")
        r = self.logp[1] - self.logp[0]
        idx = torch.argsort(r.abs(), descending=True)[:n].tolist()
        words = self.vocab.words
        return [(words[i], float(r[i])) for i in idx]
