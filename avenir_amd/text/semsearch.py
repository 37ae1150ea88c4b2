"""Semantic document search over token / sentence embeddings.

Reference: ``ssearch.py`` (P/app/ssearch.py:32-346) embeds documents with spaCy-transformers BERT
and compares a query with nine document-similarity algorithms: token max, token avg-max, token
max-avg, token avg, token median, sentence avg, sentence median, sentence max, plus whole-document
average.  spaCy / BERT are not available, so embeddings come from any encoder (our
:class:`~avenir_amd.text.models.Word2Vec`, an external model's vectors, or hashing vectors);
the similarity algorithms are implemented exactly as batched device reductions: all
query-token x document-token cosine similarities of the whole corpus are ONE GEMM, followed by
segmented max / mean / median reductions per document.
"""
from __future__ import annotations

from typing import Callable, Sequence

import torch

from .preprocess import clean_tokens, split_sentences

ALGOS = ("tokenMax", "tokenAvMax", "tokenMaxAv", "tokenAv", "tokenMed", "sentAv", "sentMed", "sentMax", "docAv")


def _norm(x):
    return x / x.norm(dim=-1, keepdim=True).clamp_min(1e-12)


class SemanticSearch:
    def __init__(self, embed_tokens: Callable[[Sequence[str]], torch.Tensor], device="cpu"):
        """``embed_tokens(list of tokens) -> [n, d]`` embedding matrix."""
        self.embed = embed_tokens
        self.device = torch.device(device)
        self.docs: list[str] = []
        self.tok_emb: list[torch.Tensor] = []
        self.sent_emb: list[torch.Tensor] = []

    def add(self, text: str):
        toks = clean_tokens(text)
        e = torch.as_tensor(self.embed(toks)).float().to(self.device) if toks else torch.zeros((0, 1))
        self.tok_emb.append(_norm(e))
        sents = [clean_tokens(s) for s in split_sentences(text)]
        se = [torch.as_tensor(self.embed(s)).float().mean(0) for s in sents if s]
        self.sent_emb.append(_norm(torch.stack(se).to(self.device)) if se else e[:0])
        self.docs.append(text)
        return self

    def add_many(self, texts: Sequence[str], sent_tokens: Sequence[Sequence[Sequence[str]]] | None = None):
        """``add`` for a whole corpus: with an embedder that has ``many`` (nn/bert.py's, the corpus
        embedder's), the tokens of every document and every sentence are embedded in one batched
        call, and the sentence means and all normalisations are batched reductions.

        A document's cleaned tokens are exactly the concatenation of its sentences' (tokens and
        contractions never span the whitespace split_sentences cuts at), so with a context-free
        embedder (``emb.context_free``, the corpus embedder) every token is looked up once and the
        document rows are the sentence rows; ``sent_tokens`` (per document, per sentence) may be
        passed in when the caller already cleaned them."""
        many = getattr(self.embed, "many", None)
        if many is None:
            for t in texts:
                self.add(t)
            return self
        if sent_tokens is None:
            sent_tokens = [[clean_tokens(x) for x in split_sentences(t)] for t in texts]
        sents = [[s for s in ss if s] for ss in sent_tokens]
        ns = [len(ss) for ss in sents]
        flat_sents = [s for ss in sents for s in ss]
        if getattr(self.embed, "context_free", False):
            toks = [[w for s in ss for w in s] for ss in sents]
            E = torch.cat([e.float() for e in many(flat_sents)], 0) if flat_sents else torch.zeros((0, 1))
            E = E.to(self.device)
            doc_rows = E                                         # sentence rows in document order
        else:
            toks = [clean_tokens(t) for t in texts]
            embs = many(toks + flat_sents)
            doc_rows = torch.cat([e.float() for e, t in zip(embs[:len(texts)], toks) if t], 0).to(self.device) \
                if any(toks) else torch.zeros((0, 1), device=self.device)
            E = torch.cat([e.float() for e in embs[len(texts):]], 0).to(self.device) if flat_sents else \
                torch.zeros((0, doc_rows.shape[1]), device=self.device)
        # sentence means: one segmented sum over the sentence rows
        lens = torch.tensor([len(s) for s in flat_sents], dtype=torch.long, device=self.device)
        if flat_sents:
            seg = torch.repeat_interleave(torch.arange(len(flat_sents), device=self.device), lens)
            S = torch.zeros((len(flat_sents), E.shape[1]), device=self.device).index_add_(0, seg, E)
            S = _norm(S / lens.view(-1, 1).float())
        else:
            S = torch.zeros((0, max(1, E.shape[1])), device=self.device)
        Tn = _norm(doc_rows)
        tl = [len(t) for t in toks]
        tok_parts = list(torch.split(Tn, tl)) if Tn.shape[0] else [Tn[:0]] * len(texts)
        sent_parts = list(torch.split(S, ns)) if S.shape[0] else [S[:0]] * len(texts)
        for i, t in enumerate(texts):
            self.tok_emb.append(tok_parts[i] if tl[i] else torch.zeros((0, 1), device=self.device))
            self.sent_emb.append(sent_parts[i] if ns[i] else torch.zeros((0, 1), device=self.device))
            self.docs.append(t)
        return self

    def _flat(self, embs):
        lens = torch.tensor([e.shape[0] for e in embs], device=self.device)
        cat = torch.cat([e for e in embs if e.shape[0]], 0)
        seg = torch.repeat_interleave(torch.arange(len(embs), device=self.device), lens)
        return cat, seg, lens

    def scores(self, query: str, algo: str = "tokenAvMax") -> torch.Tensor:
        """Similarity of the query to every document: [n_docs]."""
        qt = clean_tokens(query)
        q = _norm(torch.as_tensor(self.embed(qt)).float().to(self.device))          # [m, d]
        if algo.startswith("sent"):
            cat, seg, lens = self._flat(self.sent_emb)
            qv = _norm(q.mean(0, keepdim=True))
            s = (cat @ qv.T).view(-1)                                               # [S]
            return self._segment(s, seg, lens, {"sentAv": "mean", "sentMed": "median", "sentMax": "max"}[algo])
        if algo == "docAv":
            cat, seg, lens = self._flat(self.tok_emb)
            D = torch.zeros((len(self.docs), cat.shape[1]), device=self.device).index_add_(0, seg, cat)
            return (_norm(D) @ _norm(q.mean(0, keepdim=True)).T).view(-1)
        cat, seg, lens = self._flat(self.tok_emb)
        S = q @ cat.T                                                               # [m, T] one GEMM
        nd = len(self.docs)
        if algo == "tokenMax":
            return self._segment(S.max(0).values, seg, lens, "max")
        if algo == "tokenAvMax":     # per query token: max over doc tokens; then average
            mx = torch.full((S.shape[0], nd), -2.0, device=self.device).scatter_reduce(
                1, seg.view(1, -1).expand_as(S), S, "amax", include_self=True)
            return mx.mean(0)
        if algo == "tokenMaxAv":     # per query token: mean over doc tokens; then max
            sm = torch.zeros((S.shape[0], nd), device=self.device).index_add_(1, seg, S)
            return (sm / lens.clamp_min(1).view(1, -1)).max(0).values
        if algo == "tokenAv":
            return self._segment(S.mean(0), seg, lens, "mean")
        if algo == "tokenMed":
            return self._segment(S.median(0).values, seg, lens, "median")
        raise ValueError(f"unknown algorithm {algo}")

    def _segment(self, v, seg, lens, how):
        nd = len(self.docs)
        if how == "max":
            return torch.full((nd,), -2.0, device=self.device).scatter_reduce(0, seg, v, "amax", include_self=True)
        if how == "mean":
            return torch.zeros(nd, device=self.device).index_add_(0, seg, v) / lens.clamp_min(1)
        out = torch.empty(nd, device=self.device)
        o = 0
        for i, L in enumerate(lens.tolist()):
            out[i] = v[o:o + L].median() if L else -2.0
            o += L
        return out

    def search(self, query: str, algo: str = "tokenAvMax", top: int = 5) -> list[tuple[int, float]]:
        s = self.scores(query, algo)
        idx = torch.argsort(s, descending=True)[:top].tolist()
        return [(i, float(s[i])) for i in idx]


def hashing_embedder(dim: int = 256, seed: int = 0):
    """Deterministic random-projection token vectors (a stand-in encoder when no trained model is
    available): each token hashes to a fixed gaussian vector."""
    import hashlib

    def emb(tokens):
        out = []
        for t in tokens:
            h = int(hashlib.md5(f"{seed}:{t}".encode()).hexdigest()[:8], 16)
            g = torch.Generator().manual_seed(h)
            out.append(torch.randn(dim, generator=g))
        return torch.stack(out) if out else torch.zeros((0, dim))
    return emb


def corpus_embedder(docs: Sequence[str], dim: int = 100, epochs: int = 10, window: int = 5, device="cpu",
                    seed: int = 0, sentences: Sequence[Sequence[str]] | None = None):
    """Document embedder trained on the corpus itself: skip-gram Word2Vec (negative sampling, on
    ``device``) over the cleaned sentences of ``docs``; tokens outside its vocabulary fall back to
    scaled hashing vectors.  Stands in for ssearch.py's spaCy-transformers BERT encoder
    (P/app/ssearch.py:184-186), which needs pretrained weights this environment cannot fetch —
    parity unpinned; the tests check retrieval quality on a seeded topical corpus instead."""
    from .models import Word2Vec
    if sentences is None:
        sentences = [clean_tokens(s) for d in docs for s in split_sentences(d)]
    sents = [s for s in sentences if s]
    w2v = Word2Vec(dim=dim, window=window, epochs=epochs, seed=seed, device=device).fit(sents)
    fallback = hashing_embedder(dim, seed)
    W = w2v.W
    scale = float(W.norm(dim=1).mean()) if W.numel() else 1.0

    def emb(tokens):
        if not tokens:
            return torch.zeros((0, dim), device=W.device)
        idx = [w2v.vocab.index.get(t, -1) for t in tokens]
        out = torch.empty((len(tokens), dim), device=W.device)
        known = [k for k, i in enumerate(idx) if i >= 0]
        if known:
            out[known] = W[torch.tensor([idx[k] for k in known], device=W.device)]
        unk = [k for k, i in enumerate(idx) if i < 0]
        if unk:
            v = fallback([tokens[k] for k in unk]).to(W.device)
            out[unk] = v / v.norm(dim=1, keepdim=True).clamp_min(1e-12) * scale
        return out

    def many(token_lists):
        """``emb`` of many token lists with one vocabulary lookup and one gather."""
        lens = [len(t) for t in token_lists]
        flat = [t for ts in token_lists for t in ts]
        if not flat:
            return [torch.zeros((0, dim), device=W.device) for _ in token_lists]
        return list(torch.split(emb(flat), lens))
    emb.model = w2v
    emb.many = many
    emb.context_free = True           # a token's vector does not depend on its neighbours
    return emb


def search_corpus(docs: Sequence[str], dim: int = 100, epochs: int = 10, device="cpu", seed: int = 0) -> SemanticSearch:
    """A :class:`SemanticSearch` over ``docs`` with the corpus-trained embedder."""
    sent_tokens = [[clean_tokens(x) for x in split_sentences(d)] for d in docs]     # cleaned once
    emb = corpus_embedder(docs, dim, epochs, device=device, seed=seed,
                          sentences=[s for ss in sent_tokens for s in ss])
    ss = SemanticSearch(emb, device=device)
    return ss.add_many(docs, sent_tokens=sent_tokens)
