"""Text: preprocessing, n-grams, tf-idf (vs sklearn oracle), summarisers, LDA, word2vec, text NB."""
import random

import numpy as np
import pytest
import torch

from avenir_amd.text import (BiGram, DocSentences, Doc2Vec, LatentDirichletAllocation, LatentSemSumm,
                             NonNegMatFactSumm, SumBasicSumm, TermFreqSumm, TextNaiveBayes, TextPreProcessor,
                             TextRankSumm, TfIdf, Vocabulary, Word2Vec, WordVectorContainer, doc_term_matrix, nmf,
                             pagerank, porter_stem, split_sentences, tfidf_matrix)

DOC = ("The GPU accelerates matrix multiplication for deep learning workloads. "
       "Matrix cores on the accelerator perform fused multiply add operations at high throughput. "
       "Bananas are a popular fruit rich in potassium and eaten around the world. "
       "Memory bandwidth limits many deep learning kernels that are not compute bound. "
       "Fruit markets sell bananas, apples and oranges every single morning. "
       "Kernel fusion reduces memory traffic by keeping intermediate tiles in local memory. "
       "The weather today is sunny with a light breeze from the west.")


def test_porter_stemmer_known_words():
    cases = {"caresses": "caress", "ponies": "poni", "running": "run", "relational": "relat", "happiness": "happi",
             "generalization": "gener", "hopping": "hop", "filing": "file", "agreed": "agre", "sky": "sky"}
    for w, s in cases.items():
        assert porter_stem(w) == s, w


def test_preprocessor_pipeline():
    pp = TextPreProcessor()
    t = pp.denoiseText("<p>Hello [note] world &amp; friends</p>")
    assert "note" not in t and "&" in t
    toks = pp.tokenize(pp.replaceContractions("I can't run 3 miles, it's 100 degrees!"))
    n = pp.normalize(toks)
    assert "cannot" not in n and "three" in n and "one hundred" in n and "miles" in n
    assert pp.removeShortWords(["a", "abc"], 2) == ["abc"]
    assert pp.removeLowFreqWords(["a", "a", "b"], 1) == ["a", "a"]
    assert pp.lemmatizeWords(["cats", "ponies"]) == ["cat", "pony"]


def test_ngrams_and_tfidf_vs_sklearn():
    from sklearn.feature_extraction.text import TfidfVectorizer
    docs = [["gpu", "matrix", "gpu"], ["matrix", "memory"], ["banana", "fruit", "fruit", "gpu"]]
    bg = BiGram()
    for d in docs:
        bg.countDocNGrams(d)
    assert bg.counts["gpu matrix"] == 1 and bg.getVocabSize() == 6
    vocab = Vocabulary(docs)
    X = doc_term_matrix(docs, vocab)
    W = tfidf_matrix(X).numpy()
    sk = TfidfVectorizer(analyzer=lambda d: d, vocabulary=vocab.words).fit_transform(docs).toarray()
    assert np.allclose(W, sk, atol=1e-6)
    tf = TfIdf(None, True)
    for d in docs:
        tf.countDocWords(d)
    assert tf.getCount("gpu") == 3
    v = tf.getVector(["gpu", "memory"], True, True)
    assert float(v.sum()) == pytest.approx(1.0)


def test_sentences_and_summarizers():
    assert len(split_sentences(DOC)) == 7
    ds = DocSentences(text=DOC, min_length=5)
    assert len(ds.getSentences()) == 7
    for S in (TermFreqSumm(size=3), SumBasicSumm(size=3), LatentSemSumm(num_topics=2, size=3),
              NonNegMatFactSumm(num_topics=2, size=3), TextRankSumm(size=3), TextRankSumm(size=3, diversify=True)):
        out = S.summarize(text=DOC)
        assert len(out) == 3
        sents = split_sentences(DOC)
        pos = [sents.index(s) for s, _ in out]
        assert pos == sorted(pos)           # document order
    assert len(TermFreqSumm(size=50, by_count=False).summarize(text=DOC)) == 3


def test_nmf_and_pagerank():
    g = torch.Generator().manual_seed(0)
    W0, H0 = torch.rand((30, 3), generator=g), torch.rand((3, 20), generator=g)
    W, H = nmf(W0 @ H0, 3, iters=500)
    assert float(((W @ H) - W0 @ H0).norm() / (W0 @ H0).norm()) < 0.05
    S = torch.tensor([[0, 1, 1], [1, 0, 0], [1, 0, 0]], dtype=torch.float64)
    r = pagerank(S)
    assert float(r.sum()) == pytest.approx(1.0) and int(r.argmax()) == 0


def _topic_corpus(n=300, seed=0):
    rnd = random.Random(seed)
    topics = [["gpu", "kernel", "memory", "matrix", "cache", "tile"],
              ["banana", "apple", "fruit", "orange", "market", "juice"],
              ["rain", "sunny", "weather", "wind", "cloud", "storm"]]
    docs, labels = [], []
    for i in range(n):
        t = rnd.randrange(3)
        docs.append([rnd.choice(topics[t]) for _ in range(20)])
        labels.append(t)
    return docs, labels, topics


def test_lda_recovers_topics():
    docs, labels, topics = _topic_corpus()
    lda = LatentDirichletAllocation(3, iters=30, seed=1).fit(docs)
    found = [set(w for w, _ in lda.top_terms(k, 6)) for k in range(3)]
    for t in topics:
        assert max(len(set(t) & f) for f in found) >= 5
    th = lda.doc_topic()
    assert torch.allclose(th.sum(1), torch.ones(len(docs), dtype=th.dtype))
    assert lda.transform(docs[:5]).shape == (5, 3)


def test_word2vec_and_doc2vec(tmp_path):
    docs, labels, topics = _topic_corpus(400)
    w2v = Word2Vec(dim=16, window=3, epochs=5, batch=2048, seed=0).fit(docs)
    sim = dict(w2v.most_similar("gpu", 5))
    assert len(set(sim) & set(topics[0])) >= 4
    p = tmp_path / "w2v.safetensors"
    w2v.save(p)
    w2 = Word2Vec.load(p)
    assert torch.allclose(w2.vector("gpu"), w2v.vector("gpu"))
    d2v = Doc2Vec(dim=16, epochs=10, seed=0).fit(docs)
    D = d2v.doc_vectors()
    D = D - D.mean(0)                       # remove the corpus-frequency direction
    D = D / D.norm(dim=1, keepdim=True)
    same = [(D[i] @ D[j]).item() for i in range(20) for j in range(20) if i != j and labels[i] == labels[j]]
    diff = [(D[i] @ D[j]).item() for i in range(20) for j in range(20) if labels[i] != labels[j]]
    assert np.mean(same) > np.mean(diff) + 0.2


def test_text_nb_and_similarity():
    docs, labels, _ = _topic_corpus(300, seed=3)
    nb = TextNaiveBayes().fit(docs[:200], labels[:200])
    assert nb.accuracy(docs[200:], labels[200:]) > 0.97
    wc = WordVectorContainer()
    for d in docs[:6]:
        wc.addWords(d)
    S = wc.getPairWiseSimilarity()
    assert S.shape == (6, 6) and torch.allclose(S.diagonal(), torch.ones(6))
    J = wc.withSimilarityAlgo("jaccard").getInterSetSimilarity(True, False, 3)
    assert J.shape == (3, 3)


# ------------------------------------------------------------------------------------------------
# K28 kernels (text.hip): TF-IDF rows, persistent pagerank, SGNS word2vec / doc2vec
# ------------------------------------------------------------------------------------------------
@pytest.mark.gpu
def test_tfidf_kernel_matches_sklearn(cuda):
    from sklearn.feature_extraction.text import TfidfVectorizer
    docs, _, _ = _topic_corpus(200, seed=5)
    docs[3] = []                                            # an empty document row
    vocab = Vocabulary(docs)
    X = doc_term_matrix(docs, vocab, device=cuda)
    for norm in ("l2", "l1", None):
        for sub in (False, True):
            W = tfidf_matrix(X, sublinear=sub, norm=norm).cpu().numpy()
            sk = TfidfVectorizer(analyzer=lambda d: d, vocabulary=vocab.words, norm=norm,
                                 sublinear_tf=sub).fit_transform(docs).toarray()
            assert np.allclose(W, sk, atol=1e-6), (norm, sub)


@pytest.mark.gpu
def test_tfidf_csr_large_vocab_and_range_checks(cuda):
    """Zipf columns over V > 32768 (LDS-counted hot ids + global-atomic tail) against sklearn's
    TfidfTransformer, smooth and unsmoothed idf; out-of-range ids fail loudly."""
    import scipy.sparse as sp
    from sklearn.feature_extraction.text import TfidfTransformer

    from avenir_amd.text.preprocess import tfidf_csr
    rng = np.random.default_rng(3)
    D, V, per = 3000, 40000, 50
    cols = np.minimum(rng.zipf(1.3, size=D * per) - 1, V - 1)
    M = sp.csr_matrix((np.ones(D * per, dtype=np.float32), (np.repeat(np.arange(D), per), cols)), shape=(D, V))
    M.sum_duplicates()
    G = torch.sparse_csr_tensor(torch.tensor(M.indptr, dtype=torch.long), torch.tensor(M.indices, dtype=torch.long),
                                torch.tensor(M.data), size=(D, V)).to(cuda)
    for smooth in (True, False):
        for sub in (False, True):
            W = tfidf_csr(G, smooth=smooth, sublinear=sub).to_dense().cpu().numpy()
            sk = TfidfTransformer(smooth_idf=smooth, sublinear_tf=sub).fit_transform(M).toarray()
            assert np.allclose(W, sk, atol=1e-6), (smooth, sub)
    from avenir_amd import _native
    col = G.col_indices().clone()
    col[7] = V + 5
    with pytest.raises(RuntimeError, match="column id out of range"):
        _native.C().tfidf_csr(G.crow_indices(), col, G.values().clone(), V, True, False, 2)
    crow = G.crow_indices().clone()
    crow[5] = crow[6] + 1                                   # a row pointer past its successor
    with pytest.raises(RuntimeError, match="row pointers"):
        _native.C().tfidf_csr(crow, G.col_indices(), G.values().clone(), V, True, False, 2)


@pytest.mark.gpu
def test_pagerank_kernel_matches_tensor_path(cuda):
    g = torch.Generator().manual_seed(2)
    for n in (3, 130, 1500):
        S = torch.rand((n, n), generator=g, dtype=torch.float64)
        S[:, 1] = 0
        S[1, :] = 0                                         # a dangling node
        S.fill_diagonal_(0)
        ref = pagerank(S)
        got = pagerank(S.to(cuda)).cpu()
        assert torch.allclose(got, ref, rtol=1e-10, atol=1e-13), n


@pytest.mark.gpu
def test_pagerank_multi_workgroup(cuda):
    """Graphs above the one-workgroup size (and the multi-workgroup kernels at small n, incl. an
    iteration cap hit before convergence) against the tensor path, iteration counts included."""
    from avenir_amd import _native
    g = torch.Generator().manual_seed(3)
    for n, iters, tol in ((3, 100, 1e-10), (300, 100, 1e-10), (700, 4, 1e-10), (3000, 100, 1e-10)):
        S = torch.rand((n, n), generator=g, dtype=torch.float64)
        S[:, 1] = 0
        S[1, :] = 0
        S.fill_diagonal_(0)
        ref = pagerank(S, iters=iters, tol=tol)
        out = S.sum(1, keepdim=True)
        P = torch.where(out > 0, S / out.clamp_min(1e-300), torch.full_like(S, 1.0 / n))
        r, it = _native.C().pagerank_multi(P.to(cuda).contiguous(), 0.85, iters, tol)
        r1, it1 = _native.C().pagerank(P.to(cuda).contiguous(), 0.85, iters, tol) if n <= 8192 else (r, it)
        assert torch.allclose(r.cpu(), ref, rtol=1e-10, atol=1e-13), n
        assert int(it) == int(it1), (n, int(it), int(it1))
        if n > 2048:
            assert torch.allclose(pagerank(S.to(cuda), iters=iters, tol=tol).cpu(), ref, rtol=1e-10, atol=1e-13)


@pytest.mark.gpu
def test_word2vec_and_doc2vec_kernel(cuda):
    docs, labels, topics = _topic_corpus(400)
    w2v = Word2Vec(dim=16, window=3, epochs=5, seed=0, device=cuda).fit(docs)
    assert w2v.W.shape[1] == 16
    sim = dict(w2v.most_similar("gpu", 5))
    assert len(set(sim) & set(topics[0])) >= 4
    d2v = Doc2Vec(dim=16, epochs=10, seed=0, device=cuda).fit(docs)
    D = d2v.doc_vectors().cpu()
    D = D - D.mean(0)
    D = D / D.norm(dim=1, keepdim=True)
    same = [(D[i] @ D[j]).item() for i in range(20) for j in range(20) if i != j and labels[i] == labels[j]]
    diff = [(D[i] @ D[j]).item() for i in range(20) for j in range(20) if labels[i] != labels[j]]
    assert np.mean(same) > np.mean(diff) + 0.2


def test_clean_tokens_one_pass_equals_stepwise_pipeline():
    """The one-pass clean_tokens (one contraction alternation, one tokeniser, ASCII fast path)
    equals the step-by-step pipeline on fuzzed text: contractions in any case, apostrophes and
    hyphens inside and around words, unicode letters, underscores, numbers, punctuation."""
    import random
    from avenir_amd.text.preprocess import clean_tokens, clean_tokens_reference
    rng = random.Random(0)
    frags = ["won't", "Won't", "CAN'T", "can't", "don't", "isn't", "they're", "it's", "I'd", "we'll", "you've", "I'm",
             "o'brien", "well-known", "rock'n'roll", "-", "'", "--", "a-", "students'", "naïve", "café", "É", "_",
             "__init__", "x_y", "3.14", "1,000", "42", "e-mail", "Hello", "WORLD", "the", "and", "a", "!", "?", "(",
             "\"", "$5", "@home", "#tag", "Zürich", "n't", "'s", "can'tn't", "a'", "'a", "K", "ﬁne", "a-'b"]
    for _ in range(5000):
        text = " ".join(rng.choice(frags) + rng.choice([".", ",", "", ""]) for _ in range(rng.randint(1, 12)))
        for stem in (False, True):
            for ml in (1, 2, 3):
                assert clean_tokens(text, stem=stem, min_len=ml) == clean_tokens_reference(text, stem=stem, min_len=ml)
