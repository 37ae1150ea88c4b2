"""Text preprocessing and vectorisation.

Reference: ``TextPreProcessor`` (P/text/preprocess.py:45-199, nltk-based), ``NGram`` / ``BiGram`` /
``TriGram`` (:201-336, :497-524), ``TfIdf`` (:355-495), ``DocSentences`` (:526-564) and
``WordVectorContainer`` (:566-697).

nltk / contractions / inflect / BeautifulSoup are not available here, so tokenisation, stop words,
the Porter stemmer and a rule lemmatiser are implemented in this module (stemming follows the
published Porter algorithm; lemmatisation is suffix-rule based — parity with WordNet unpinned).
Vectorisation is MI355X-first: a corpus becomes ONE sparse CSR doc-term matrix on the device, and
TF-IDF weighting, normalisation and all pairwise document similarities are SpMM / GEMM.
"""
from __future__ import annotations

import html
import json
import math
import re
import warnings
from collections import Counter, defaultdict
from pathlib import Path
from typing import Iterable, Sequence

import torch

STOP_WORDS = frozenset("""a about above after again against all am an and any are aren't as at be because been before
being below between both but by can can't cannot could couldn't did didn't do does doesn't doing don't down during each
few for from further had hadn't has hasn't have haven't having he he'd he'll he's her here here's hers herself him
himself his how how's i i'd i'll i'm i've if in into is isn't it it's its itself let's me more most mustn't my myself
no nor not of off on once only or other ought our ours ourselves out over own same shan't she she'd she'll she's
should shouldn't so some such than that that's the their theirs them themselves then there there's these they they'd
they'll they're they've this those through to too under until up very was wasn't we we'd we'll we're we've were weren't
what what's when when's where where's which while who who's whom why why's with won't would wouldn't you you'd you'll
you're you've your yours yourself yourselves s t just don now will""".split())

CONTRACTIONS = {"won't": "will not", "can't": "cannot", "n't": " not", "'re": " are", "'s": " is", "'d": " would",
                "'ll": " will", "'ve": " have", "'m": " am"}

_ONES = "zero one two three four five six seven eight nine ten eleven twelve thirteen fourteen fifteen sixteen " \
        "seventeen eighteen nineteen".split()
_TENS = "_ _ twenty thirty forty fifty sixty seventy eighty ninety".split()


def number_to_words(n: int) -> str:
    if n < 20:
        return _ONES[n]
    if n < 100:
        return _TENS[n // 10] + ("" if n % 10 == 0 else "-" + _ONES[n % 10])
    if n < 1000:
        return _ONES[n // 100] + " hundred" + ("" if n % 100 == 0 else " and " + number_to_words(n % 100))
    for div, name in ((10 ** 9, "billion"), (10 ** 6, "million"), (1000, "thousand")):
        if n >= div:
            r = n % div
            return number_to_words(n // div) + " " + name + ("" if r == 0 else " " + number_to_words(r))
    return str(n)


# ------------------------------------------------------------------------------------------------
# Porter stemmer (M.F. Porter, 1980)
# ------------------------------------------------------------------------------------------------
def _cons(w, i):
    c = w[i]
    if c in "aeiou":
        return False
    if c == "y":
        return i == 0 or not _cons(w, i - 1)
    return True


def _m(stem):
    n, i, L = 0, 0, len(stem)
    while i < L and _cons(stem, i):
        i += 1
    while i < L:
        while i < L and not _cons(stem, i):
            i += 1
        if i >= L:
            break
        n += 1
        while i < L and _cons(stem, i):
            i += 1
    return n


def _has_vowel(stem):
    return any(not _cons(stem, i) for i in range(len(stem)))


def _double_c(w):
    return len(w) >= 2 and w[-1] == w[-2] and _cons(w, len(w) - 1)


def _cvc(w):
    return len(w) >= 3 and _cons(w, len(w) - 3) and not _cons(w, len(w) - 2) and _cons(w, len(w) - 1) \
        and w[-1] not in "wxy"


def porter_stem(word: str) -> str:
    w = word.lower()
    if len(w) <= 2:
        return w
    # 1a
    if w.endswith("sses"):
        w = w[:-2]
    elif w.endswith("ies"):
        w = w[:-2]
    elif w.endswith("ss"):
        pass
    elif w.endswith("s"):
        w = w[:-1]
    # 1b
    flag = False
    if w.endswith("eed"):
        if _m(w[:-3]) > 0:
            w = w[:-1]
    elif w.endswith("ed") and _has_vowel(w[:-2]):
        w, flag = w[:-2], True
    elif w.endswith("ing") and _has_vowel(w[:-3]):
        w, flag = w[:-3], True
    if flag:
        if w.endswith(("at", "bl", "iz")):
            w += "e"
        elif _double_c(w) and w[-1] not in "lsz":
            w = w[:-1]
        elif _m(w) == 1 and _cvc(w):
            w += "e"
    # 1c
    if w.endswith("y") and _has_vowel(w[:-1]):
        w = w[:-1] + "i"
    # 2
    for suf, rep in (("ational", "ate"), ("tional", "tion"), ("enci", "ence"), ("anci", "ance"), ("izer", "ize"),
                     ("abli", "able"), ("alli", "al"), ("entli", "ent"), ("eli", "e"), ("ousli", "ous"),
                     ("ization", "ize"), ("ation", "ate"), ("ator", "ate"), ("alism", "al"), ("iveness", "ive"),
                     ("fulness", "ful"), ("ousness", "ous"), ("aliti", "al"), ("iviti", "ive"), ("biliti", "ble")):
        if w.endswith(suf):
            if _m(w[:-len(suf)]) > 0:
                w = w[:-len(suf)] + rep
            break
    # 3
    for suf, rep in (("icate", "ic"), ("ative", ""), ("alize", "al"), ("iciti", "ic"), ("ical", "ic"), ("ful", ""),
                     ("ness", "")):
        if w.endswith(suf):
            if _m(w[:-len(suf)]) > 0:
                w = w[:-len(suf)] + rep
            break
    # 4
    for suf in ("al", "ance", "ence", "er", "ic", "able", "ible", "ant", "ement", "ment", "ent", "ion", "ou", "ism",
                "ate", "iti", "ous", "ive", "ize"):
        if w.endswith(suf):
            st = w[:-len(suf)]
            if _m(st) > 1 and (suf != "ion" or (st and st[-1] in "st")):
                w = st
            break
    # 5
    if w.endswith("e"):
        st = w[:-1]
        if _m(st) > 1 or (_m(st) == 1 and not _cvc(st)):
            w = st
    if _m(w) > 1 and _double_c(w) and w.endswith("l"):
        w = w[:-1]
    return w


_LEMMA_RULES = (("ies", "y"), ("ves", "f"), ("sses", "ss"), ("xes", "x"), ("ches", "ch"), ("shes", "sh"), ("s", ""))
_VERB_RULES = (("ying", "ie"), ("ing", ""), ("ied", "y"), ("ed", ""), ("es", ""), ("s", ""))


def lemmatize(word: str, pos: str = "n") -> str:
    rules = _VERB_RULES if pos == "v" else _LEMMA_RULES
    for suf, rep in rules:
        if word.endswith(suf) and len(word) - len(suf) >= 3 and not word.endswith("ss"):
            return word[: -len(suf)] + rep
    return word


class TextPreProcessor:
    def __init__(self, stemmer: str = "porter", verbose: bool = False):
        self.stemmer = stemmer
        self.verbose = verbose

    def stripHtml(self, text: str) -> str:
        return html.unescape(re.sub(r"<[^>]+>", " ", text))

    def removeBetweenSquareBrackets(self, text):
        return re.sub(r"\[[^]]*\]", "", text)

    def denoiseText(self, text):
        return self.removeBetweenSquareBrackets(self.stripHtml(text))

    def replaceContractions(self, text):
        for k, v in CONTRACTIONS.items():
            text = re.sub(re.escape(k), v, text, flags=re.IGNORECASE)
        return text

    def tokenize(self, text: str) -> list[str]:
        return re.findall(r"[A-Za-z0-9]+(?:['\-][A-Za-z0-9]+)*|[^\sA-Za-z0-9]", text)

    def removeNonAscii(self, words):
        return [w.encode("ascii", "ignore").decode() for w in words]

    def replaceNonAsciiFromText(self, text):
        return "".join(c if ord(c) < 128 else " " for c in text)

    def removeNonAsciiFromText(self, text):
        return "".join(c for c in text if ord(c) < 128)

    def allow(self, words):
        return [w for w in words if re.match(r"^[A-Za-z0-9\.\,\:\;\!\?\(\)'\-\$\@\%\"]+$", w)]

    def toLowercase(self, words):
        return [w.lower() for w in words]

    def removePunctuation(self, words):
        out = []
        for w in words:
            nw = re.sub(r"[^\w\s]", "", w)
            if nw:
                out.append(nw)
        return out

    def replaceNumbers(self, words):
        return [number_to_words(int(w)) if w.isdigit() and len(w) < 13 else w for w in words]

    def removeStopwords(self, words):
        return [w for w in words if w not in STOP_WORDS]

    def removeCustomStopwords(self, words, stop_words):
        s = set(stop_words)
        return [w for w in words if w not in s]

    def removeLowFreqWords(self, words, min_freq):
        f = Counter(words)
        return [w for w in words if f[w] > min_freq]

    def removeNumbers(self, words):
        return [w for w in words if not re.fullmatch(r"[-+]?\d*\.?\d+(e[-+]?\d+)?", w)]

    def removeShortWords(self, words, min_length):
        return [w for w in words if len(w) >= min_length]

    def keepAllowedWords(self, words, keep):
        k = set(keep)
        return [w for w in words if w in k]

    def stemWords(self, words):
        return [porter_stem(w) for w in words]

    def lemmatizeWords(self, words):
        return [lemmatize(w) for w in words]

    def lemmatizeVerbs(self, words):
        return [lemmatize(w, "v") for w in words]

    def normalize(self, words):
        words = self.removeNonAscii(words)
        words = self.toLowercase(words)
        words = self.removePunctuation(words)
        words = self.replaceNumbers(words)
        return self.removeStopwords(words)

    def documentFeatures(self, document: Iterable[str], word_features: Iterable[str]) -> dict:
        d = set(document)
        return {f"contains({w})": (w in d) for w in word_features}


def clean_tokens_reference(text: str, pp: TextPreProcessor | None = None, stem: bool = False,
                           min_len: int = 2) -> list[str]:
    """The step-by-step pipeline (contractions, tokens, lower case, punctuation, stop words, short
    words): the oracle of :func:`clean_tokens`."""
    pp = pp or TextPreProcessor()
    w = pp.removeStopwords(pp.removePunctuation(pp.toLowercase(pp.tokenize(pp.replaceContractions(text)))))
    w = pp.removeShortWords(w, min_len)
    return pp.stemWords(w) if stem else w


# clean_tokens in one pass: the contraction table as ONE alternation (its keys in table order, so
# "won't" / "can't" win over "n't" at their position, as the sequential substitutions; none of the
# replacements contains an apostrophe, so no substitution can feed a later one), one precompiled
# tokeniser, and the per-word punctuation regex replaced by deleting ' and - inside alphanumeric
# tokens (the only non-word characters the tokeniser lets into them).  The semantic-search corpus
# spent most of its host time in ~3.5 M uncached re.sub calls of the step-by-step version.
_CONTR_RE = re.compile("|".join(re.escape(k) for k in CONTRACTIONS), re.IGNORECASE)
_CONTR_LOWER = {k.lower(): v for k, v in CONTRACTIONS.items()}
_TOKEN_RE = re.compile(r"[A-Za-z0-9]+(?:['\-][A-Za-z0-9]+)*|[^\sA-Za-z0-9]")
_WORDCHAR_RE = re.compile(r"\w")
_DROP_APOS_HYPHEN = str.maketrans("", "", "'-")


_ASCII_WORD_RE = re.compile(r"[a-z0-9]+(?:['\-][a-z0-9]+)*")


def _contraction(m) -> str:
    return _CONTR_LOWER[m.group(0).lower()]


def clean_tokens(text: str, pp: TextPreProcessor | None = None, stem: bool = False, min_len: int = 2) -> list[str]:
    text = _CONTR_RE.sub(_contraction, text)
    if min_len >= 2 and text.isascii():
        # ASCII fast path: lower-casing first tokenises identically; the single-character tokens
        # are punctuation (dropped) or "_" (shorter than min_len), so only words are matched
        out = []
        for t in _ASCII_WORD_RE.findall(text.lower()):
            if "'" in t or "-" in t:
                t = t.translate(_DROP_APOS_HYPHEN)
            if len(t) >= min_len and t not in STOP_WORDS:
                out.append(t)
        return [porter_stem(w) for w in out] if stem else out
    out = []
    for t in _TOKEN_RE.findall(text):
        t = t.lower()
        c = t[0]
        if "a" <= c <= "z" or "0" <= c <= "9":
            t = t.translate(_DROP_APOS_HYPHEN)
        elif not _WORDCHAR_RE.match(t):
            continue
        if len(t) >= min_len and t not in STOP_WORDS:
            out.append(t)
    return [porter_stem(w) for w in out] if stem else out


# ------------------------------------------------------------------------------------------------
# sentence splitting
# ------------------------------------------------------------------------------------------------
def split_sentences(text: str) -> list[str]:
    parts = re.split(r"(?<=[.!?])\s+(?=[A-Z0-9\"'])", text.strip())
    return [p.strip() for p in parts if p.strip()]


class DocSentences:
    """Sentences of a document with their cleaned tokens (min sentence length in words)."""

    def __init__(self, file_path=None, min_length: int = 5, verbose: bool = False, text: str | None = None):
        text = text if text is not None else Path(file_path).read_text()
        pp = TextPreProcessor()
        self.sents, self.tokens = [], []
        for s in split_sentences(text.replace("\n", " ")):
            if len(s.split()) < min_length:
                continue
            toks = clean_tokens(s, pp)
            if toks:
                self.sents.append(s)
                self.tokens.append(toks)

    def getSentences(self):
        return list(self.sents)

    def getSentencesAsTokens(self):
        return [list(t) for t in self.tokens]

    def getTermFreqTable(self):
        t = TfIdf(None, False)
        for w in self.tokens:
            t.countDocWords(w)
        return t


# ------------------------------------------------------------------------------------------------
# n-grams and tf-idf
# ------------------------------------------------------------------------------------------------
class NGram:
    n = 1

    def __init__(self, voc_filt: Sequence[str] | None = None, verbose: bool = False):
        self.voc_filt = set(voc_filt) if voc_filt else None
        self.counts: Counter = Counter()
        self.index: dict | None = None

    def toNGram(self, words):
        return [" ".join(words[i:i + self.n]) for i in range(len(words) - self.n + 1)]

    def countDocNGrams(self, words):
        grams = self.toNGram([w for w in words if self.voc_filt is None or w in self.voc_filt])
        self.counts.update(grams)
        return grams

    def remLowCount(self, min_count):
        self.counts = Counter({k: v for k, v in self.counts.items() if v >= min_count})
        self.index = None

    def getVocabSize(self):
        return len(self.counts)

    def getNGramFreq(self):
        tot = sum(self.counts.values())
        return {k: v / tot for k, v in self.counts.items()}

    def getNGramIndex(self, show: bool = False):
        if self.index is None:
            self.index = {g: i for i, g in enumerate(sorted(self.counts))}
        return self.index

    def getVector(self, words, by_count: bool = True, normalized: bool = False) -> torch.Tensor:
        idx = self.getNGramIndex()
        v = torch.zeros(len(idx))
        hit = torch.tensor([idx[g] for g in self.toNGram(words) if g in idx], dtype=torch.long)
        if hit.numel():
            if by_count:
                v.index_add_(0, hit, torch.ones(hit.numel()))
            else:
                v[hit] = 1.0
        if normalized and v.sum() > 0:
            v /= v.sum()
        return v

    def getNonZeroCount(self):
        return sum(1 for v in self.counts.values() if v > 0)

    def save(self, path):
        Path(path).write_text(json.dumps({"n": self.n, "counts": self.counts}))

    @classmethod
    def load(cls, path):
        d = json.loads(Path(path).read_text())
        o = cls()
        o.n = d["n"]
        o.counts = Counter(d["counts"])
        return o


class BiGram(NGram):
    n = 2


class TriGram(NGram):
    n = 3


class TfIdf:
    """Word counts across documents + document frequencies; vectors by count or binary,
    optionally normalised, optionally IDF weighted (preprocess.py:355-495)."""

    def __init__(self, voc_filt: Sequence[str] | None = None, do_idf: bool = False, verbose: bool = False):
        self.voc_filt = set(voc_filt) if voc_filt else None
        self.do_idf = do_idf
        self.counts: Counter = Counter()
        self.doc_freq: Counter = Counter()
        self.n_docs = 0
        self.vocab: list[str] | None = None
        self.index: dict | None = None

    def countDocWords(self, words):
        ws = [w for w in words if self.voc_filt is None or w in self.voc_filt]
        self.counts.update(ws)
        self.doc_freq.update(set(ws))
        self.n_docs += 1

    def getWordFreq(self) -> dict:
        tot = sum(self.counts.values())
        if self.do_idf:
            return {w: c / tot * math.log(self.n_docs / self.doc_freq[w]) for w, c in self.counts.items()}
        return {w: c / tot for w, c in self.counts.items()}

    def getCount(self, word):
        return self.counts.get(word, 0)

    def getFreq(self, word):
        return self.getWordFreq().get(word, 0.0)

    def resetCounter(self):
        self.counts.clear()

    def buildVocabulary(self, words):
        self.vocab = sorted(set(words) | set(self.counts))
        self.index = None

    def getVocabulary(self):
        return self.vocab if self.vocab is not None else sorted(self.counts)

    def creatWordIndex(self):
        self.index = {w: i for i, w in enumerate(self.getVocabulary())}
        return self.index

    def getVector(self, words, by_count: bool = True, normalized: bool = False) -> torch.Tensor:
        idx = self.index or self.creatWordIndex()
        v = torch.zeros(len(idx))
        for w in words:
            if w in idx:
                if by_count:
                    v[idx[w]] += 1
                else:
                    v[idx[w]] = 1
        if normalized and v.sum() > 0:
            v /= v.sum()
        return v

    def save(self, path):
        Path(path).write_text(json.dumps({"counts": self.counts, "df": self.doc_freq, "n": self.n_docs}))

    @classmethod
    def load(cls, path):
        d = json.loads(Path(path).read_text())
        o = cls()
        o.counts, o.doc_freq, o.n_docs = Counter(d["counts"]), Counter(d["df"]), d["n"]
        return o


# ------------------------------------------------------------------------------------------------
# corpus -> device doc-term matrix
# ------------------------------------------------------------------------------------------------
class Vocabulary:
    def __init__(self, docs: Iterable[Sequence[str]] | None = None, min_count: int = 1):
        self.index: dict[str, int] = {}
        if docs is not None:
            c = Counter(w for d in docs for w in d)
            for w in sorted(k for k, v in c.items() if v >= min_count):
                self.index[w] = len(self.index)

    def __len__(self):
        return len(self.index)

    @property
    def words(self):
        return sorted(self.index, key=self.index.get)


def doc_term_matrix(docs: Sequence[Sequence[str]], vocab: Vocabulary, device="cpu", binary: bool = False) -> torch.Tensor:
    """Sparse CSR [D, V] float32 term counts (one host pass builds the CSR arrays)."""
    crow, col, val = [0], [], []
    for d in docs:
        c = Counter(vocab.index[w] for w in d if w in vocab.index)
        for k in sorted(c):
            col.append(k)
            val.append(1.0 if binary else float(c[k]))
        crow.append(len(col))
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return torch.sparse_csr_tensor(torch.tensor(crow, dtype=torch.int64), torch.tensor(col, dtype=torch.int64),
                                   torch.tensor(val, dtype=torch.float32), size=(len(docs), len(vocab))).to(device)


def tfidf_csr(counts: torch.Tensor, smooth: bool = True, sublinear: bool = False, norm: str | None = "l2"):
    """Sparse CSR TF-IDF [D, V] from a CSR count matrix on the GPU: two K28 launches (text.hip):
    document frequencies by an LDS-privatised count of the column ids, then a wavefront per row
    weights its entries (idf inline) and normalises them in place; index checks on the device."""
    from .. import _native
    D, V = counts.shape
    crow, col = counts.crow_indices().contiguous(), counts.col_indices().contiguous()
    val = counts.values().float().clone().contiguous()
    _native.C().tfidf_csr(crow, col, val, int(V), bool(smooth), bool(sublinear), {None: 0, "l1": 1, "l2": 2}[norm])
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return torch.sparse_csr_tensor(crow, col, val, size=(D, V))


def tfidf_matrix(counts: torch.Tensor, smooth: bool = True, sublinear: bool = False, norm: str | None = "l2"):
    """Dense TF-IDF [D, V] from a (sparse or dense) count matrix: idf = ln((1+D)/(1+df)) + 1.
    Sparse CSR input on the GPU goes through the K28 row kernel (``tfidf_csr``)."""
    if counts.is_sparse_csr and counts.is_cuda:
        return tfidf_csr(counts, smooth, sublinear, norm).to_dense()
    X = counts.to_dense() if counts.is_sparse_csr or counts.is_sparse else counts
    D = X.shape[0]
    df = (X > 0).sum(0).float()
    idf = torch.log((1 + D) / (1 + df)) + 1 if smooth else torch.log(D / df.clamp_min(1)) + 1
    tf = torch.where(X > 0, 1 + torch.log(X.clamp_min(1e-30)), torch.zeros_like(X)) if sublinear else X
    W = tf * idf
    if norm == "l2":
        W = W / W.norm(dim=1, keepdim=True).clamp_min(1e-12)
    elif norm == "l1":
        W = W / W.abs().sum(1, keepdim=True).clamp_min(1e-12)
    return W


def cosine_similarity_matrix(A: torch.Tensor, B: torch.Tensor | None = None) -> torch.Tensor:
    A = A / A.norm(dim=1, keepdim=True).clamp_min(1e-12)
    B = A if B is None else B / B.norm(dim=1, keepdim=True).clamp_min(1e-12)
    return A @ B.T


class WordVectorContainer:
    """Documents as bags of words; pairwise / inter-set similarity by one GEMM over the device
    doc-term matrix (preprocess.py:566-697: cosine or jaccard)."""

    def __init__(self, dir_path=None, verbose: bool = False, device="cpu"):
        self.docs: list[list[str]] = []
        self.names: list[str] = []
        self.device = device
        self.algo, self.normalizer = "cosine", None
        if dir_path:
            self.addDir(dir_path)

    def addDir(self, dir_path):
        for p in sorted(Path(dir_path).iterdir()):
            if p.is_file():
                self.addFile(p)

    def addFile(self, path):
        self.names.append(str(path))
        self.addWords(clean_tokens(Path(path).read_text()))

    def addText(self, text):
        self.names.append(f"text{len(self.docs)}")
        self.addWords(clean_tokens(text))

    def addWords(self, words):
        self.docs.append(list(words))

    def withSimilarityAlgo(self, algo: str, normalizer=None):
        self.algo, self.normalizer = algo, normalizer
        return self

    def getDocsWords(self):
        return self.docs

    def getDocs(self):
        return self.names

    def getTermFreqTable(self):
        t = TfIdf(None, False)
        for d in self.docs:
            t.countDocWords(d)
        return t

    def _matrix(self, by_count: bool, normalized: bool):
        vocab = Vocabulary(self.docs)
        X = doc_term_matrix(self.docs, vocab, self.device, binary=not by_count).to_dense()
        if normalized:
            X = X / X.sum(1, keepdim=True).clamp_min(1e-12)
        return X

    def _sim(self, A, B):
        if self.algo == "jaccard":
            a, b = (A > 0).float(), (B > 0).float()
            inter = a @ b.T
            return inter / (a.sum(1, keepdim=True) + b.sum(1).view(1, -1) - inter).clamp_min(1e-12)
        return cosine_similarity_matrix(A, B)

    def getPairWiseSimilarity(self, by_count: bool = True, normalized: bool = False) -> torch.Tensor:
        X = self._matrix(by_count, normalized)
        return self._sim(X, X)

    def getInterSetSimilarity(self, by_count: bool = True, normalized: bool = False, split: int = 0) -> torch.Tensor:
        X = self._matrix(by_count, normalized)
        return self._sim(X[:split], X[split:])

    def getNumWordVectors(self):
        return len(self.docs)
