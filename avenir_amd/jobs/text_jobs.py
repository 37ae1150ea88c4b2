"""Text application drivers (P/app/summd.py, topic.py, tf.py, tfe.py, dvd.py, wvd.py, classify.py,
ssearch.py) as CLI jobs over the ``avenir_amd.text`` library.

Each keeps the reference's operation names (``--mode``) and ``.properties`` keys
(``common.*``, ``train.*``, ``generate.*``, ``analyze.*``).  The differences are these:

* The corpora the reference downloads (20 newsgroups for the base term distribution, nltk's
  movie reviews for ``classify``) are not reachable here.  They come from ``--input`` instead:
  a directory of documents, or a file with one document per line.
* Models are saved as safetensors / JSON, not gensim pickles.
* Results go to ``--output`` (or stdout) as text lines, not Python ``print`` dumps.

The numeric work runs on the job's device (``--device``): the doc-term matrices, SVD / NMF / LDA
updates, PageRank, skip-gram / PV-DBOW SGD and the similarity GEMMs.
"""
from __future__ import annotations

import json
import math
from pathlib import Path

import torch

from .common import JobContext, job


def _docs(path: str) -> tuple[list[str], list[str]]:
    """(texts, names): every visible file of a directory (sorted), or one document per line."""
    p = Path(path)
    if p.is_dir():
        files = sorted(f for f in p.iterdir() if f.is_file() and not f.name.startswith((".", "_")))
        return [f.read_text(errors="ignore") for f in files], [str(f) for f in files]
    lines = [l for l in p.read_text(errors="ignore").splitlines() if l.strip()]
    return lines, [f"{p.name}:{i}" for i in range(len(lines))]


def _clean(texts):
    from ..text.preprocess import TextPreProcessor, clean_tokens
    pp = TextPreProcessor()
    return [clean_tokens(t, pp) for t in texts]


def _out(ctx: JobContext, lines: list[str]) -> None:
    if getattr(ctx.args, "output", None):
        ctx.emit_root(lines)
    elif ctx.is_root:
        print("\n".join(lines), flush=True)


def _input(ctx: JobContext, *keys: str) -> str:
    for k in keys:
        v = ctx.get_str(k, None)
        if v:
            return ctx.path(k)
    if getattr(ctx.args, "input", None):
        return ctx.args.input
    raise SystemExit(f"missing input: --input or {' / '.join(keys)}")


# ------------------------------------------------------------------------------------------------
@job("textSummarizer", "extractive summaries (P/app/summd.py): --mode tfSumm|sbSumm|lsSumm|nmfSumm|trSumm|etrSumm",
     aliases=("summd",))
def summarize(args):
    """Keys: ``common.data.file``, ``common.size``, ``common.byCount``, ``common.min.sentence.length``,
    ``common.show.score``, ``tf.length.normalizer``, ``tf.diversify[.regularizer|.aggr]``,
    ``tr.diversify*``, ``lsi.num.topics``, ``nmf.num.topics``, ``nmf.max.iter``, ``etr.model.path``
    (a word2vec model saved by ``wordToVec``)."""
    from ..text import models as TM
    ctx = JobContext(args)
    op = args.mode or "tfSumm"
    common = dict(size=ctx.get_int("common.size", 5), by_count=ctx.get_bool("common.byCount", True),
                  min_sentence_length=ctx.get_int("common.min.sentence.length", 5), device=ctx.device)

    def div(prefix):
        return dict(diversify=ctx.get_bool(f"{prefix}.diversify", False),
                    reg=ctx.get_float(f"{prefix}.diversify.regularizer", 0.7),
                    aggr=ctx.get_str(f"{prefix}.diversify.aggr", "average"))
    if op == "tfSumm":
        s = TM.TermFreqSumm(normalizer=ctx.get_str("tf.length.normalizer", "linear"), **common, **div("tf"))
    elif op == "sbSumm":
        s = TM.SumBasicSumm(**common)
    elif op == "lsSumm":
        s = TM.LatentSemSumm(num_topics=ctx.get_int("lsi.num.topics", 5), **common)
    elif op == "nmfSumm":
        s = TM.NonNegMatFactSumm(num_topics=ctx.get_int("nmf.num.topics", 5),
                                 iters=ctx.get_int("nmf.max.iter", 200), **common)
    elif op == "trSumm":
        s = TM.TextRankSumm(**common, **div("tr"))
    elif op == "etrSumm":
        emb = TM.Word2Vec.load(ctx.path("etr.model.path"), device=ctx.device)
        s = TM.EmbeddingTextRankSumm(emb, **common)
    else:
        raise SystemExit(f"invalid summarizer {op}")
    show = ctx.get_bool("common.show.score", False)
    res = s.summarize(_input(ctx, "common.data.file"))
    _out(ctx, [f"{t}  ({sc})" if show else t for t, sc in res])


# ------------------------------------------------------------------------------------------------
def _top_by_odds(distr, odds, min_count=None):
    """Leading entries until their cumulative probability's odds pass ``odds`` (topic.py:34-47)."""
    s, sel = 0.0, []
    for d in distr:
        s += d[1]
        sel.append(d)
        if s >= 1.0 or s / (1.0 - s) > odds:
            break
    if min_count and len(sel) < min_count:
        sel = list(distr[:min_count])
    return sel


@job("topicModel", "LDA topics (P/app/topic.py): --mode train|analyze; per-doc topics by odds ratio, topic words",
     aliases=("topic",))
def topic(args):
    """``train``: fit on ``train.data.dir`` (``train.num.topics``, ``train.num.iter``) and save
    the model to ``common.model.directory/common.model.file``; ``analyze``: load it, infer topic
    mixtures for ``analyze.data.dir`` and report each document's leading topics
    (``analyze.doc.topic.odds.ratio``, ``.min.count``) with their leading words
    (``analyze.topic.word.top.max``, ``analyze.topic.word.odds.ratio``, ``.min.count``)."""
    from ..text.models import LatentDirichletAllocation
    from ..text.preprocess import Vocabulary
    ctx = JobContext(args)
    mode = args.mode or ctx.get_str("common.mode", "train")
    mdir = ctx.get_str("common.model.directory", None)
    mfile = ctx.get_str("common.model.file", "lda")
    mpath = Path(args.model) if args.model else (Path(mdir) / f"{mfile}.safetensors" if mdir else None)
    if mode == "train":
        texts, names = _docs(_input(ctx, "train.data.dir"))
        docs = _clean(texts)
        lda = LatentDirichletAllocation(num_topics=ctx.get_int("train.num.topics", 10),
                                        iters=ctx.get_int("train.num.iter", 50), seed=args.seed, device=ctx.device)
        lda.fit(docs, min_count=ctx.get_int("train.min.word.count", 1))
        if mpath is not None and ctx.is_root:
            from safetensors.torch import save_file
            mpath.parent.mkdir(parents=True, exist_ok=True)
            save_file({"lam": lda.lam.cpu().contiguous()}, str(mpath),
                      metadata={"words": "\n".join(lda.vocab.words), "alpha": str(lda.alpha), "K": str(lda.K)})
        theta = lda.doc_topic()
    elif mode == "analyze":
        from safetensors import safe_open
        if mpath is None:
            raise SystemExit("analyze needs --model or common.model.directory")
        with safe_open(str(mpath), "pt") as f:
            lam, meta = f.get_tensor("lam"), f.metadata()
        lda = LatentDirichletAllocation(num_topics=int(meta["K"]), alpha=float(meta["alpha"]), device=ctx.device)
        lda.lam = lam.to(ctx.device)
        lda.vocab = Vocabulary()
        lda.vocab.index = {w: i for i, w in enumerate(meta["words"].split("\n"))}
        texts, names = _docs(_input(ctx, "analyze.data.dir"))
        theta = lda.transform(_clean(texts))
    else:
        raise SystemExit(f"invalid mode {mode}")
    dt_odds = ctx.get_float("analyze.doc.topic.odds.ratio", 3.0)
    tw_odds = ctx.get_float("analyze.topic.word.odds.ratio", 3.0)
    tw_max = ctx.get_int("analyze.topic.word.top.max", 20)
    dt_min = ctx.get_int("analyze.doc.topic.min.count", 1)
    tw_min = ctx.get_int("analyze.topic.word.min.count", 5)
    lines = []
    words_cache: dict[int, list] = {}
    for d, name in enumerate(names):
        dist = sorted(((k, float(p)) for k, p in enumerate(theta[d].tolist())), key=lambda t: -t[1])
        top = _top_by_odds(dist, dt_odds, dt_min)
        net: dict[str, float] = {}
        for k, p in top:
            if k not in words_cache:
                words_cache[k] = _top_by_odds(lda.top_terms(k, tw_max), tw_odds, tw_min)
            for w, wp in words_cache[k]:
                net[w] = net.get(w, 0.0) + wp * p
        words = sorted(net.items(), key=lambda t: -t[1])
        lines.append(json.dumps({"doc": name, "topics": [[k, round(p, 6)] for k, p in top],
                                 "words": [[w, round(v, 6)] for w, v in words]}))
    for k in sorted(words_cache):
        lines.append(json.dumps({"topic": k, "words": [[w, round(v, 6)] for w, v in words_cache[k]]}))
    _out(ctx, lines)


# ------------------------------------------------------------------------------------------------
@job("termDistribution", "term distributions (P/app/tf.py): --mode buildBaseTf|tfDiff; relative-entropy "
     "ranking of a corpus' words against a base distribution", aliases=("tf",))
def term_distr(args):
    """``buildBaseTf``: term frequencies of the ``--input`` corpus saved to ``--model`` (JSON).
    ``tfDiff``: words of ``--input`` ranked by their frequency among those with positive
    p log(p/q) against the base file (unseen base words count as 1000, tf.py:59-78), top 100."""
    from ..text.preprocess import TfIdf
    ctx = JobContext(args)
    mode = args.mode or "tfDiff"
    texts, _ = _docs(_input(ctx))
    tf = TfIdf(None, False)
    for d in _clean(texts):
        tf.countDocWords(d)
    if mode == "buildBaseTf":
        if not args.model:
            raise SystemExit("buildBaseTf needs --model <file>")
        ctx.check()
        if ctx.is_root:
            tf.save(args.model)
        ctx.report({"terms": len(tf.counts), "docs": tf.n_docs})
        return
    if mode != "tfDiff":
        raise SystemExit(f"invalid mode {mode}")
    base = TfIdf.load(args.model).getWordFreq()
    this = tf.getWordFreq()
    out = []
    for w in sorted(set(base) | set(this)):
        p, q = this.get(w, 0.0), base.get(w, 0.0)
        if p > 0:
            rent = p * math.log(p / q) if q > 0 else 1000.0
        else:
            rent = -1000.0 if q > 1e-7 else 0.0
        if rent > 0:
            out.append((w, rent, p))
    out.sort(key=lambda t: -t[2])
    _out(ctx, [f"{w},{r:.6f},{p:.6f}" for w, r, p in out[:100]])


# ------------------------------------------------------------------------------------------------
@job("textEncoder", "n-gram vectors and an auto-encoder over them (P/app/tfe.py): --mode distr|vectorise|train|encode",
     aliases=("tfe",))
def text_encoder(args):
    """``distr`` / ``vectorise``: bigram (``--kind bi``) or trigram (``tri``) counts over the
    ``--input`` corpus, low counts (< 3) removed; ``vectorise`` writes each document's normalised
    n-gram vector.  ``train`` / ``encode``: the config's AutoEncoder (``train.*`` keys of
    nn/unsupervised.py) over ``train.data.file`` vectors, saved to / loaded from
    ``common.model.directory/common.model.file``; ``encode`` writes the codes."""
    import numpy as np
    from ..text.preprocess import BiGram, TriGram
    ctx = JobContext(args)
    mode = args.mode or "vectorise"
    if mode in ("distr", "vectorise"):
        texts, _ = _docs(_input(ctx))
        docs = _clean(texts)
        kind = args.kind or "bi"
        if kind not in ("bi", "tri"):
            raise SystemExit("invalid ngram type")
        ng = BiGram() if kind == "bi" else TriGram()
        for d in docs:
            ng.countDocNGrams(d)
        ng.remLowCount(3)
        if mode == "distr":
            fr = ng.getNGramFreq()
            items = sorted(fr.items(), key=lambda t: -t[1]) if isinstance(fr, dict) else fr
            _out(ctx, [f"{' '.join(k) if isinstance(k, tuple) else k},{v:.6f}" for k, v in items])
            return
        # the [docs, n-grams] count matrix from one scatter-add, rows normalised, and the text from
        # the native formatter (a per-document Python vector build and per-value f-string took
        # 1.5 s for 6,000 documents)
        idx = ng.getNGramIndex()
        V = len(idx)
        ids = [[idx[g] for g in ng.toNGram(d) if g in idx] for d in docs]
        flat = torch.tensor([r * V + j for r, row in enumerate(ids) for j in row], dtype=torch.long)
        M = torch.zeros(len(docs) * max(V, 1))
        if flat.numel():
            M.index_add_(0, flat, torch.ones(flat.numel()))
        M = M.view(len(docs), max(V, 1))[:, :V]
        keep = (M != 0).any(1)
        M = M[keep]
        M = M / M.sum(1, keepdim=True)
        if getattr(ctx.args, "output", None) and V:
            ctx.emit_columns([("f", M[:, j].double().contiguous(), 6) for j in range(V)], int(M.shape[0]))
        else:
            _out(ctx, [",".join(f"{x:.6f}" for x in row) for row in M.tolist()])
        return
    from ..nn.unsupervised import AutoEncoder
    ae = AutoEncoder.from_config(ctx.cfg, device=ctx.device)
    mdir = ctx.get_str("common.model.directory", None)
    mpath = Path(args.model) if args.model else (
        Path(mdir) / ctx.get_str("common.model.file", "tfe.pt") if mdir else None)
    data = torch.from_numpy(np.loadtxt(_input(ctx, "train.data.file" if mode == "train" else "encode.data.file"),
                                       delimiter=",", ndmin=2)).float()
    if mode == "train":
        ae.fit(data, seed=args.seed)
        ctx.check()
        if mpath is not None and ctx.is_root:
            mpath.parent.mkdir(parents=True, exist_ok=True)
            ae.save(mpath)
        ctx.report({"final_loss": ae.losses[-1] if ae.losses else None, "iterations": len(ae.losses)})
    elif mode == "encode":
        if mpath is None:
            raise SystemExit("encode needs --model or common.model.directory")
        ae.restore(mpath)
        codes = ae.encode(data).cpu().tolist()
        _out(ctx, [",".join(f"{x:.6f}" for x in r) for r in codes])
    else:
        raise SystemExit("invalid command")


# ------------------------------------------------------------------------------------------------
def _units(ctx: JobContext, key_dir: str, key_file: str):
    """Document- or sentence-granularity training units (``train.text.granularity``)."""
    from ..text.preprocess import DocSentences
    gran = ctx.get_str("train.text.granularity", "document")
    if gran == "document":
        texts, names = _docs(_input(ctx, key_dir))
        return _clean(texts), names
    ds = DocSentences(_input(ctx, key_file), ctx.get_int("train.min.sentence.length", 5))
    return ds.getSentencesAsTokens(), ds.getSentences()


@job("docToVec", "PV-DBOW document / sentence vectors (P/app/dvd.py): --mode train|genVec|neighbor",
     aliases=("dvd",))
def doc_to_vec(args):
    """``train`` fits on ``train.data.dir`` (documents) or ``train.data.file`` (sentences) and
    writes the vectors to ``--model`` (safetensors, the units' names as metadata); ``genVec``
    writes them as CSV lines; ``neighbor --name <index>`` ranks all units by
    ``distance.algorithm`` (cosine | euclidean) from unit <index>."""
    from safetensors import safe_open
    from safetensors.torch import save_file
    from ..text.models import Doc2Vec
    ctx = JobContext(args)
    mode = args.mode or "train"
    if mode == "train":
        units, names = _units(ctx, "train.data.dir", "train.data.file")
        m = Doc2Vec(dim=ctx.get_int("train.vector.size", 100), window=ctx.get_int("train.window", 5),
                    negative=ctx.get_int("train.negative", 5), min_count=ctx.get_int("train.min.word.count", 1),
                    epochs=ctx.get_int("train.epochs", 20), seed=args.seed, device=ctx.device).fit(units)
        if not args.model:
            raise SystemExit("train needs --model <file>")
        if ctx.is_root:
            save_file({"D": m.doc_vectors().cpu().contiguous()}, args.model, metadata={"names": json.dumps(names)})
        ctx.report({"units": len(units), "dim": m.dim})
        return
    with safe_open(args.model, "pt") as f:
        D, names = f.get_tensor("D").to(ctx.device), json.loads(f.metadata()["names"])
    if mode == "genVec":
        _out(ctx, [",".join(f"{x:.6f}" for x in r) for r in D.tolist()])
    elif mode == "neighbor":
        i = int(args.name or 0)
        algo = ctx.get_str("distance.algorithm", "cosine")
        if algo == "cosine":
            Dn = torch.nn.functional.normalize(D, dim=1)
            dist = 1.0 - Dn @ Dn[i]
        else:
            dist = (D - D[i]).norm(dim=1)
        order = torch.argsort(dist).tolist()
        _out(ctx, [f"{j},{names[j]},{float(dist[j]):.6f}" for j in order if j != i])
    else:
        raise SystemExit("invalid operation")


@job("wordToVec", "skip-gram word vectors (P/app/wvd.py): --mode train|fsw (--name words, comma separated)",
     aliases=("wvd",))
def word_to_vec(args):
    from ..text.models import Word2Vec
    ctx = JobContext(args)
    mode = args.mode or "train"
    if mode == "train":
        texts, _ = _docs(_input(ctx, "train.data.dir"))
        m = Word2Vec(dim=ctx.get_int("train.vector.size", 100), window=ctx.get_int("train.window", 5),
                     negative=ctx.get_int("train.negative", 5), min_count=ctx.get_int("train.min.word.count", 1),
                     epochs=ctx.get_int("train.epochs", 5), seed=args.seed, device=ctx.device).fit(_clean(texts))
        if not args.model:
            raise SystemExit("train needs --model <file>")
        ctx.check()
        if ctx.is_root:
            m.save(args.model)
        ctx.report({"vocab": len(m.vocab.index), "dim": m.dim})
    elif mode == "fsw":
        m = Word2Vec.load(args.model, device=ctx.device)
        k = int(args.k or 5)
        lines = []
        for w in (args.name or "").split(","):
            lines.append(json.dumps({"word": w, "similar": [[s, round(v, 6)] for s, v in m.most_similar(w, k)]}))
        _out(ctx, lines)
    else:
        raise SystemExit("invalid operation")


@job("textClassifier", "bag-of-words naive Bayes text classifier (P/app/classify.py): --input labelled corpus, "
     "--name test text", aliases=("classify",))
def text_classifier(args):
    """Input: a directory with one sub-directory per class (the movie-review layout), or a file of
    ``text<delim>label`` lines.  The first ``test.size`` (default 100) documents after a seeded
    shuffle are held out (classify.py:63); prints accuracy, the most informative words and, with
    ``--name``, the class of that text."""
    import random
    from ..text.models import TextNaiveBayes
    ctx = JobContext(args)
    p = Path(_input(ctx))
    if p.is_dir():
        pairs = [(f.read_text(errors="ignore"), c.name) for c in sorted(p.iterdir()) if c.is_dir()
                 for f in sorted(c.iterdir()) if f.is_file()]
    else:
        sp = ctx.split
        pairs = []
        for l in ctx.all_lines():
            parts = sp(l)
            pairs.append((ctx.delim_in.join(parts[:-1]), parts[-1]))
    random.Random(args.seed).shuffle(pairs)
    docs = _clean([t for t, _ in pairs])
    labels = [c for _, c in pairs]
    n_test = min(ctx.get_int("test.size", 100), max(len(docs) - 1, 0))
    nb = TextNaiveBayes(device=ctx.device).fit(docs[n_test:], labels[n_test:])
    res = {"accuracy": nb.accuracy(docs[:n_test], labels[:n_test]) if n_test else None,
           "classes": nb.classes}
    if len(nb.classes) == 2:
        res["informative"] = [[w, round(v, 4)] for w, v in nb.most_informative(10)]
    if args.name:
        res["prediction"] = nb.predict(_clean([args.name]))[0]
    ctx.report(res)


@job("semanticSearch", "semantic document search (P/app/ssearch.py): --mode <algo> --name query over the --input corpus",
     aliases=("ssearch",))
def semantic_search(args):
    """Algorithms: tokenMax, tokenAvMax, tokenMaxAv, tokenAv, tokenMed, sentAv, sentMed, sentMax,
    docAv (text/semsearch.py).  Embedder: with ``bert.model.dir`` (a directory holding a Hugging
    Face BERT ``config.json``, ``model.safetensors`` or ``pytorch_model.bin`` and ``vocab.txt`` —
    e.g. bert-base-uncased, the model behind the reference's spaCy pipeline) the contextual token
    vectors of nn/bert.py; otherwise a skip-gram embedder trained on the corpus itself."""
    from ..text.semsearch import ALGOS, SemanticSearch, search_corpus
    ctx = JobContext(args)
    algo = args.mode or "tokenAvMax"
    if algo not in ALGOS:
        raise SystemExit(f"invalid algorithm {algo}; one of {', '.join(ALGOS)}")
    texts, names = _docs(_input(ctx))
    bert_dir = ctx.get("bert.model.dir", None)
    if bert_dir:
        import os
        from ..nn.bert import BertEncoder, WordPiece, bert_embedder
        enc = BertEncoder.from_pretrained_dir(bert_dir, device=ctx.device)
        vocab = os.path.join(bert_dir, "vocab.txt")
        ss = SemanticSearch(bert_embedder(enc, WordPiece(vocab if os.path.exists(vocab) else None,
                                                         enc.config.vocab_size)), device=ctx.device)
        ss.add_many(texts)                 # the corpus in batched encoder passes
    else:
        ss = search_corpus(texts, dim=ctx.get_int("embed.dim", 100), epochs=ctx.get_int("embed.epochs", 10),
                           device=ctx.device, seed=args.seed)
    top = int(args.k or len(texts))
    _out(ctx, [f"{i},{names[i]},{s:.6f}" for i, s in ss.search(args.name or "", algo, top)])
