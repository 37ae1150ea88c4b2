"""CLI text drivers (P/app/summd.py, topic.py, tf.py, tfe.py, dvd.py, wvd.py, classify.py,
ssearch.py) run through ``avenir_amd.cli.main`` on small seeded corpora; each stage is compared
with the library call it wraps."""
import json
import random

import pytest
import torch

from avenir_amd.cli import JOBS, main

TOPICS = {
    "autos": "car engine wheel brake tire fuel driver road speed garage motor gear".split(),
    "med": "doctor patient hospital disease medicine nurse surgery drug health clinic therapy".split(),
    "space": "rocket orbit planet launch astronaut moon satellite galaxy telescope mission star".split(),
}


def _corpus(tmp_path, n_per=12, seed=0):
    rng = random.Random(seed)
    d = tmp_path / "docs"
    d.mkdir()
    for t, words in TOPICS.items():
        for i in range(n_per):
            sents = []
            for _ in range(6):
                sents.append(" ".join(rng.choice(words) for _ in range(9)).capitalize() + ".")
            (d / f"{t}_{i:02d}.txt").write_text(" ".join(sents))
    return d


def test_text_jobs_registered():
    for name in ("textSummarizer", "summd", "topicModel", "topic", "termDistribution", "tf", "textEncoder",
                 "tfe", "docToVec", "dvd", "wordToVec", "wvd", "textClassifier", "classify",
                 "semanticSearch", "ssearch"):
        assert name in JOBS


def test_summarizers(tmp_path):
    from avenir_amd.text.models import TermFreqSumm
    doc = tmp_path / "doc.txt"
    rng = random.Random(1)
    words = TOPICS["autos"] + TOPICS["med"]
    doc.write_text(" ".join(" ".join(rng.choice(words) for _ in range(8)).capitalize() + "." for _ in range(20)))
    props = tmp_path / "summ.properties"
    props.write_text(f"common.data.file={doc}\ncommon.size=3\ncommon.show.score=true\n")
    for op in ("tfSumm", "sbSumm", "lsSumm", "nmfSumm", "trSumm"):
        out = tmp_path / f"{op}.txt"
        assert main(["textSummarizer", "--config", str(props), "--mode", op, "--output", str(out)]) in (0, None)
        lines = out.read_text().splitlines()
        assert len(lines) == 3 and all(l.endswith(")") for l in lines)
    lib = TermFreqSumm(size=3).summarize(str(doc))
    got = (tmp_path / "tfSumm.txt").read_text().splitlines()
    assert [l.rsplit("  (", 1)[0] for l in got] == [s for s, _ in lib]


def test_topic_train_analyze(tmp_path):
    d = _corpus(tmp_path)
    model = tmp_path / "lda.safetensors"
    out = tmp_path / "topics.txt"
    main(["topicModel", "--mode", "train", "--input", str(d), "--model", str(model), "--output", str(out),
          "-D", "train.num.topics=3", "-D", "train.num.iter=40"])
    recs = [json.loads(l) for l in out.read_text().splitlines()]
    docs = [r for r in recs if "doc" in r]
    assert len(docs) == 36
    # documents of one generating topic share their leading LDA topic
    lead = {}
    for r in docs:
        lead.setdefault(r["doc"].rsplit("/", 1)[1].split("_")[0], []).append(r["topics"][0][0])
    for t, ks in lead.items():
        assert max(ks.count(k) for k in set(ks)) >= 10, (t, ks)
    out2 = tmp_path / "an.txt"
    main(["topicModel", "--mode", "analyze", "--input", str(d), "--model", str(model), "--output", str(out2)])
    an = [json.loads(l) for l in out2.read_text().splitlines() if '"doc"' in l]
    same = sum(a["topics"][0][0] == b["topics"][0][0] for a, b in zip(an, docs))
    assert same >= 34


def test_term_distribution_diff(tmp_path):
    d = _corpus(tmp_path)
    base = tmp_path / "base"
    base.mkdir()
    for f in sorted(d.iterdir())[:12]:           # autos only
        (base / f.name).write_text(f.read_text())
    bf = tmp_path / "base.json"
    main(["termDistribution", "--mode", "buildBaseTf", "--input", str(base), "--model", str(bf)])
    out = tmp_path / "diff.txt"
    main(["termDistribution", "--mode", "tfDiff", "--input", str(d), "--model", str(bf), "--output", str(out)])
    words = [l.split(",")[0] for l in out.read_text().splitlines()]
    # words absent from the base distribution rank first; no autos word has a positive entropy term
    assert set(words) <= set(TOPICS["med"]) | set(TOPICS["space"]) | set(TOPICS["autos"])
    assert set(TOPICS["med"]) | set(TOPICS["space"]) <= set(words)


def test_text_encoder_vectorise_train_encode(tmp_path):
    d = _corpus(tmp_path, n_per=5)
    vec = tmp_path / "vec.csv"
    main(["textEncoder", "--mode", "vectorise", "--kind", "bi", "--input", str(d), "--output", str(vec)])
    rows = [list(map(float, l.split(","))) for l in vec.read_text().splitlines()]
    assert rows and all(abs(sum(r) - 1) < 1e-4 for r in rows)
    width = len(rows[0])
    props = tmp_path / "ae.properties"
    props.write_text(f"train.num.input={width}\ntrain.num.hidden.units=4\ntrain.encoder.activations=relu\n"
                     f"train.decoder.activations=none\ntrain.num.iterations=5\ntrain.batch.size=4\n"
                     f"train.data.file={vec}\nencode.data.file={vec}\ncommon.device=cpu\n")
    m = tmp_path / "ae.pt"
    main(["textEncoder", "--mode", "train", "--config", str(props), "--model", str(m), "--device", "cpu"])
    enc = tmp_path / "enc.csv"
    main(["textEncoder", "--mode", "encode", "--config", str(props), "--model", str(m), "--output", str(enc),
          "--device", "cpu"])
    codes = enc.read_text().splitlines()
    assert len(codes) == len(rows) and len(codes[0].split(",")) == 4


def test_doc_and_word_vectors(tmp_path):
    d = _corpus(tmp_path)
    m = tmp_path / "d2v.safetensors"
    main(["docToVec", "--mode", "train", "--input", str(d), "--model", str(m), "-D", "train.vector.size=32",
          "-D", "train.epochs=30"])
    out = tmp_path / "nb.txt"
    main(["docToVec", "--mode", "neighbor", "--model", str(m), "--name", "0", "--output", str(out)])
    nbrs = [l.split(",")[1].rsplit("/", 1)[1] for l in out.read_text().splitlines()]
    assert len(nbrs) == 35
    assert sum(n.startswith("autos") for n in nbrs[:11]) >= 8
    w = tmp_path / "w2v.safetensors"
    main(["wordToVec", "--mode", "train", "--input", str(d), "--model", str(w), "-D", "train.vector.size=32",
          "-D", "train.epochs=10"])
    out2 = tmp_path / "fsw.txt"
    main(["wordToVec", "--mode", "fsw", "--model", str(w), "--name", "rocket", "--k", "5", "--output", str(out2)])
    sim = json.loads(out2.read_text().splitlines()[0])["similar"]
    assert len(sim) == 5 and sum(s in TOPICS["space"] for s, _ in sim) >= 3


def test_text_classifier_and_search(tmp_path, capsys):
    root = tmp_path / "lab"
    rng = random.Random(3)
    for c in ("autos", "med"):
        (root / c).mkdir(parents=True)
        for i in range(60):
            (root / c / f"{i}.txt").write_text(" ".join(rng.choice(TOPICS[c]) for _ in range(30)))
    main(["textClassifier", "--input", str(root), "--name", "the doctor and the nurse at the clinic",
          "-D", "test.size=20"])
    res = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert res["accuracy"] == 1.0 and res["prediction"] == "med" and len(res["informative"]) == 10
    d = _corpus(tmp_path)
    out = tmp_path / "ss.txt"
    main(["semanticSearch", "--mode", "tokenAvMax", "--input", str(d), "--name", "rocket orbit moon",
          "--k", "5", "--output", str(out)])
    hits = [l.split(",")[1].rsplit("/", 1)[1] for l in out.read_text().splitlines()]
    assert len(hits) == 5 and sum(h.startswith("space") for h in hits) >= 4


def test_text_encoder_vectorise_equals_per_document_vectors(tmp_path):
    """The one-scatter vectorise output == each document's getVector, formatted per value."""
    from avenir_amd.jobs.text_jobs import _clean, _docs
    from avenir_amd.text.preprocess import BiGram
    d = _corpus(tmp_path, n_per=20)
    out = tmp_path / "vec.csv"
    main(["textEncoder", "--mode", "vectorise", "--kind", "bi", "--input", str(d), "--output", str(out)])
    texts, _ = _docs(str(d))
    docs = _clean(texts)
    ng = BiGram()
    for x in docs:
        ng.countDocNGrams(x)
    ng.remLowCount(3)
    ref = []
    for x in docs:
        v = ng.getVector(x, True, True)
        if int((v != 0).sum()) > 0:
            ref.append(",".join(f"{y:.6f}" for y in v.tolist()))
    assert out.read_text().splitlines() == ref


def test_corpus_embedder_batched_adds_equal_one_by_one(tmp_path):
    """search_corpus adds the corpus through the embedder's batched lookup: same vectors as one
    add per document (vocabulary words and hashed unknown words alike)."""
    from avenir_amd.text.semsearch import SemanticSearch, corpus_embedder
    d = _corpus(tmp_path, n_per=4)
    docs = [f.read_text() for f in sorted(d.iterdir())] + ["zzz unknownword rocket.", ""]
    emb = corpus_embedder(docs, dim=16, epochs=2)
    one = SemanticSearch(emb)
    for x in docs:
        one.add(x)
    many = SemanticSearch(emb).add_many(docs)
    for a, b in zip(one.tok_emb + one.sent_emb, many.tok_emb + many.sent_emb):
        # the batched sentence means are one segmented sum (another summation order than .mean)
        assert a.shape == b.shape and torch.allclose(a, b, rtol=1e-5, atol=1e-6)
