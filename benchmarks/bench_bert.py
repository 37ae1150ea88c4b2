#!/usr/bin/env python3
"""BERT-base encoder inference (the semantic-search encoder of nn/bert.py, random weights in the
bert-base-uncased shape: 12 x 768, 12 heads, 3072) against transformers.BertModel on the same GPU,
fp32 (the reference's spaCy-transformers model runs fp32).  One JSON line per (batch, seq)."""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avenir_amd.nn.bert import BertConfig, BertEncoder  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    import transformers
    dev = torch.device("cuda")
    cfg = transformers.BertConfig()          # bert-base-uncased shape
    torch.manual_seed(0)
    ref = transformers.BertModel(cfg).eval().to(dev)
    mine = BertEncoder(BertConfig.from_dict(cfg.to_dict())).load_hf_state_dict(ref.state_dict()).to(dev).eval()
    for B, S in ((1, 128), (32, 128), (64, 256)):
        ids = torch.randint(0, cfg.vocab_size, (B, S), device=dev)
        mask = torch.ones(B, S, dtype=torch.long, device=dev)
        with torch.no_grad():
            want = ref(input_ids=ids, attention_mask=mask).last_hidden_state
            got = mine(ids, mask)
            err = float((got - want).abs().max())
            t_ref = timed(lambda: ref(input_ids=ids, attention_mask=mask))
            t_mine = timed(lambda: mine(ids, mask))
        print(json.dumps({"bench": "bert_base_encoder", "gemm": os.environ.get("AVMI_BERT_GEMM", "bf16x3"), "B": B, "S": S, "ours_ms": t_mine * 1e3,
                          "transformers_ms": t_ref * 1e3, "speedup": t_ref / t_mine, "max_abs_diff": err,
                          "tokens_per_s": B * S / t_mine}), flush=True)


def corpus():
    """semanticSearch's corpus encoding: 256 synthetic documents of ~100 words (5 sentences each),
    one encoder pass per document / sentence (``add``) against the batched ``add_many``."""
    import random
    from avenir_amd.nn.bert import WordPiece, bert_embedder
    from avenir_amd.text.semsearch import SemanticSearch
    torch.manual_seed(0)
    enc = BertEncoder(BertConfig()).to("cuda")
    emb = bert_embedder(enc, WordPiece())
    rnd = random.Random(0)
    words = [f"w{i}" for i in range(5000)]
    docs = [". ".join(" ".join(rnd.choice(words) for _ in range(20)) for _ in range(5)) + "." for _ in range(256)]
    res = {}
    for name, fn in (("add", lambda: [ss.add(d) for d in docs]), ("add_many", lambda: ss.add_many(docs))):
        ss = SemanticSearch(emb, device="cuda")
        fn()                                      # warm-up
        ss = SemanticSearch(emb, device="cuda")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        res[name] = time.perf_counter() - t0
    print(json.dumps({"bench": "semantic_search_corpus_encoding", "docs": len(docs), "add_s": res["add"],
                      "add_many_s": res["add_many"], "speedup": res["add"] / res["add_many"],
                      "docs_per_s": len(docs) / res["add_many"]}), flush=True)


if __name__ == "__main__":
    main()
    corpus()
