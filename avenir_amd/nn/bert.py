"""BERT encoder for semantic search (the reference's P/app/ssearch.py:184-300 embeds
documents and queries with spaCy-transformers' ``en_trf_bertbaseuncased_lg`` and compares their
token / sentence vectors).

The module takes a Hugging Face BERT state dict as is (``BertModel`` parameter names, loaded with
``torch.load(weights_only=True)`` or safetensors) and a WordPiece vocabulary (``tokenizers``), so a
user's bert-base-uncased checkpoint drops in; no weights ship with the framework (none can be
fetched here), and the tests pin the ARCHITECTURE against ``transformers.BertModel`` with random
weights instead.

MI355X path (inference, fp32 like the reference's model):
* embeddings: word + position + token-type gathers, the sum and the LayerNorm in ONE kernel
  (transformer.hip ``embed_layernorm_kernel``; host token ids are range-checked before their
  upload, so no device synchronisation per pass);
* per layer: the Q, K, V projections as ONE GEMM with concatenated weights; attention in ONE
  transformer.hip kernel (``attn_f32_kernel``, head dim 64: scores, mask, online softmax and
  context on fp32 MFMA, read from the fused [B*S, 3H] projection and written as [B*S, H], no head
  transposes; torch's fused attention for other head sizes); the output projection with its bias,
  the residual and the LayerNorm in one split-K + LayerNorm pass (``linear_add_layernorm``); the
  feed-forward up-projection with bias + GELU in the tile epilogue; the down-projection fused with
  its residual + LayerNorm the same way.  Projections of up to ``MFMA_MAX_ROWS`` rows (a query, a
  short document) run on mlp.hip's f32-MFMA tile kernel (split over K when it has few output
  tiles); larger batches on hipBLASLt (profiles/r5_bert_base_bench.jsonl).
CPU tensors run the same math with torch ops.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import asdict, dataclass, fields

import torch

from .. import _native
from ..utils.params import param_epoch

#: activation code of mlp.hip's linear_act_fwd for the erf GELU
_GELU = 6


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    layer_norm_eps: float = 1e-12
    hidden_act: str = "gelu"

    @classmethod
    def from_dict(cls, d: dict) -> "BertConfig":
        names = {f.name for f in fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in names})

    @classmethod
    def from_json(cls, path: str) -> "BertConfig":
        with open(path) as fh:
            return cls.from_dict(json.load(fh))

    def to_dict(self) -> dict:
        return asdict(self)


def _layer_names(i: int) -> dict:
    p = f"encoder.layer.{i}."
    return {"q": p + "attention.self.query", "k": p + "attention.self.key", "v": p + "attention.self.value",
            "o": p + "attention.output.dense", "ln1": p + "attention.output.LayerNorm",
            "up": p + "intermediate.dense", "down": p + "output.dense", "ln2": p + "output.LayerNorm"}


class BertEncoder(torch.nn.Module):
    """``forward(input_ids [B, S], attention_mask [B, S] = None, token_type_ids = None) ->
    last hidden state [B, S, H]`` — the same function as ``transformers.BertModel(...)
    .last_hidden_state`` (eval mode), parameters under the same names."""

    def __init__(self, config: BertConfig):
        super().__init__()
        if config.hidden_act not in ("gelu",):
            raise ValueError(f"hidden_act {config.hidden_act!r}: only the erf GELU of bert-base is implemented")
        if config.hidden_size % config.num_attention_heads:
            raise ValueError("hidden_size must be a multiple of num_attention_heads")
        self.config = config
        H, I = config.hidden_size, config.intermediate_size
        P = torch.nn.Parameter
        self.params = torch.nn.ParameterDict()

        def add(name, *shape, ones=False):
            t = torch.ones(*shape) if ones else torch.zeros(*shape)
            self.params[name.replace(".", "__")] = P(t)

        add("embeddings.word_embeddings.weight", config.vocab_size, H)
        add("embeddings.position_embeddings.weight", config.max_position_embeddings, H)
        add("embeddings.token_type_embeddings.weight", config.type_vocab_size, H)
        add("embeddings.LayerNorm.weight", H, ones=True)
        add("embeddings.LayerNorm.bias", H)
        for i in range(config.num_hidden_layers):
            n = _layer_names(i)
            for k in ("q", "k", "v", "o"):
                add(n[k] + ".weight", H, H)
                add(n[k] + ".bias", H)
            add(n["up"] + ".weight", I, H)
            add(n["up"] + ".bias", I)
            add(n["down"] + ".weight", H, I)
            add(n["down"] + ".bias", H)
            for k in ("ln1", "ln2"):
                add(n[k] + ".weight", H, ones=True)
                add(n[k] + ".bias", H)
        self._qkv_cache: dict = {}
        self.reset_parameters()

    def reset_parameters(self, std: float = 0.02, seed: int = 0):
        g = torch.Generator().manual_seed(seed)
        for name, p in self.params.items():
            if name.endswith("weight") and p.dim() == 2:
                with torch.no_grad():
                    p.copy_(torch.randn(p.shape, generator=g) * std)

    def p(self, name: str) -> torch.Tensor:
        return self.params[name.replace(".", "__")]

    # -- loading -------------------------------------------------------------------------------
    def load_hf_state_dict(self, sd: dict, strict: bool = True) -> "BertEncoder":
        """A ``transformers.BertModel`` state dict (keys with or without the ``bert.`` prefix of
        task models; the pooler and heads are ignored)."""
        own = {k.replace("__", "."): k for k in self.params.keys()}
        seen = set()
        for k, v in sd.items():
            kk = k[5:] if k.startswith("bert.") else k
            if kk in own:
                tgt = self.params[own[kk]]
                if tuple(tgt.shape) != tuple(v.shape):
                    raise ValueError(f"{k}: shape {tuple(v.shape)} != {tuple(tgt.shape)}")
                with torch.no_grad():
                    tgt.copy_(v.to(tgt.dtype))
                seen.add(kk)
        missing = set(own) - seen
        if strict and missing:
            raise KeyError(f"missing BERT parameters: {sorted(missing)[:5]} ...")
        self._qkv_cache.clear()
        self.__dict__.pop("_planes_cache", None)
        return self

    @classmethod
    def from_pretrained_dir(cls, path: str, device="cpu") -> "BertEncoder":
        """A directory with ``config.json`` and ``model.safetensors`` or ``pytorch_model.bin``
        (loaded without executing anything from the file)."""
        cfg = BertConfig.from_json(os.path.join(path, "config.json"))
        m = cls(cfg)
        st = os.path.join(path, "model.safetensors")
        if os.path.exists(st):
            from safetensors.torch import load_file
            sd = load_file(st)
        else:
            sd = torch.load(os.path.join(path, "pytorch_model.bin"), map_location="cpu", weights_only=True)
        return m.load_hf_state_dict(sd).to(device).eval()

    # -- forward -------------------------------------------------------------------------------
    def _qkv(self, i: int):
        """[3H, H] weights and [3H] bias of layer i's Q, K, V (cached per parameter version)."""
        n = _layer_names(i)
        ps = [self.p(n[k] + s) for k in ("q", "k", "v") for s in (".weight", ".bias")]
        key = (i, param_epoch()) + tuple((t.data_ptr(), t._version) for t in ps)
        hit = self._qkv_cache.get(i)
        if hit is not None and hit[0] == key:
            return hit[1], hit[2]
        if hit is not None:                 # the old fused weight's planes go with it
            self.__dict__.get("_planes_cache", {}).pop((hit[1].data_ptr(), tuple(hit[1].shape)), None)
        W = torch.cat([ps[0], ps[2], ps[4]], 0).detach().contiguous()
        b = torch.cat([ps[1], ps[3], ps[5]], 0).detach().contiguous()
        self._qkv_cache[i] = (key, W, b)
        return W, b

    #: rows from which the projections run on hipBLASLt (+ a separate erf-GELU pass) instead of the
    #: tile kernels with the GELU epilogue.  Round 5 (exact-f32 MFMA tiles) stopped at 1,024 rows
    #: (8.2 vs 6.6 ms per pass at 4-16 k rows); the split-bf16 tiles beat hipBLASLt's fp32 GEMM at
    #: every bert-base shape (1.4-1.6x at 4,096 rows, profiles/r6_gemm_*.jsonl), so no limit by default
    MFMA_MAX_ROWS = int(os.environ.get("AVMI_BERT_MFMA_MAX_ROWS", str(1 << 62)))
    #: arithmetic of the projections (mlp.hip prec): 3 = split-bf16 x3 (inference default: max error
    #: ~2e-5 at unit-scale activations, inside the fp32 parity bar against transformers), 6 = x6
    #: (fp32-level error), 0 = exact-f32 MFMA.  AVMI_BERT_GEMM = bf16x3 | bf16x6 | f32
    GEMM_PREC = {"bf16x3": 3, "bf16x6": 6, "f32": 0}[os.environ.get("AVMI_BERT_GEMM", "bf16x3")]

    def _weight_planes(self, x2, W):
        """W's cached bf16 term planes when this call takes mlp.hip's pre-split planes path (large
        row counts): the weight is split once per (W, version, optimiser epoch), not per call."""
        C = _native.C()
        if C.linear_act_fwd_planes_bytes(x2.shape[0], W.shape[0], W.shape[1], self.GEMM_PREC) == 0:
            return None
        # keyed by storage (callers pass fresh .detach() views; a detached view shares the
        # parameter's version counter); the entry holds W, so its address cannot be reused by
        # another tensor while cached
        cache = self.__dict__.setdefault("_planes_cache", {})
        addr = (W.data_ptr(), tuple(W.shape))
        key = (W._version, param_epoch(), self.GEMM_PREC)
        hit = cache.get(addr)
        if hit is not None and hit[1] == key:
            return hit[2]
        p = C.sbf16_weight_planes(W.detach(), self.GEMM_PREC)
        cache[addr] = (W, key, p)
        return p

    def _linear(self, x2, W, b, act: int = 0):
        if x2.is_cuda and x2.shape[0] <= self.MFMA_MAX_ROWS:
            return _native.C().linear_act_fwd(x2, W, b, act, self.GEMM_PREC, self._weight_planes(x2, W))
        y = torch.nn.functional.linear(x2, W, b)
        return torch.nn.functional.gelu(y) if act == _GELU else y

    def _add_ln(self, x, res, g, b):
        eps = self.config.layer_norm_eps
        if x.is_cuda:
            return _native.C().add_layernorm(x.contiguous(), None if res is None else res.contiguous(), g.detach(),
                                             b.detach(), eps)
        return torch.nn.functional.layer_norm(x if res is None else x + res, (x.shape[-1],), g, b, eps)

    def _check_ids(self, ids: torch.Tensor, tt: torch.Tensor | None) -> None:
        """Range check of HOST token ids / types (no device synchronisation)."""
        V, T = self.config.vocab_size, self.config.type_vocab_size
        if ids.numel() and (int(ids.min()) < 0 or int(ids.max()) >= V):
            raise RuntimeError("BertEncoder: token id out of range")
        if tt is not None and tt.numel() and (int(tt.min()) < 0 or int(tt.max()) >= T):
            raise RuntimeError("BertEncoder: token type out of range")

    def _apply(self, fn, *a, **k):          # .to() / .cuda(): the Q/K/V cache holds the old storage
        self._qkv_cache.clear()
        self.__dict__.pop("_planes_cache", None)
        return super()._apply(fn, *a, **k)

    def _linear_ln(self, x2, W, b, res, g, bb):
        """LN(x2 W^T + b + res): one fused split-K + LayerNorm pass for a query's rows on the GPU."""
        N = W.shape[0]
        if x2.is_cuda and x2.shape[0] <= self.MFMA_MAX_ROWS and N <= 1024 and N % 4 == 0:
            return _native.C().linear_add_layernorm(x2, W, b, res.contiguous(), g.detach(), bb.detach(),
                                                    self.config.layer_norm_eps, self.GEMM_PREC,
                                                    self._weight_planes(x2, W))
        return self._add_ln(self._linear(x2, W, b), res, g, bb)

    @torch.no_grad()
    def forward(self, input_ids: torch.Tensor, attention_mask: torch.Tensor | None = None,
                token_type_ids: torch.Tensor | None = None) -> torch.Tensor:
        """Last hidden states [B, S, H].  Inputs may be host tensors (checked on the host, then
        uploaded) or device tensors (checked by one device -> host copy)."""
        dev = self.p("embeddings.word_embeddings.weight").device
        if dev.type != "cuda":
            return self._forward(input_ids, attention_mask, token_type_ids, True)
        validated = False
        if not input_ids.is_cuda:
            self._check_ids(input_ids, token_type_ids)
            validated = True
        ids = input_ids.to(dev, torch.long).contiguous()
        tt = None if token_type_ids is None else token_type_ids.to(dev, torch.long).contiguous()
        mask = None if attention_mask is None else attention_mask.to(dev)
        return self._forward(ids, mask, tt, not validated)

    def _forward(self, input_ids, attention_mask, token_type_ids, validate: bool) -> torch.Tensor:
        cfg = self.config
        B, S = input_ids.shape
        H, nh = cfg.hidden_size, cfg.num_attention_heads
        dh = H // nh
        ids = input_ids.long().contiguous()
        tt = None if token_type_ids is None else token_type_ids.long().contiguous()
        word, pos = self.p("embeddings.word_embeddings.weight"), self.p("embeddings.position_embeddings.weight")
        typ = self.p("embeddings.token_type_embeddings.weight")
        g0, b0 = self.p("embeddings.LayerNorm.weight"), self.p("embeddings.LayerNorm.bias")
        if ids.is_cuda:
            x = _native.C().embed_layernorm(ids, tt, word.detach(), pos.detach(), typ.detach(), g0.detach(),
                                            b0.detach(), cfg.layer_norm_eps, validate)
        else:
            e = word[ids] + typ[tt if tt is not None else torch.zeros_like(ids)] + pos[:S].unsqueeze(0)
            x = torch.nn.functional.layer_norm(e, (H,), g0, b0, cfg.layer_norm_eps)
        # additive mask: 0 where attended, the dtype minimum where padded (as transformers)
        bias = None
        if attention_mask is not None:
            m = attention_mask.to(x.dtype).view(B, 1, 1, S)
            bias = (1.0 - m) * torch.finfo(x.dtype).min
        kbias = None if bias is None else bias.view(B, S).contiguous()
        scale = 1.0 / math.sqrt(dh)
        for i in range(cfg.num_hidden_layers):
            n = _layer_names(i)
            x2 = x.reshape(B * S, H)
            Wqkv, bqkv = self._qkv(i)
            qkv2 = self._linear(x2, Wqkv, bqkv)                                   # [B*S, 3H]
            if qkv2.is_cuda and dh == 64:
                # transformer.hip attention: straight from [B*S, 3H] to [B*S, H], no head transposes
                ctx = _native.C().attention_f32(qkv2, kbias, B, S, nh, scale)
            else:
                qkv = qkv2.view(B, S, 3, nh, dh).permute(2, 0, 3, 1, 4)            # [3, B, nh, S, dh]
                ctx = torch.nn.functional.scaled_dot_product_attention(qkv[0], qkv[1], qkv[2], attn_mask=bias,
                                                                       scale=scale)
                ctx = ctx.permute(0, 2, 1, 3).reshape(B * S, H)
            x2 = self._linear_ln(ctx.contiguous(), self.p(n["o"] + ".weight").detach(), self.p(n["o"] + ".bias").detach(),
                                 x2, self.p(n["ln1"] + ".weight"), self.p(n["ln1"] + ".bias"))
            h = self._linear(x2, self.p(n["up"] + ".weight").detach(), self.p(n["up"] + ".bias").detach(), _GELU)
            x = self._linear_ln(h, self.p(n["down"] + ".weight").detach(), self.p(n["down"] + ".bias").detach(),
                                x2, self.p(n["ln2"] + ".weight"), self.p(n["ln2"] + ".bias")).view(B, S, H)
        return x


class WordPiece:
    """BERT's uncased WordPiece tokenizer over a ``vocab.txt`` (the ``tokenizers`` library), or —
    for tests without a vocabulary — a hashing stand-in mapping each word to one id."""

    def __init__(self, vocab_path: str | None = None, vocab_size: int = 30522, lowercase: bool = True):
        self.vocab_size = vocab_size
        self.tok = None
        if vocab_path is not None:
            from tokenizers import BertWordPieceTokenizer
            self.tok = BertWordPieceTokenizer(vocab_path, lowercase=lowercase)
            self.vocab_size = self.tok.get_vocab_size()
        self.cls_id, self.sep_id = (self.tok.token_to_id("[CLS]"), self.tok.token_to_id("[SEP]")) if self.tok else (1, 2)

    def word_ids(self, word: str) -> list[int]:
        if self.tok is not None:
            return self.tok.encode(word, add_special_tokens=False).ids or [self.tok.token_to_id("[UNK]")]
        import zlib
        return [3 + zlib.crc32(word.encode()) % (self.vocab_size - 3)]


def bert_embedder(model: BertEncoder, tokenizer: WordPiece, max_len: int | None = None, batch_tokens: int = 8192):
    """``embed(tokens) -> [n_tokens, H]`` contextual token vectors for :class:`~avenir_amd.text.
    semsearch.SemanticSearch`: the token sequence is encoded as ONE [CLS] ... [SEP] input (windows
    of ``max_len`` word pieces for long texts), and each token's vector is the mean of its word
    pieces' last hidden states — the alignment spaCy-transformers uses for ``token.vector``.

    ``embed.many(list of token lists) -> list of [n_i, H]`` does the same for many inputs at once:
    all their windows, sorted by length, go through the encoder as padded batches of up to
    ``batch_tokens`` tokens (attention mask on the padding) — a corpus is encoded in a few large
    passes instead of one small pass per document (bert-base: 32 x 128 tokens in 6.2 ms against
    1.1 ms per single 128-token pass)."""
    dev = next(model.parameters()).device
    H = model.config.hidden_size
    L = max_len or model.config.max_position_embeddings
    step = L - 2

    def windows(tokens):
        pieces, owner = [], []
        for t, w in enumerate(tokens):
            ids = tokenizer.word_ids(w)
            pieces += ids
            owner += [t] * len(ids)
        return [([tokenizer.cls_id] + pieces[s0:s0 + step] + [tokenizer.sep_id], owner[s0:s0 + step])
                for s0 in range(0, len(pieces), step)]

    def emb(tokens):
        if not tokens:
            return torch.zeros((0, H), device=dev)
        out = torch.zeros((len(tokens), H), device=dev)
        cnt = torch.zeros(len(tokens), device=dev)
        for ids, own in windows(tokens):
            h = model(torch.tensor([ids]))[0, 1:-1]          # host ids: checked on the host, then uploaded
            ow = torch.tensor(own, device=dev)
            out.index_add_(0, ow, h)
            cnt.index_add_(0, ow, torch.ones_like(ow, dtype=torch.float32))
        return out / cnt.clamp_min(1).view(-1, 1)

    def many(token_lists):
        outs = [torch.zeros((len(t), H), device=dev) for t in token_lists]
        cnts = [torch.zeros(len(t), device=dev) for t in token_lists]
        wins = [(i, ids, own) for i, t in enumerate(token_lists) if t for ids, own in windows(t)]
        wins.sort(key=lambda w: len(w[1]))
        b0 = 0
        while b0 < len(wins):
            S = len(wins[b0][1])
            b1 = b0 + 1                       # grow the batch while the padded size fits the budget
            while b1 < len(wins) and (b1 + 1 - b0) * len(wins[b1][1]) <= batch_tokens:
                b1 += 1
            grp = wins[b0:b1]
            S = len(grp[-1][1])
            ids = torch.zeros((len(grp), S), dtype=torch.long)
            mask = torch.zeros((len(grp), S), dtype=torch.long)
            for r, (_, w, _) in enumerate(grp):
                ids[r, :len(w)] = torch.tensor(w)
                mask[r, :len(w)] = 1
            h = model(ids, mask)                               # [b, S, H]
            for r, (i, w, own) in enumerate(grp):
                ow = torch.tensor(own, device=dev)
                outs[i].index_add_(0, ow, h[r, 1:len(w) - 1])
                cnts[i].index_add_(0, ow, torch.ones_like(ow, dtype=torch.float32))
            b0 = b1
        return [o / c.clamp_min(1).view(-1, 1) for o, c in zip(outs, cnts)]

    emb.model = model
    emb.many = many
    return emb
