"""Counting ops (K2/K3/K4/moments).  GPU tensors -> hand-written HIP kernels (``_C``);
CPU tensors -> the PyTorch reference implementation of the same op (golden oracle)."""
from __future__ import annotations

import os

from dataclasses import dataclass
from typing import Sequence

import torch

from .. import _native


_CONST_CACHE: dict = {}


def _dev_i32(vals: Sequence[int], device) -> torch.Tensor:
    """Small int32 metadata tensors, cached per (values, device) so repeated launches do not pay a
    host->device copy (and its implicit synchronisation) every call."""
    key = (tuple(int(v) for v in vals), str(device))
    t = _CONST_CACHE.get(key)
    if t is None:
        if len(_CONST_CACHE) > 4096:
            _CONST_CACHE.clear()
        t = torch.tensor(list(key[0]), dtype=torch.int32, device=device)
        _CONST_CACHE[key] = t
    return t


def class_histogram(codes: torch.Tensor, n: int, bins: Sequence[int], labels: torch.Tensor | None,
                    n_classes: int, out: torch.Tensor | None = None, mode: int = 0,
                    count_labels: bool = False) -> torch.Tensor:
    """Class-conditional histogram ``out[c, off_f + b]`` (int64 ``[C, sum(bins)]``; with
    ``count_labels`` an extra last column holds the per-class record counts, fused in the same
    pass so no host synchronisation is needed).

    ``codes`` uint8 ``[F, ld]`` (feature-major), codes >= bins[f] (e.g. 255) are skipped;
    ``labels`` uint8 ``[>= n]`` or None (then C = 1).  ``mode``: 0 auto (packed byte-counter fast
    path when C*bins <= 16), 1 LDS path, 2 global-atomic path (for tests).
    """
    F = codes.shape[0]
    bins = [int(b) for b in bins]
    assert len(bins) == F, "bins length must equal number of feature rows"
    tb = sum(bins) + (1 if count_labels else 0)
    C = int(n_classes) if labels is not None else 1
    if out is None:
        out = torch.zeros((C, tb), dtype=torch.int64, device=codes.device)
    if (F == 0 and not count_labels) or n == 0:
        return out
    if codes.is_cuda:
        offs = [0] * F
        for f in range(1, F):
            offs[f] = offs[f - 1] + bins[f - 1]
        _native.C().class_histogram(codes.contiguous(), int(n),
                                    None if labels is None else labels.contiguous(),
                                    _dev_i32(bins, codes.device), _dev_i32(offs, codes.device),
                                    bins, tb, C, out, int(mode), bool(count_labels))
        return out
    # --- CPU reference ---
    lab = labels[:n].long() if labels is not None else torch.zeros(n, dtype=torch.long)
    if count_labels:
        ok = lab < C
        out[:, tb - 1] += torch.bincount(lab[ok], minlength=C)[:C]
    o = 0
    for f, b in enumerate(bins):
        v = codes[f, :n].long()
        ok = (v < b) & (lab < C)
        idx = lab[ok] * b + v[ok]
        out[:, o:o + b] += torch.bincount(idx, minlength=C * b).view(C, b)
        o += b
    return out


# ------------------------------------------------------------------------------------------------
# row-packed records: every categorical code of a record and its class in ONE 16-bit word
# ------------------------------------------------------------------------------------------------
@dataclass
class RowPacked:
    """Records packed one 16-bit word each (``pack_rows``): feature k's code in bits
    [shifts[k], shifts[k] + widths[k]) (its all-ones value = missing code); for C = 2 the class
    as two one-hot bits at label_shift (bit c set = class c, none set = unknown class)."""
    words: torch.Tensor      # int16 [>= n], numel a multiple of 8 (16-byte vector loads)
    n: int
    bins: list[int]
    shifts: list[int]
    widths: list[int]
    label_shift: int
    label_width: int         # 0: no class field (C = 1)
    n_classes: int
    dense: torch.Tensor | None = None   # GPU: the same records as a dense B-bit stream (pack_dense)
    bits: int = 16                      # B: bits per record actually used

    def ensure_dense(self) -> "RowPacked":
        """Attach the dense B-bit stream (32 records per B dwords, 1.6 B/record for churn) the
        joint-table kernel streams instead of the 16-bit words; GPU only, B in 4..15."""
        if self.dense is None and self.words.is_cuda and 4 <= self.bits <= 15 and self.n > 0:
            self.dense = _native.C().pack_dense(self.words, int(self.n), int(self.bits))
        return self


def rowpack_layout(bins: Sequence[int], n_classes: int, missing: Sequence[bool] | None = None):
    """(shifts, widths, label_shift, label_width) of the 16-bit record, or None when the schema
    does not fit: at most 8 features of at most 3 bits and 1 or 2 classes (C = 2: two one-hot
    class bits).  A feature with missing values takes bit_length(b) bits so its all-ones value
    (>= b) is free for 'missing'; one without (``missing[k]`` False) only bit_length(b - 1)."""
    bins = [int(b) for b in bins]
    C = int(n_classes)
    if missing is None:
        missing = [True] * len(bins)
    if not bins or len(bins) > 8 or C < 1 or C > 2 or min(bins) < 1:
        return None
    widths = [max(1, (b if m else b - 1).bit_length()) for b, m in zip(bins, missing)]
    if max(widths) > 3:
        return None
    lw = 2 if C == 2 else 0            # C = 2: class bits 0-1, the fields from bit 2
    shifts, s = [], lw
    for w in widths:
        shifts.append(s)
        s += w
    if s > 16:
        return None
    return shifts, widths, 0 if lw else s, lw


def pack_rows(codes: torch.Tensor, n: int, bins: Sequence[int], labels: torch.Tensor | None,
              n_classes: int) -> RowPacked | None:
    """Pack ``codes`` uint8 [F, >= n] (+ ``labels``) into one 16-bit word per record, on the
    tensors' device; None when ``rowpack_layout`` refuses the schema.  Codes >= bins[k] and
    labels >= C become the field's all-ones value, which every consumer skips — exactly the
    records the column histogram skips, so the counts are identical."""
    bins = [int(b) for b in bins]
    C = int(n_classes) if labels is not None else 1
    if labels is not None and C == 1:
        return None                      # a 1-class label column still filters rows: keep columns
    if codes.shape[0] != len(bins):
        return None
    # data-adaptive widths: a feature without missing codes needs no all-ones 'missing' value
    missing = [bool((codes[k, :n] >= b).any()) for k, b in enumerate(bins)] if n else [False] * len(bins)
    lay = rowpack_layout(bins, C, missing)
    if lay is None:
        return None
    shifts, widths, lsh, lw = lay
    w = torch.zeros(max(8, (n + 7) // 8 * 8), dtype=torch.int32, device=codes.device)
    body = w[:n]
    for k, (b, s, wd) in enumerate(zip(bins, shifts, widths)):
        v = codes[k, :n].to(torch.int32)
        body |= torch.where(v < b, v, torch.full_like(v, (1 << wd) - 1)) << s
    if lw:
        v = labels[:n].to(torch.int32)
        body |= torch.where(v < C, 1 << v.clamp_max(C - 1), torch.zeros_like(v)) << lsh
    words = torch.where(w >= 32768, w - 65536, w).to(torch.int16)
    bits = max([s + wd for s, wd in zip(shifts, widths)] + [lsh + lw])
    return RowPacked(words, int(n), bins, shifts, widths, lsh, lw, C, bits=bits).ensure_dense()


def unpack_rows(rp: RowPacked) -> tuple[torch.Tensor, torch.Tensor | None]:
    """Inverse of ``pack_rows``: (codes uint8 [F, pad16(n)], labels uint8 [pad16(n)] or None),
    missing / unknown values as 255."""
    n = rp.n
    ld = max(16, (n + 15) // 16 * 16)
    w = rp.words[:n].to(torch.int32) & 0xFFFF
    codes = torch.full((len(rp.bins), ld), 255, dtype=torch.uint8, device=w.device)
    for k, (b, s, wd) in enumerate(zip(rp.bins, rp.shifts, rp.widths)):
        v = (w >> s) & ((1 << wd) - 1)
        codes[k, :n] = torch.where(v < b, v, torch.full_like(v, 255)).to(torch.uint8)
    labels = None
    if rp.label_width:
        labels = torch.full((ld,), 255, dtype=torch.uint8, device=w.device)
        v = (w >> rp.label_shift) & ((1 << rp.label_width) - 1)
        cls = torch.full_like(v, 255)                                     # one-hot class bits
        for c in range(rp.n_classes):
            cls = torch.where(v == (1 << c), torch.full_like(v, c), cls)
        labels[:n] = cls.to(torch.uint8)
    return codes, labels


def class_histogram_packed(rp: RowPacked, out: torch.Tensor | None = None,
                           count_labels: bool = False) -> torch.Tensor:
    """``class_histogram`` over row-packed records (same ``[C, sum(bins) (+1)]`` int64 result).
    GPU: the K2 row-packed kernel streams 2 bytes per record (8 records per 16-byte load)
    instead of F + 1 bytes of code columns; CPU: unpack + the column reference."""
    C = rp.n_classes
    tb = sum(rp.bins) + (1 if count_labels else 0)
    if out is None:
        out = torch.zeros((C, tb), dtype=torch.int64, device=rp.words.device)
    if rp.n == 0:
        return out
    if rp.words.is_cuda:
        offs = [0] * len(rp.bins)
        for f in range(1, len(rp.bins)):
            offs[f] = offs[f - 1] + rp.bins[f - 1]
        # kernel order: features of <= 2 bits first (for C = 2 they share one counter per record
        # across both classes); output columns stay in schema order through offs
        order = sorted(range(len(rp.bins)), key=lambda k: (C == 2 and rp.widths[k] > 2, k))
        dev = rp.words.device
        kind = os.environ.get("AVMI_ROWPACK_KERNEL", "dense")
        if kind == "dense" and rp.dense is not None:
            # dense B-bit records, one LDS atomic per record into the joint table
            _native.C().class_histogram_dense(rp.dense, int(rp.n), int(rp.bits), list(rp.shifts), list(rp.widths),
                                              rp.label_shift, rp.label_width, _dev_i32(rp.bins, dev),
                                              _dev_i32(offs, dev), tb, C, out, bool(count_labels),
                                              list(rp.bins), offs)
            return out
        _native.C().class_histogram_rowpacked(rp.words, int(rp.n), [rp.shifts[k] for k in order],
                                              [rp.widths[k] for k in order], rp.label_shift, rp.label_width,
                                              _dev_i32([rp.bins[k] for k in order], dev),
                                              _dev_i32([offs[k] for k in order], dev), tb, C, out,
                                              bool(count_labels))
        return out
    codes, labels = unpack_rows(rp)
    return class_histogram(codes, rp.n, rp.bins, labels, C, out=out, count_labels=count_labels)


def pair_histogram(codes: torch.Tensor, n: int, bins: Sequence[int],
                   pairs: Sequence[tuple[int, int]], labels: torch.Tensor | None,
                   n_classes: int) -> list[torch.Tensor]:
    """Joint histograms for feature pairs: list of int64 ``[C, B_a, B_b]`` tensors."""
    bins = [int(b) for b in bins]
    C = int(n_classes) if labels is not None else 1
    sizes = [C * bins[a] * bins[b] for a, b in pairs]
    if not pairs:
        return []
    if codes.is_cuda:
        offs = [0] * len(pairs)
        for i in range(1, len(pairs)):
            offs[i] = offs[i - 1] + sizes[i - 1]
        flat = torch.zeros(sum(sizes), dtype=torch.int64, device=codes.device)
        pt = torch.tensor([list(p) for p in pairs], dtype=torch.int32, device=codes.device)
        po = torch.tensor(offs, dtype=torch.int64, device=codes.device)
        _native.C().pair_histogram(codes.contiguous(), int(n),
                                   None if labels is None else labels.contiguous(),
                                   _dev_i32(bins, codes.device), pt, po, max(sizes), C, flat)
        return [flat[o:o + s].view(C, bins[a], bins[b]) for o, s, (a, b) in zip(offs, sizes, pairs)]
    lab = labels[:n].long() if labels is not None else torch.zeros(n, dtype=torch.long)
    res = []
    for a, b in pairs:
        va, vb = codes[a, :n].long(), codes[b, :n].long()
        ok = (va < bins[a]) & (vb < bins[b]) & (lab < C)
        idx = (lab[ok] * bins[a] + va[ok]) * bins[b] + vb[ok]
        res.append(torch.bincount(idx, minlength=C * bins[a] * bins[b]).view(C, bins[a], bins[b]))
    return res


def bigram_histogram(states: torch.Tensor, n_states: int, labels: torch.Tensor | None = None,
                     n_classes: int = 1) -> torch.Tensor:
    """Markov transition counts ``[C, S, S]`` from int16 state sequences ``[N, L]`` (negative =
    padding)."""
    C = int(n_classes) if labels is not None else 1
    S = int(n_states)
    out = torch.zeros((C, S, S), dtype=torch.int64, device=states.device)
    if states.numel() == 0 or states.shape[1] < 2:
        return out
    if states.is_cuda:
        _native.C().bigram_histogram(states.to(torch.int16).contiguous(),
                                     None if labels is None else labels.contiguous(), C, S, out)
        return out
    a = states[:, :-1].long()
    b = states[:, 1:].long()
    lab = (labels[: states.shape[0]].long() if labels is not None
           else torch.zeros(states.shape[0], dtype=torch.long)).unsqueeze(1).expand_as(a)
    ok = (a >= 0) & (b >= 0) & (a < S) & (b < S) & (lab < C)
    idx = (lab[ok] * S + a[ok]) * S + b[ok]
    out += torch.bincount(idx, minlength=C * S * S).view(C, S, S)
    return out


def class_moments(x: torch.Tensor, n: int, labels: torch.Tensor | None, n_classes: int) -> torch.Tensor:
    """``[C, F, 3]`` float64 (count, sum, sum of squares) per class and continuous feature."""
    C = int(n_classes) if labels is not None else 1
    F = x.shape[0]
    if F == 0 or n == 0:
        return torch.zeros((C, F, 3), dtype=torch.float64, device=x.device)
    if x.is_cuda:
        return _native.C().class_moments(x.float().contiguous(), int(n),
                                         None if labels is None else labels.contiguous(), C)
    lab = labels[:n].long() if labels is not None else torch.zeros(n, dtype=torch.long)
    xv = x[:, :n].double()
    out = torch.zeros((C, F, 3), dtype=torch.float64)
    for c in range(C):
        m = lab == c
        xc = xv[:, m]
        out[c, :, 0] = float(m.sum())
        out[c, :, 1] = xc.sum(1)
        out[c, :, 2] = (xc * xc).sum(1)
    return out
