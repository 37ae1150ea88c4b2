"""Forest-builder ops (forest.hip): chunk histograms, K6/K7 split scoring, stable partitioning.

GPU tensors go to the HIP kernels; CPU tensors run the PyTorch oracle of the same op (identical
semantics, used by the CPU tests and as the numerics reference of the GPU tests).  Work lists
(``node``/``slot`` int32, ``start`` int64, ``len`` int32, bases int64) are always HOST tensors: the
binding bound-checks them on the CPU before anything is launched.
"""
from __future__ import annotations

import math

import torch

from .. import _native


def _i32(x):
    return torch.as_tensor(x, dtype=torch.int32)


def _i64(x):
    return torch.as_tensor(x, dtype=torch.int64)


def forest_hist(codes, lab, wt, slot, start, length, bins_d, offs_d, bins, TB: int, C: int, hist) -> None:
    """hist[slot[i]][c][b] += w over the rows [start[i], start[i] + len[i]) (in place)."""
    slot, start, length = _i32(slot), _i64(start), _i32(length)
    if codes.is_cuda:
        _native.C().forest_hist(codes, lab, wt, slot, start, length, bins_d, offs_d, int(TB), int(C), hist)
        return
    offs = [0]
    for b in bins[:-1]:
        offs.append(offs[-1] + b)
    flat = hist.view(-1)
    for s, a, n in zip(slot.tolist(), start.tolist(), length.tolist()):
        if n <= 0:
            continue
        c = lab[a:a + n].long()
        w = wt[a:a + n].long()
        ok = (c < C) & (w > 0)
        base = (s * C + c) * TB
        for f, (B, o) in enumerate(zip(bins, offs)):
            v = codes[f, a:a + n].long()
            m = ok & (v < B)
            flat.index_add_(0, base[m] + o + v[m], w[m])
        flat.index_add_(0, base[ok] + TB - 1, w[ok])


def _impurity(cnt: torch.Tensor, tot: torch.Tensor, algo: int) -> torch.Tensor:
    p = cnt / tot.clamp_min(1e-300).unsqueeze(-1)
    if algo == 0:
        v = 1.0 - (p * p).sum(-1)
    else:
        v = -(torch.where(p > 0, p * torch.log2(p.clamp_min(1e-300)), torch.zeros_like(p))).sum(-1)
    return torch.where(tot > 0, v, torch.zeros_like(v))


def forest_split(hist, fmask, bins_d, offs_d, bins, algo: int, topk: int, rnd):
    """Per node: (feature, threshold, weighted child impurity, node impurity, left class counts)."""
    if hist.is_cuda:
        return _native.C().forest_split(hist, fmask, bins_d, offs_d, int(algo), int(topk), rnd)
    A, C, TB = hist.shape
    F = len(bins)
    h = hist.double()
    tot = h[:, :, TB - 1]                                              # [A, C]
    ntot = tot.sum(1)
    best = torch.full((A, F), math.inf, dtype=torch.float64)
    bthr = torch.full((A, F), -1, dtype=torch.int64)
    o = 0
    for f, B in enumerate(bins):
        if B >= 2:
            cs = torch.cumsum(h[:, :, o:o + B - 1], 2).transpose(1, 2)   # [A, B-1, C] left counts
            nl = cs.sum(-1)
            nr = ntot.unsqueeze(1) - nl
            right = tot.unsqueeze(1) - cs
            s = (nl * _impurity(cs, nl, algo) + nr * _impurity(right, nr, algo)) / ntot.clamp_min(1e-300).unsqueeze(1)
            s = torch.where((nl > 0) & (nr > 0), s, torch.full_like(s, math.inf))
            v, i = s.min(1)                                             # first minimum
            ok = fmask[:, f].bool()
            best[:, f] = torch.where(ok, v, torch.full_like(v, math.inf))
            bthr[:, f] = torch.where(ok & torch.isfinite(v), i, torch.full_like(i, -1))
        o += B
    feat = torch.full((A,), -1, dtype=torch.int32)
    thr = torch.full((A,), -1, dtype=torch.int32)
    score = torch.full((A,), math.inf, dtype=torch.float32)
    left = torch.zeros((A, C), dtype=torch.int64)
    offs = [0]
    for b in bins[:-1]:
        offs.append(offs[-1] + b)
    for a in range(A):
        row = best[a]
        if topk <= 1:
            v, f = row.min(0)
            pick = int(f) if math.isfinite(float(v)) else -1
        else:
            order = sorted([f for f in range(F) if math.isfinite(float(row[f]))], key=lambda f: (float(row[f]), f))
            chosen = order[: min(topk, 32)]
            pick = chosen[min(int(float(rnd[a]) * len(chosen)), len(chosen) - 1)] if chosen else -1
        if pick >= 0:
            t = int(bthr[a, pick])
            feat[a], thr[a], score[a] = pick, t, float(row[pick])
            left[a] = hist[a, :, offs[pick]: offs[pick] + t + 1].sum(1)
    imp = _impurity(tot, ntot, algo).float()
    return feat, thr, score, imp, left


def forest_part_count(codes, node, start, length, feat, thr) -> torch.Tensor:
    node, start, length = _i32(node), _i64(start), _i32(length)
    if codes.is_cuda:
        return _native.C().forest_part_count(codes, node, start, length, feat.int().contiguous(), thr.int().contiguous())
    out = torch.zeros(node.numel(), dtype=torch.int32)
    for i, (a, s, n) in enumerate(zip(node.tolist(), start.tolist(), length.tolist())):
        f = int(feat[a])
        if f >= 0 and n > 0:
            out[i] = int((codes[f, s:s + n].long() <= int(thr[a])).sum())
    return out


def forest_part_scatter(codes, lab, wt, dcodes, dlab, dwt, node, start, length, left_base, right_base, item_left,
                        feat, thr):
    """Stable partition; ``item_left`` = forest_part_count's per-chunk left counts (host), which
    the binding uses to bound-check every destination range."""
    node, start, length = _i32(node), _i64(start), _i32(length)
    left_base, right_base, item_left = _i64(left_base), _i64(right_base), _i32(torch.as_tensor(item_left).cpu())
    if codes.is_cuda:
        _native.C().forest_part_scatter(codes, lab, wt, dcodes, dlab, dwt, node, start, length, left_base, right_base,
                                        item_left, feat.int().contiguous(), thr.int().contiguous())
        return
    for a, s, n, lb, rb in zip(node.tolist(), start.tolist(), length.tolist(), left_base.tolist(), right_base.tolist()):
        f = int(feat[a])
        if f < 0 or n <= 0:
            continue
        r = torch.arange(s, s + n)
        go = codes[f, s:s + n].long() <= int(thr[a])
        li, ri = r[go], r[~go]
        dl = torch.arange(lb, lb + li.numel())
        dr = torch.arange(rb, rb + ri.numel())
        dcodes[:, dl] = codes[:, li]
        dcodes[:, dr] = codes[:, ri]
        dlab[dl], dlab[dr] = lab[li], lab[ri]
        dwt[dl], dwt[dr] = wt[li], wt[ri]
