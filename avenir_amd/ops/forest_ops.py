"""Forest-builder ops (forest.hip): chunk histograms, K6/K7 split scoring, stable partitioning.

GPU tensors go to the HIP kernels; CPU tensors run the PyTorch oracle of the same op (identical
semantics, used by the CPU tests and as the numerics reference of the GPU tests).  Work lists
(``node``/``slot`` int32, ``start`` int64, ``len`` int32, bases int64) are always HOST tensors: the
binding bound-checks them on the CPU before anything is launched.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .. import _native


def _i32(x):
    return torch.as_tensor(x, dtype=torch.int32)


def _i64(x):
    return torch.as_tensor(x, dtype=torch.int64)


POISSON1_CDF = np.array([1580030168, 3160060337, 3950075421, 4213413783, 4279248373, 4292415291, 4294609777,
                         4294923276, 4294962463, 4294966817, 4294967252, 4294967292], dtype=np.uint64)
BOOT_MODES = {"none": 0, "withReplace": 1, "withoutReplace": 2}


def boot_weights(key: int, rows: np.ndarray, mode: int, rate32: int) -> np.ndarray:
    """Bootstrap multiplicity of each global row for one tree key (the kernel's ``boot_weight``):
    splitmix64(key + row * golden) -> high 32 bits u -> Poisson(1) by inverse CDF (mode 1),
    u < rate32 (mode 2) or 1 (mode 0).  uint8."""
    if mode == 0:
        return np.ones(rows.shape, np.uint8)
    with np.errstate(over="ignore"):
        z = np.uint64(key & 0xFFFFFFFFFFFFFFFF) + rows.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    u = z >> np.uint64(32)
    if mode == 2:
        return (u < np.uint64(rate32)).astype(np.uint8)
    return (u[:, None] >= POISSON1_CDF[None, :]).sum(1).astype(np.uint8)


def forest_bootstrap(codes, lab, n: int, keys, row_off: int, mode: int, rate32: int):
    """Per-tree bootstrap row buffers: the kept rows (multiplicity > 0) of every tree, tree-major,
    compacted into (codes [F, ldb], labels [ldb], weights [ldb]) plus the host int64 row count
    per tree.  ``keys`` int64 [T] (one per tree); rows are keyed by ``row_off + r`` (global)."""
    keys = torch.as_tensor(keys, dtype=torch.int64)
    if codes.is_cuda:
        cb, lb, wb, per = _native.C().forest_bootstrap(codes.contiguous(), lab.contiguous(), int(n),
                                                       keys.to(codes.device), int(row_off), int(mode), int(rate32))
        return cb, lb, wb, per
    rows = np.arange(row_off, row_off + n, dtype=np.int64)
    ws = [boot_weights(int(k), rows, mode, rate32) for k in keys.tolist()]
    idx = [np.nonzero(w)[0] for w in ws]
    R = int(sum(i.size for i in idx))
    ldb = max(16, (R + 15) // 16 * 16)
    F = codes.shape[0]
    cb = torch.empty((F, ldb), dtype=torch.uint8)
    lb = torch.empty(ldb, dtype=torch.uint8)
    wb = torch.zeros(ldb, dtype=torch.uint8)
    sel = torch.from_numpy(np.concatenate(idx) if idx else np.zeros(0, np.int64))
    cb[:, :R] = codes[:, :n].index_select(1, sel)
    lb[:R] = lab[:n].index_select(0, sel)
    wb[:R] = torch.from_numpy(np.concatenate([w[i] for w, i in zip(ws, idx)]) if idx else np.zeros(0, np.uint8))
    return cb, lb, wb, torch.tensor([i.size for i in idx], dtype=torch.int64)


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
    """Per node: (feature, threshold, weighted child impurity, node impurity, left class counts).

    GPU with <= 16 classes: the fused K6/K7 kernel (forest.hip).  Otherwise the batched tensor
    twin below, on the histogram's own device (no per-node host loop, any class count)."""
    if hist.is_cuda and hist.shape[1] <= 16:
        return _native.C().forest_split(hist, fmask, bins_d, offs_d, int(algo), int(topk), rnd)
    return _forest_split_tensor(hist, fmask, bins, algo, topk, rnd)


def _forest_split_tensor(hist, fmask, bins, algo: int, topk: int, rnd):
    A, C, TB = hist.shape
    dev = hist.device
    F = len(bins)
    h = hist.double()
    tot = h[:, :, TB - 1]                                              # [A, C]
    ntot = tot.sum(1)
    best = torch.full((A, F), math.inf, dtype=torch.float64, device=dev)
    bthr = torch.full((A, F), -1, dtype=torch.int64, device=dev)
    offs = [0]
    for b in bins[:-1]:
        offs.append(offs[-1] + b)
    for f, B in enumerate(bins):
        if B >= 2:
            o = offs[f]
            cs = torch.cumsum(h[:, :, o:o + B - 1], 2).transpose(1, 2)   # [A, B-1, C] left counts
            nl = cs.sum(-1)
            nr = ntot.unsqueeze(1) - nl
            right = tot.unsqueeze(1) - cs
            s = (nl * _impurity(cs, nl, algo) + nr * _impurity(right, nr, algo)) / ntot.clamp_min(1e-300).unsqueeze(1)
            s = torch.where((nl > 0) & (nr > 0), s, torch.full_like(s, math.inf))
            v, i = s.min(1)                                             # first minimum
            ok = fmask[:, f].to(dev).bool()
            best[:, f] = torch.where(ok, v, torch.full_like(v, math.inf))
            bthr[:, f] = torch.where(ok & torch.isfinite(v), i, torch.full_like(i, -1))
    fin = torch.isfinite(best)
    if topk <= 1:
        v, pick = best.min(1)                                           # first minimum feature
        has = torch.isfinite(v)
    else:
        # stable sort by (score, feature): the random choice among the top min(topk, 32) features
        order = torch.sort(best, dim=1, stable=True).indices
        kk = torch.clamp(fin.sum(1), max=min(int(topk), 32))
        has = kk > 0
        j = (rnd[:A].to(dev).double() * kk.double()).long()
        j = torch.minimum(j, (kk - 1).clamp_min(0))
        pick = order.gather(1, j.view(-1, 1)).view(-1)
    pick = torch.where(has, pick, torch.zeros_like(pick))
    t = bthr.gather(1, pick.view(-1, 1)).view(-1)
    sc = best.gather(1, pick.view(-1, 1)).view(-1)
    feat = torch.where(has, pick, torch.full_like(pick, -1)).int()
    thr = torch.where(has, t, torch.full_like(t, -1)).int()
    score = torch.where(has, sc, torch.full_like(sc, math.inf)).float()
    # left counts = class histogram of the chosen feature's bins 0..thr (exact int64 prefix sums)
    offs_t = torch.tensor(offs, dtype=torch.int64, device=dev)
    cum = torch.cumsum(hist.long(), 2)                                  # [A, C, TB]
    o = offs_t[pick]
    hi = (o + t.clamp_min(0)).view(-1, 1, 1).expand(A, C, 1)
    lo = (o - 1).clamp_min(0).view(-1, 1, 1).expand(A, C, 1)
    left = cum.gather(2, hi).squeeze(2) - torch.where((o > 0).view(-1, 1), cum.gather(2, lo).squeeze(2), 0)
    left = torch.where(has.view(-1, 1), left, torch.zeros_like(left))
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
