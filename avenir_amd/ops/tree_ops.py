"""Tree kernels (K7/K8): GPU -> HIP (``tree.hip``); CPU -> PyTorch reference of the same op."""
from __future__ import annotations

from typing import Sequence

import torch

from .. import _native
from .histogram import _dev_i32

# fixed-point scale of the GBT gradient histograms: 2^-16 per row (node_grad_hist_kernel packs the
# g and h sums of a block into one 64-bit LDS word)
_GRAD_SCALE = float(1 << 16)


def _offs(bins: Sequence[int]) -> list[int]:
    o, out = 0, []
    for b in bins:
        out.append(o)
        o += int(b)
    return out


def node_histogram(codes: torch.Tensor, n: int, labels: torch.Tensor, node: torch.Tensor,
                   weight: torch.Tensor | None, bins: Sequence[int], n_classes: int,
                   n_nodes: int, node_rows: torch.Tensor | None = None) -> torch.Tensor:
    """Class counts per (frontier node, class, fine bin): int64 ``[A, C, TB]``.  ``node_rows``
    (int64 ``[A, 2]``, optional): a [lo, hi) row range holding every row of each node (a forest's
    trees are contiguous row blocks), so the kernel scans only those rows per node chunk."""
    bins = [int(b) for b in bins]
    tb = sum(bins)
    out = torch.zeros((n_nodes, n_classes, tb), dtype=torch.int64, device=codes.device)
    if n == 0 or n_nodes == 0:
        return out
    if codes.is_cuda:
        _native.C().node_histogram(codes, int(n), labels, node, weight, _dev_i32(bins, codes.device),
                                   _dev_i32(_offs(bins), codes.device), tb, int(n_classes),
                                   int(n_nodes), out,
                                   None if node_rows is None else node_rows.to(codes.device, torch.long).contiguous())
        return out
    nd = node[:n].long()
    lab = labels[:n].long()
    w = weight[:n].long() if weight is not None else torch.ones(n, dtype=torch.long)
    ok_r = (nd >= 0) & (nd < n_nodes) & (lab < n_classes) & (w > 0)
    for f, (b, o) in enumerate(zip(bins, _offs(bins))):
        v = codes[f, :n].long()
        ok = ok_r & (v < b)
        idx = (nd[ok] * n_classes + lab[ok]) * tb + o + v[ok]
        out.view(-1).index_add_(0, idx, w[ok])
    return out


def node_grad_histogram(codes: torch.Tensor, n: int, node: torch.Tensor, g: torch.Tensor,
                        h: torch.Tensor, bins: Sequence[int], n_nodes: int, even_only: bool = False,
                        bins_d: torch.Tensor | None = None, offs_d: torch.Tensor | None = None,
                        raw: bool = False, tot_slot: int = -1) -> torch.Tensor:
    """Exact fixed-point (2^-16 per row) sums of gradient and hessian per (node, bin): float64
    [A, TB, 2] (int64 raw sums with ``raw``).  ``even_only``: only rows of even node ids, counted at
    id / 2 (the left children of a level, for sibling subtraction).  ``tot_slot``: rows whose
    feature-0 code is missing are counted in that bin (feature 0 + it = the node total).
    ``bins_d`` / ``offs_d``: cached device copies of the bin tables."""
    bins = [int(b) for b in bins]
    tb = sum(bins)
    if codes.is_cuda:
        out = torch.zeros((n_nodes, tb, 2), dtype=torch.int64, device=codes.device)
        if n and n_nodes:
            _native.C().node_grad_histogram(codes, int(n), node, g.float().contiguous(),
                                            h.float().contiguous(),
                                            bins_d if bins_d is not None else _dev_i32(bins, codes.device),
                                            offs_d if offs_d is not None else _dev_i32(_offs(bins), codes.device),
                                            tb, int(n_nodes), out, bool(even_only), int(tot_slot), _GRAD_SCALE)
        return out if raw else out.double() / _GRAD_SCALE
    out = torch.zeros((n_nodes, tb, 2), dtype=torch.int64)
    nd = node[:n].long()
    if even_only:
        nd = torch.where((nd >= 0) & (nd % 2 == 0), nd // 2, torch.full_like(nd, -1))
    gi = torch.round(g[:n].float() * _GRAD_SCALE).long()
    hi = torch.round(h[:n].float() * _GRAD_SCALE).long()
    ok_r = (nd >= 0) & (nd < n_nodes)
    flat = out.view(-1)
    for f, (b, o) in enumerate(zip(bins[: codes.shape[0]], _offs(bins))):
        v = codes[f, :n].long()
        ok = ok_r & (v < b)
        base = (nd[ok] * tb + o + v[ok]) * 2
        flat.index_add_(0, base, gi[ok])
        flat.index_add_(0, base + 1, hi[ok])
        if f == 0 and tot_slot >= 0:
            miss = ok_r & (v >= b)
            base = (nd[miss] * tb + tot_slot) * 2
            flat.index_add_(0, base, gi[miss])
            flat.index_add_(0, base + 1, hi[miss])
    return out if raw else out.double() / _GRAD_SCALE


def gbt_split(hist, parent, left, out_hist, A: int, tot: int, scan: dict, l2: float, level: int,
              feat, thr, val) -> None:
    """One GBT level's split scoring on the device (gbt.hip gbt_split_kernel): raw int64 fixed-point
    histograms in (``hist`` [A, TB, 2], or ``parent`` / ``left`` [A/2, TB, 2] for sibling
    subtraction), heap feat / thr / val out; ``out_hist`` receives the level's histogram.  The
    host twin is the tensor scan in models/tree.py GradientBoostedTrees._build_tree."""
    _native.C().gbt_split(hist, parent, left, out_hist, int(A), int(tot), scan["feat_i"], scan["thr_i"],
                          scan["start_i"], scan["end_i"], scan["valid_u8"], float(l2), _GRAD_SCALE, int(level),
                          feat, thr, val)


def gbt_grad(F: torch.Tensor, k: int, y: torch.Tensor, n: int, row_off: int, seed: int, rate32: int,
             g: torch.Tensor, h: torch.Tensor, loss: torch.Tensor | None = None) -> None:
    """In place: g, h = gradient / hessian of the deviance loss for class ``k`` (sigmoid when
    ``F`` has one column, softmax otherwise) at the raw scores ``F`` [>= n, K]; rows outside the
    counter-hash subsample (``rate32`` / 2^32, keyed by ``seed`` and the GLOBAL row) get 0;
    ``loss`` (when given) += the summed loss of the current scores (gbt.hip)."""
    if F.is_cuda:
        _native.C().gbt_grad(F, int(k), y, int(n), int(row_off), int(seed) & 0x7FFFFFFFFFFFFFFF, int(rate32), g, h,
                             loss)
        return
    K = F.shape[1]
    f = F[:n].double()
    yl = y[:n].long()
    if K == 1:
        p = torch.sigmoid(f[:, 0])
        target = yl.double()
        lv = f[:, 0].clamp_min(0) - f[:, 0] * target + torch.log1p(torch.exp(-f[:, 0].abs()))
    else:
        lse = torch.logsumexp(f, 1)
        p = torch.exp(f[:, k] - lse)
        target = (yl == k).double()
        lv = lse - f.gather(1, yl.clamp_max(K - 1).view(-1, 1))[:, 0]
    gr = (p - target).float()
    hr = (p * (1 - p)).float().clamp_min(1e-6)
    if rate32 != 0xFFFFFFFF:
        rows = torch.arange(row_off, row_off + n, dtype=torch.int64)
        u = _mix32((int(seed) & 0xFFFFFFFFFFFFFFFF), rows)
        keep = u < rate32
        gr, hr = torch.where(keep, gr, torch.zeros_like(gr)), torch.where(keep, hr, torch.zeros_like(hr))
    g[:n], h[:n] = gr, hr
    if loss is not None:
        loss += lv.sum()


def _mix32(seed: int, rows: torch.Tensor) -> torch.Tensor:
    """splitmix64 finaliser of seed + row * golden, high 32 bits (gbt.hip mix32), via numpy uint64."""
    import numpy as np
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + rows.numpy().astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return torch.from_numpy((z >> np.uint64(32)).astype(np.int64))


def gbt_assign(codes: torch.Tensor, n: int, node: torch.Tensor, feat: torch.Tensor, thr: torch.Tensor,
               value: torch.Tensor, bins_t: torch.Tensor, level: int, last: bool, lr: float, F: torch.Tensor,
               k: int) -> None:
    """In place: rows of slot s at ``level`` (heap index 2^level - 1 + s) move to child 2s / 2s+1
    by ``code <= thr``; rows reaching a leaf (no split, missing code, or the last level) add
    ``lr * value[leaf]`` to ``F[:, k]`` and leave (node = -1)."""
    if codes.is_cuda:
        _native.C().gbt_assign(codes, int(n), node, feat, thr, value, bins_t, int(level), bool(last), float(lr), F,
                               int(k))
        return
    hb, hc = (1 << level) - 1, (2 << level) - 1
    s = node[:n].long()
    act = s >= 0
    i = (hb + s).clamp_min(0)
    f = feat.long()[i]
    fc = f.clamp_min(0)
    c = codes[fc, torch.arange(n)].long()
    has = act & (f >= 0) & (c < bins_t.long()[fc])
    child = 2 * s + (c > thr.long()[i]).long()
    leaf_val = torch.where(has & last, value[(hc + child).clamp_min(0).clamp_max(value.numel() - 1)], value[i])
    finish = act & (~has | last)
    F[:n, k] += torch.where(finish, (lr * leaf_val.float()), torch.zeros_like(F[:n, k]))
    node[:n] = torch.where(act & has & (not last), child, torch.full_like(s, -1)).to(node.dtype)


def tree_assign(codes: torch.Tensor, n: int, node: torch.Tensor, split_feat: torch.Tensor,
                segmap: torch.Tensor, child_of: torch.Tensor) -> None:
    """In place: node[r] <- child_of[a, segmap[a, codes[split_feat[a], r]]] (or -1)."""
    if n == 0:
        return
    if codes.is_cuda:
        _native.C().tree_assign(codes, int(n), node, split_feat.int().contiguous(),
                                segmap.to(torch.int16).contiguous(), child_of.int().contiguous())
        return
    nd = node[:n].long()
    act = nd >= 0
    a = nd.clamp_min(0)
    f = split_feat.long()[a]
    expand = act & (f >= 0)
    fc = f.clamp_min(0)
    v = codes[fc, torch.arange(n)].long()
    mb = segmap.shape[1]
    vok = v < mb
    seg = torch.where(vok, segmap.long()[a, v.clamp_max(mb - 1)], torch.full_like(v, -1))
    nxt = torch.where(seg >= 0, child_of.long()[a, seg.clamp_min(0)], torch.full_like(v, -1))
    node[:n] = torch.where(expand, nxt, torch.full_like(v, -1)).to(node.dtype)


def tree_predict(codes: torch.Tensor, n: int, forest: dict, mode: int = 0) -> torch.Tensor:
    """Forest inference.  ``forest`` holds int32/int16/float32 device arrays (see
    ``models.tree.flatten_forest``).  Returns float32 ``[n, V]``."""
    V = int(forest["values"].shape[1])
    out = torch.zeros((max(n, 1), V), dtype=torch.float32, device=codes.device)
    if n == 0:
        return out[:0]
    if codes.is_cuda and "bin_nodes" in forest and V <= 8 and codes.shape[0] <= 255 and \
            forest["bin_nodes"].shape[0] * 8 + 256 * codes.shape[0] <= 160 * 1024:
        # threshold-split forests: node table of all trees in LDS, register accumulation
        _native.C().forest_predict_bin(codes, int(n), forest["bin_nodes"], forest["values"], forest["tree_root"],
                                       forest.get("tree_w"), int(mode), out)
        return out[:n]
    if codes.is_cuda:
        _native.C().tree_predict(codes, int(n), forest["feat"], forest["seg_base"], forest["segmap"],
                                 forest["child_base"], forest["child"], forest["leaf_idx"],
                                 forest["values"], forest["tree_root"], forest.get("tree_w"), int(mode),
                                 out)
        return out[:n]
    feat = forest["feat"].tolist()
    seg_base = forest["seg_base"].tolist()
    child_base = forest["child_base"].tolist()
    child = forest["child"].tolist()
    leaf_idx = forest["leaf_idx"].tolist()
    segmap = forest["segmap"]
    values = forest["values"]
    tw = forest.get("tree_w")
    mb = segmap.shape[1]
    # vectorised level-synchronous traversal (all rows at once)
    for t, root in enumerate(forest["tree_root"].tolist()):
        k = torch.full((n,), root, dtype=torch.long)
        for _ in range(4096):
            fk = torch.tensor(feat, dtype=torch.long)[k]
            live = fk >= 0
            if not bool(live.any()):
                break
            v = codes[fk.clamp_min(0), torch.arange(n)].long()
            sb = torch.tensor(seg_base, dtype=torch.long)[k]
            seg = torch.where(v < mb, segmap.long()[sb.clamp_min(0), v.clamp_max(mb - 1)],
                              torch.full_like(v, -1))
            cb = torch.tensor(child_base, dtype=torch.long)[k]
            ct = torch.tensor(child + [-1], dtype=torch.long)
            nk = torch.where(seg >= 0, ct[(cb + seg).clamp(0, len(child))], torch.full_like(v, -1))
            move = live & (seg >= 0) & (nk >= 0)
            if not bool(move.any()):
                break
            k = torch.where(move, nk, k)
        val = values[torch.tensor(leaf_idx, dtype=torch.long)[k]]
        w = float(tw[t]) if tw is not None else 1.0
        if mode == 0:
            out[:n] += w * val
        else:
            out[torch.arange(n), val.argmax(1)] += w
    return out[:n]
