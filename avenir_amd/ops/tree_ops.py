"""Tree kernels (K7/K8): GPU -> HIP (``tree.hip``); CPU -> PyTorch reference of the same op."""
from __future__ import annotations

from typing import Sequence

import torch

from .. import _native
from .histogram import _dev_i32

_GRAD_SCALE = float(1 << 24)


def _offs(bins: Sequence[int]) -> list[int]:
    o, out = 0, []
    for b in bins:
        out.append(o)
        o += int(b)
    return out


def node_histogram(codes: torch.Tensor, n: int, labels: torch.Tensor, node: torch.Tensor,
                   weight: torch.Tensor | None, bins: Sequence[int], n_classes: int,
                   n_nodes: int) -> torch.Tensor:
    """Class counts per (frontier node, class, fine bin): int64 ``[A, C, TB]``."""
    bins = [int(b) for b in bins]
    tb = sum(bins)
    out = torch.zeros((n_nodes, n_classes, tb), dtype=torch.int64, device=codes.device)
    if n == 0 or n_nodes == 0:
        return out
    if codes.is_cuda:
        _native.C().node_histogram(codes, int(n), labels, node, weight, _dev_i32(bins, codes.device),
                                   _dev_i32(_offs(bins), codes.device), tb, int(n_classes),
                                   int(n_nodes), out)
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
                        h: torch.Tensor, bins: Sequence[int], n_nodes: int) -> torch.Tensor:
    """Exact fixed-point (2^-24) sums of gradient and hessian per (node, bin): float64 [A, TB, 2]."""
    bins = [int(b) for b in bins]
    tb = sum(bins)
    if codes.is_cuda:
        out = torch.zeros((n_nodes, tb, 2), dtype=torch.int64, device=codes.device)
        if n and n_nodes:
            _native.C().node_grad_histogram(codes, int(n), node, g.float().contiguous(),
                                            h.float().contiguous(), _dev_i32(bins, codes.device),
                                            _dev_i32(_offs(bins), codes.device), tb, int(n_nodes), out)
        return out.double() / _GRAD_SCALE
    out = torch.zeros((n_nodes, tb, 2), dtype=torch.int64)
    nd = node[:n].long()
    gi = torch.round(g[:n].float() * _GRAD_SCALE).long()
    hi = torch.round(h[:n].float() * _GRAD_SCALE).long()
    ok_r = (nd >= 0) & (nd < n_nodes)
    flat = out.view(-1)
    for f, (b, o) in enumerate(zip(bins, _offs(bins))):
        v = codes[f, :n].long()
        ok = ok_r & (v < b)
        base = (nd[ok] * tb + o + v[ok]) * 2
        flat.index_add_(0, base, gi[ok])
        flat.index_add_(0, base + 1, hi[ok])
    return out.double() / _GRAD_SCALE


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
