"""Split statistics for all candidate splits of all attributes in one pass.

Reference:
* ``AttributeSplitStat`` (J/util/AttributeSplitStat.java:40-474): per (split, segment, class) counts
  -> ``entropy`` / ``giniIndex`` (segment-size weighted impurity), ``hellingerDistance`` (binary
  class: sqrt(sum_seg (sqrt(n0/N0) - sqrt(n1/N1))^2)), ``classConfidenceRatio`` (per segment the
  class confidences n_c/N_c normalised to ratios, their entropy, size weighted), and the split
  info content used for gain ratio (:150-170).
* ``InfoContentStat`` (J/util/InfoContentStat.java:71-101): entropy / gini of a class distribution.
* ``ClassPartitionGenerator`` (MR, J/explore/ClassPartitionGenerator.java): emits, for every
  candidate split of every attribute, the class distribution per segment and its score.
* ``AttributeSplitHandler`` (J/util/AttributeSplitHandler.java:43-220): split keys — numeric split
  points joined by ``:``, categorical groups ``[a, b]`` joined by ``:``.

MI355X design: ONE K2 class-histogram launch over the fine-bin codes of every attribute gives a
[C, total_fine_bins] table; every candidate split is a fine-bin -> segment map, so the
[splits, segments, classes] count tensor of ALL splits is a batched gather/segment-sum of that
table, and all statistics are vectorised over splits.
"""
from __future__ import annotations

import math
from typing import Sequence

import torch

from ..data.table import Table
from ..ops import histogram as H
from . import tree as T


def split_stat(counts: torch.Tensor, algorithm: str = "entropy") -> torch.Tensor:
    """counts [..., G, C] (segments x classes) -> stat [...] for each split."""
    c = counts.double()
    seg_tot = c.sum(-1)                                    # [..., G]
    tot = seg_tot.sum(-1).clamp_min(1)                     # [...]
    if algorithm in ("entropy", "giniIndex", "gini"):
        imp = T.impurity(c, "entropy" if algorithm == "entropy" else "giniIndex")   # [..., G]
        return (imp * seg_tot).sum(-1) / tot
    cls_tot = c.sum(-2, keepdim=True).clamp_min(1)         # [..., 1, C]
    conf = c / cls_tot                                     # class confidence per segment
    if algorithm == "hellingerDistance":
        if c.shape[-1] != 2:
            raise ValueError("Hellinger distance algorithm is only valid for binary valued class attributes")
        d = conf[..., 0].sqrt() - conf[..., 1].sqrt()
        return (d * d).sum(-1).sqrt()
    if algorithm == "classConfidenceRatio":
        ratio = conf / conf.sum(-1, keepdim=True).clamp_min(1e-300)
        ent = -(torch.where(ratio > 0, ratio * torch.log2(ratio.clamp_min(1e-300)), torch.zeros_like(ratio))).sum(-1)
        return (ent * seg_tot).sum(-1) / tot
    raise ValueError(f"unknown split algorithm {algorithm}")


def split_info(counts: torch.Tensor) -> torch.Tensor:
    """Entropy of the segment sizes (gain-ratio denominator)."""
    s = counts.double().sum(-1)
    p = s / s.sum(-1, keepdim=True).clamp_min(1)
    return -(torch.where(p > 0, p * torch.log2(p.clamp_min(1e-300)), torch.zeros_like(p))).sum(-1)


def info_content(class_counts: torch.Tensor, algorithm: str = "entropy") -> torch.Tensor:
    return T.impurity(class_counts, algorithm)


def split_key(fs: T.FeatureSplits, sp: T.Split) -> str:
    """AttributeSplitHandler key: numeric split points or categorical groups joined by ':'."""
    if fs.kind == "num":
        pts = []
        for b in range(1, len(sp.segmap)):
            if sp.segmap[b] != sp.segmap[b - 1]:
                pts.append(fs.pred_value(fs.points[b - 1]))
        return ":".join(pts)
    groups: dict[int, list[str]] = {}
    for b, g in enumerate(sp.segmap):
        groups.setdefault(g, []).append(fs.field.cardinality[b])
    return ":".join("[" + ", ".join(groups[g]) + "]" for g in sorted(groups))


def parse_split_key(key: str, kind: str):
    if kind == "num":
        return [float(v) for v in key.split(":") if v]
    return [[x.strip() for x in g.strip("[]").split(",")] for g in key.split(":")]


def class_partition_stats(t: Table, algorithm: str = "entropy", attrs: Sequence[int] | None = None,
                          max_bins: int = 32, comm=None) -> list[dict]:
    """Score every candidate split of every attribute (ClassPartitionGenerator).

    Returns dicts {attr, key, stat, gain, gain_ratio, counts [G, C]} sorted by attribute then
    stat; ``gain`` = parent impurity - split impurity for entropy / gini (for Hellinger the stat
    itself is the quality)."""
    space = T.build_split_space(t.schema, t, attrs)
    codes = T.encode_for_tree(space, t)
    bins = [fs.n_bins for fs in space]
    C = t.n_classes
    hist = H.class_histogram(codes, t.n, bins, t.labels, C, count_labels=True)          # [C, TB + 1]
    if comm is not None and comm.is_distributed:
        comm.all_reduce(hist)
    hist = hist.cpu()
    parent_counts = hist[:, -1].double()
    parent = float(info_content(parent_counts, "entropy" if algorithm == "entropy" else "giniIndex")) \
        if algorithm in ("entropy", "giniIndex", "gini") else 0.0
    out = []
    o = 0
    for fs, b in zip(space, bins):
        fine = hist[:, o:o + b].T.double()                 # [B, C]
        o += b
        if not fs.splits:
            continue
        G = max(sp.n_seg for sp in fs.splits)
        M = torch.zeros((len(fs.splits), G, b), dtype=torch.float64)
        for i, sp in enumerate(fs.splits):
            M[i, torch.tensor(sp.segmap), torch.arange(b)] = 1.0
        cnt = M @ fine                                      # [S, G, C] for all splits at once
        st = split_stat(cnt, algorithm)
        si = split_info(cnt)
        for i, sp in enumerate(fs.splits):
            g = cnt[i, : sp.n_seg]
            gain = parent - float(st[i]) if algorithm in ("entropy", "giniIndex", "gini") else float(st[i])
            out.append({"attr": fs.field.ordinal, "key": split_key(fs, sp), "stat": float(st[i]), "gain": gain,
                        "gain_ratio": gain / float(si[i]) if float(si[i]) > 0 else 0.0, "counts": g})
    return out


def partition_lines(stats: list[dict], delim: str = ",") -> list[str]:
    """attr, splitKey, stat lines (the MR reducer output layout)."""
    return [f"{s['attr']}{delim}{s['key']}{delim}{s['stat']:.6f}" for s in stats]
