"""Isolation forest outlier detection, grown and scored as batched tensors on the device.

The reference calls scikit-learn's ``IsolationForest`` from ``DataExplorer.getOutliersWithIsoForest``
(P/mlextra/daexp.py:921-941).  The algorithm (Liu, Ting & Zhou 2008) is the same here:

* every tree sees ``psi`` rows drawn without replacement (``psi = min(256, n)`` by default);
* each node picks a random non-constant feature and a threshold uniform in that feature's
  [min, max] over the node's rows, down to depth ``ceil(log2 psi)``;
* a point's path length is its depth at the leaf plus ``c(leaf size)``, the expected depth of an
  unsuccessful BST search over that many points;
* the anomaly score is ``2 ** (-mean path length / c(psi))``.

The difference is in how it runs.  All trees grow level-synchronously: one segmented min/max
(``scatter_reduce``) per level covers every node of every tree.  Scoring walks all trees at once
over chunks of points.  The number of launches therefore grows with the depth (about 8), not
with trees x nodes.

``contamination="auto"`` puts the offset at -0.5, as scikit-learn does; a number sets it at that
percentile of the training scores.  The random draws differ from scikit-learn's, so the parity
is statistical (outlier sets overlap on planted-outlier data; see tests/test_outlier.py).
"""
from __future__ import annotations

import math

import numpy as np
import torch

_EULER = 0.5772156649015329


def avg_path_length(n: torch.Tensor) -> torch.Tensor:
    """c(n): expected depth of an unsuccessful search in a BST over n points (c(1)=0, c(2)=1)."""
    n = n.to(torch.float64)
    h = torch.log((n - 1).clamp_min(1)) + _EULER
    c = 2.0 * h - 2.0 * (n - 1) / n.clamp_min(1)
    return torch.where(n > 2, c, torch.where(n == 2, torch.ones_like(n), torch.zeros_like(n)))


class IsolationForest:
    def __init__(self, n_estimators: int = 100, max_samples: int | str = "auto",
                 contamination: float | str = "auto", seed: int = 0, chunk: int = 1 << 16):
        self.n_estimators = int(n_estimators)
        self.max_samples = max_samples
        self.contamination = contamination
        self.seed = int(seed)
        self.chunk = int(chunk)

    def fit(self, X) -> "IsolationForest":
        X = torch.as_tensor(X).float()
        if X.dim() == 1:
            X = X.unsqueeze(1)
        n, d = X.shape
        dev = X.device
        psi = min(256, n) if self.max_samples == "auto" else min(int(self.max_samples), n)
        psi = max(psi, 1)
        self.psi = psi
        L = max(1, math.ceil(math.log2(max(psi, 2))))
        self.depth = L
        T = self.n_estimators
        g = torch.Generator(device=dev)
        g.manual_seed(self.seed)
        if n <= (1 << 20):
            idx = torch.rand((T, n), generator=g, device=dev).argsort(1)[:, :psi]
        else:   # large n: per-tree randperm prefixes (still without replacement)
            idx = torch.stack([torch.randperm(n, generator=g, device=dev)[:psi] for _ in range(T)])
        S = X[idx]                                     # [T, psi, d]
        M = (1 << (L + 1)) - 1                         # nodes per tree (complete binary tree)
        feat = torch.full((T, M), -1, dtype=torch.long, device=dev)
        thr = torch.zeros((T, M), dtype=torch.float32, device=dev)
        size = torch.zeros((T, M), dtype=torch.long, device=dev)
        node = torch.zeros((T, psi), dtype=torch.long, device=dev)
        tree = torch.arange(T, device=dev).view(T, 1).expand(T, psi)
        for lev in range(L + 1):
            base, width = (1 << lev) - 1, 1 << lev
            alive = node >= base                       # rows whose node is on this level
            flat = torch.where(alive, tree * width + (node - base), T * width)   # dump slot
            cnt = torch.bincount(flat.view(-1), minlength=T * width + 1)[: T * width]
            size[:, base:base + width] = cnt.view(T, width)
            if lev == L:
                break
            fl = flat.view(-1, 1).expand(-1, d)
            src = S.view(-1, d)
            mn = torch.full((T * width + 1, d), float("inf"), device=dev).scatter_reduce(
                0, fl, src, "amin", include_self=True)[: T * width]
            mx = torch.full((T * width + 1, d), float("-inf"), device=dev).scatter_reduce(
                0, fl, src, "amax", include_self=True)[: T * width]
            varies = mx > mn
            split = (cnt > 1) & varies.any(1)
            r = torch.rand((T * width, d), generator=g, device=dev).masked_fill(~varies, -1.0)
            f = r.argmax(1)
            lo = mn.gather(1, f.view(-1, 1)).squeeze(1)
            hi = mx.gather(1, f.view(-1, 1)).squeeze(1)
            u = torch.rand((T * width,), generator=g, device=dev)
            t = torch.where(split, lo + u * (hi - lo), torch.zeros_like(lo))
            feat[:, base:base + width] = torch.where(split, f, -1).view(T, width)
            thr[:, base:base + width] = t.view(T, width)
            # route this level's rows of split nodes to a child
            fsel = torch.where(alive, feat.gather(1, node), -1)
            xv = S.gather(2, fsel.clamp_min(0).unsqueeze(2)).squeeze(2)
            go = fsel >= 0
            child = 2 * node + 1 + (xv > thr.gather(1, node)).long()
            node = torch.where(go, child, node)
        self.feat, self.thr = feat, thr
        self.leaf_c = avg_path_length(size).float()    # c(size) of every node, used at leaves
        self.c_psi = float(avg_path_length(torch.tensor(float(psi))))
        train = self.score_samples(X)
        if self.contamination == "auto":
            self.offset_ = -0.5
        else:
            c = float(self.contamination)
            if not 0.0 < c <= 0.5:
                raise ValueError("contamination must be in (0, 0.5]")
            self.offset_ = float(np.percentile(train.double().cpu().numpy(), 100.0 * c))
        return self

    def path_length(self, X) -> torch.Tensor:
        """Mean isolation depth over the trees (with the leaf-size correction), [n]."""
        X = torch.as_tensor(X).float().to(self.feat.device)
        if X.dim() == 1:
            X = X.unsqueeze(1)
        T = self.feat.shape[0]
        out = []
        for s in range(0, X.shape[0], self.chunk):
            xc = X[s:s + self.chunk]
            c = xc.shape[0]
            xt = xc.t().contiguous()                    # [d, c]
            node = torch.zeros((T, c), dtype=torch.long, device=X.device)
            depth = torch.zeros((T, c), dtype=torch.float32, device=X.device)
            col = torch.arange(c, device=X.device).view(1, c).expand(T, c)
            for _ in range(self.depth):
                f = self.feat.gather(1, node)
                inner = f >= 0
                xv = xt[f.clamp_min(0), col]
                node = torch.where(inner, 2 * node + 1 + (xv > self.thr.gather(1, node)).long(), node)
                depth += inner
            out.append((depth + self.leaf_c.gather(1, node)).mean(0))
        return torch.cat(out) if out else torch.zeros(0, device=X.device)

    def score_samples(self, X) -> torch.Tensor:
        """Negated anomaly score (scikit-learn's convention: lower = more abnormal)."""
        return -torch.pow(2.0, -self.path_length(X) / max(self.c_psi, 1e-12))

    def decision_function(self, X) -> torch.Tensor:
        return self.score_samples(X) - self.offset_

    def predict(self, X) -> torch.Tensor:
        return torch.where(self.decision_function(X) < 0, -1, 1)

    def fit_predict(self, X) -> torch.Tensor:
        return self.fit(X).predict(X)
