"""Vectorised synthetic-data generators (the reference's fixture generators in P/app/*.py).

Reference generators (``loan_approve.py``, ``heart_disease.py``, ``sales_lead.py``, ...) loop per
record in Python: sample each field from a sampler, add per-field scores (lookup tables / step
functions), add feature-coupling terms, and label by comparing the score with a threshold +-
margin (random inside the margin).  ``ScoreModel`` expresses the same recipe declaratively and
generates a whole data set as device tensors in one pass: categorical fields by multinomial
draws, numeric fields by clipped gaussians, scores by table gathers / bucketize, couplings as
masked adds.  ``loan_approval`` mirrors loan_approve.py ``initOne`` (P/app/loan_approve.py:18-139);
``class_conditional`` mirrors the ``initTwo`` style (feature distributions conditioned on class).
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Callable, Sequence

import torch

from ..utils.misc import gen_ids


@dataclass
class CatField:
    name: str
    values: list[str]
    weights: list[float]
    scores: list[float] | None = None          # score per value


@dataclass
class NumField:
    name: str
    mean: float
    sd: float
    lo: float | None = None
    hi: float | None = None
    integer: bool = True
    steps: list[tuple[float, float, float]] | None = None   # (lo, hi, score) step function


@dataclass
class ScoreModel:
    fields: list
    threshold: float
    margin: float = 0.0
    couplings: list[Callable] = field(default_factory=list)   # fn(cols dict) -> score delta tensor

    def generate(self, n: int, seed: int = 0, device="cpu"):
        dev = torch.device(device)
        g = torch.Generator(device=dev).manual_seed(seed)
        cols: dict[str, torch.Tensor] = {}
        score = torch.zeros(n, dtype=torch.float64, device=dev)
        for f in self.fields:
            if isinstance(f, CatField):
                w = torch.tensor(f.weights, dtype=torch.float64, device=dev)
                k = torch.multinomial(w / w.sum(), n, replacement=True, generator=g)
                cols[f.name] = k
                if f.scores is not None:
                    score += torch.tensor(f.scores, dtype=torch.float64, device=dev)[k]
            else:
                v = f.mean + f.sd * torch.randn(n, dtype=torch.float64, device=dev, generator=g)
                if f.integer:
                    v = v.trunc()
                if f.lo is not None or f.hi is not None:
                    v = v.clamp(f.lo if f.lo is not None else -float("inf"), f.hi if f.hi is not None else float("inf"))
                cols[f.name] = v
                if f.steps:
                    s = torch.zeros(n, dtype=torch.float64, device=dev)
                    for lo, hi, sc in f.steps:
                        s = torch.where((v >= lo) & (v < hi), torch.full_like(s, sc), s)
                    score += s
        for c in self.couplings:
            score += c(cols, self)
        hi, lo = self.threshold + self.margin, self.threshold - self.margin
        coin = torch.rand(n, generator=g, device=dev) < 0.5
        label = torch.where(score > hi, 1, torch.where(score < lo, 0, coin.long()))
        return cols, label, score

    def value(self, cols, name):
        f = next(x for x in self.fields if x.name == name)
        if isinstance(f, CatField):
            return cols[name], f.values
        return cols[name], None

    def lines(self, n: int, seed: int = 0, delim: str = ",") -> list[str]:
        cols, label, _ = self.generate(n, seed)
        ids = gen_ids(n, 10, seed)
        parts = []
        for f in self.fields:
            c = cols[f.name].tolist()
            parts.append([f.values[i] for i in c] if isinstance(f, CatField) else
                         [str(int(v)) if f.integer else f"{v:.3f}" for v in c])
        lab = label.tolist()
        return [delim.join([ids[i]] + [p[i] for p in parts] + [str(lab[i])]) for i in range(n)]

    def schema(self, class_name: str = "label") -> dict:
        fields = [{"name": "id", "ordinal": 0, "id": True, "dataType": "string"}]
        for j, f in enumerate(self.fields, start=1):
            if isinstance(f, CatField):
                fields.append({"name": f.name, "ordinal": j, "dataType": "categorical", "feature": True,
                               "cardinality": list(f.values)})
            else:
                fields.append({"name": f.name, "ordinal": j, "dataType": "int" if f.integer else "double",
                               "feature": True, "min": f.lo, "max": f.hi})
        fields.append({"name": class_name, "ordinal": len(self.fields) + 1, "dataType": "categorical",
                       "cardinality": ["0", "1"]})
        return {"fields": fields}


def loan_approval() -> ScoreModel:
    """loan_approve.py ``initOne`` distributions, scores, couplings and threshold 118 +- 5."""
    zip_rate = CatField("zipRate", ["high", "average", "low"], [30, 100, 60], [17, 15, 11])
    flds = [
        CatField("married", ["married", "single", "divorced"], [80, 100, 30], [16, 10, 6]),
        CatField("numChild", ["1", "2", "3"], [80, 140, 0.001], [12, 9, 4]),
        CatField("education", ["1", "2", "3"], [60, 100, 30], [7, 12, 15]),
        CatField("selfEmployed", ["1", "0"], [30, 100], [11, 15]),
        NumField("income", 100, 20, 50, 160, steps=[(50, 70, 2), (70, 90, 5), (90, 100, 8), (100, 110, 12),
                                                    (110, 130, 14), (130, 150, 18)]),
        NumField("yearsExp", 10, 3, 6, 20, steps=[(6, 10, 4), (10, 14, 9), (14, 20, 13)]),
        NumField("outstandingLoan", 20, 5, steps=[(2, 4, 16), (4, 8, 13), (8, 14, 10), (14, 22, 8), (22, 32, 6),
                                                  (32, 44, 2)]),
        NumField("loanAmount", 300, 70, 200, 500, steps=[(200, 250, 22), (250, 300, 20), (300, 350, 16),
                                                         (350, 400, 10), (400, 450, 5), (450, 500, 2)]),
        CatField("loanTerm", ["10", "15", "30"], [40, 60, 100], [15, 18, 23]),
        NumField("creditScore", 700, 50, 600, 850, steps=[(600, 650, 8), (650, 700, 12), (700, 750, 17),
                                                          (750, 800, 23), (800, 850, 31)]),
        zip_rate,
    ]

    def couple(c, m):
        inc, am, cs = c["income"], c["loanAmount"], c["creditScore"]
        d = torch.zeros_like(inc)
        d += torch.where((inc > 140) & (am < 300), 10.0, 0.0)
        d -= torch.where((inc < 80) & (am > 280), 12.0, 0.0)
        d += torch.where((cs > 760) & (am < 320), 12.0, 0.0)
        d -= torch.where((cs < 700) & (am > 260), 14.0, 0.0)
        d -= torch.where((c["numChild"] == 2) & (inc < 100), 8.0, 0.0)
        return d
    return ScoreModel(flds, threshold=118, margin=5, couplings=[couple])


def class_conditional(class_weights: Sequence[float], fields: dict[str, list], n: int, seed: int = 0,
                      device="cpu"):
    """``initTwo`` style: draw the class first, then each field from its class-conditional
    distribution.  fields[name] = per-class spec: ("cat", values, weights) or ("num", mean, sd)."""
    dev = torch.device(device)
    g = torch.Generator(device=dev).manual_seed(seed)
    cw = torch.tensor(class_weights, dtype=torch.float64, device=dev)
    y = torch.multinomial(cw / cw.sum(), n, replacement=True, generator=g)
    cols = {}
    for name, per_class in fields.items():
        if per_class[0][0] == "cat":
            W = torch.tensor([pc[2] for pc in per_class], dtype=torch.float64, device=dev)     # [C, V]
            P = W / W.sum(1, keepdim=True)
            u = torch.rand(n, dtype=torch.float64, device=dev, generator=g)
            cdf = torch.cumsum(P, 1)[y]
            cols[name] = (u.view(-1, 1) > cdf).sum(1).clamp_max(P.shape[1] - 1)
        else:
            mu = torch.tensor([pc[1] for pc in per_class], dtype=torch.float64, device=dev)[y]
            sd = torch.tensor([pc[2] for pc in per_class], dtype=torch.float64, device=dev)[y]
            cols[name] = mu + sd * torch.randn(n, dtype=torch.float64, device=dev, generator=g)
    return cols, y
