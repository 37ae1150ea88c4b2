"""Cost-based decisions and attribute-change costs.

* ``CostBasedArbitrator`` (J/util/CostBasedArbitrator.java:50-64): with integer percent
  probabilities, predict positive when ``fpCost * negProb + posProb < fnCost * posProb + negProb``;
  ``classify(posProb)``: positive when posProb > 100 * fpCost / (fpCost + fnCost).  Vectorised
  over a batch of probabilities.
* ``CostSchema`` / ``CostAttribute`` (J/util/CostSchema.java:43-72, R/churnPreventCost.json): cost
  of changing a numeric attribute = numAttrCost x change; categorical from->to costs from a map
  (missing pair = 0).  ``batch_cost`` prices [N, F] attribute changes in one reduction.
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Sequence

import torch


class CostBasedArbitrator:
    def __init__(self, neg_class: str, pos_class: str, false_neg_cost: int, false_pos_cost: int):
        self.neg, self.pos = neg_class, pos_class
        self.fn, self.fp = int(false_neg_cost), int(false_pos_cost)

    def arbitrate(self, pos_prob, neg_prob):
        """Scalar or tensor integer-percent probabilities -> class label(s)."""
        pp, npb = torch.as_tensor(pos_prob), torch.as_tensor(neg_prob)
        neg_cost = self.fn * pp + npb
        pos_cost = self.fp * npb + pp
        is_pos = pos_cost < neg_cost
        if is_pos.dim() == 0:
            return self.pos if bool(is_pos) else self.neg
        return is_pos

    def classify(self, pos_prob):
        thr = (self.fp * 100) // (self.fp + self.fn)
        r = torch.as_tensor(pos_prob) > thr
        if r.dim() == 0:
            return self.pos if bool(r) else self.neg
        return r


class CostAttribute:
    def __init__(self, name: str, ordinal: int, num_cost: float | None = None, cat_cost: dict | None = None):
        self.name, self.ordinal, self.num_cost, self.cat_cost = name, ordinal, num_cost, dict(cat_cost or {})


class CostSchema:
    def __init__(self, attributes: Sequence[CostAttribute]):
        self.attributes = list(attributes)
        self._by = {a.ordinal: a for a in self.attributes}

    @classmethod
    def from_json(cls, obj) -> "CostSchema":
        if isinstance(obj, (str, Path)):
            obj = json.loads(Path(obj).read_text())
        attrs = [CostAttribute(f.get("name", ""), int(f["ordinal"]), f.get("numAttrCost"), f.get("catAttrCost"))
                 for f in obj["fields"]]
        return cls(attrs)

    def findCostAttribute(self, attr: int) -> CostAttribute | None:
        return self._by.get(attr)

    def findCost(self, attr: int, a, b=None) -> float:
        ca = self._by.get(attr)
        if ca is None:
            raise ValueError("invalid attribute ordinal")
        if b is None:
            return float((ca.num_cost or 0.0) * float(a))
        return float(ca.cat_cost.get(f"{a},{b}", 0.0))

    def batch_cost(self, ordinals: Sequence[int], delta: torch.Tensor) -> torch.Tensor:
        """Total cost of numeric changes ``delta`` [N, F] (columns = ``ordinals``) per row."""
        w = torch.tensor([float(self._by[o].num_cost or 0.0) for o in ordinals], dtype=delta.dtype,
                         device=delta.device)
        return delta @ w
