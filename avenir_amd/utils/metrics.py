"""Metrics: counters that mirror the reference's Hadoop counter groups, and classification metrics.

Counter groups keep the reference names so outputs stay recognisable: "Validation"
(TruePositive, FalseNegative, TrueNagative [sic], FalsePositive, Accuracy, Recall, Precision,
Correct, Incorrect — ``J/bayesian/BayesianPredictor.java:172-178``), "Distribution Data"
(``J/bayesian/BayesianDistribution.java:243-320``), "Stats", "Basic".  Counters can be summed
across ranks with one all-reduce (``Counters.all_reduce``).
"""
from __future__ import annotations

import json
import math
from collections import defaultdict
from typing import Sequence

import torch


class Counters:
    def __init__(self):
        self._c: dict[str, dict[str, int]] = defaultdict(lambda: defaultdict(int))

    def incr(self, group: str, name: str, by: int = 1) -> None:
        self._c[group][name] += int(by)

    def set(self, group: str, name: str, value: int) -> None:
        self._c[group][name] = int(value)

    def get(self, group: str, name: str) -> int:
        return self._c.get(group, {}).get(name, 0)

    def as_dict(self) -> dict[str, dict[str, int]]:
        return {g: dict(v) for g, v in self._c.items()}

    def all_reduce(self, comm) -> None:
        keys = sorted((g, n) for g, v in self._c.items() for n in v)
        keys = comm.broadcast_object(keys)
        t = torch.tensor([self.get(g, n) for g, n in keys], dtype=torch.long,
                         device=comm.device if comm.backend == "nccl" else "cpu")
        comm.all_reduce(t)
        for (g, n), v in zip(keys, t.tolist()):
            self._c[g][n] = v

    def dumps(self) -> str:
        return json.dumps(self.as_dict(), indent=1, sort_keys=True)

    def __repr__(self) -> str:
        return f"Counters({self.as_dict()})"


class ConfusionMatrix:
    """Binary confusion matrix with integer-percent reports (``J/util/ConfusionMatrix.java``)."""

    def __init__(self, neg_class: str, pos_class: str):
        self.neg, self.pos = neg_class, pos_class
        self.tp = self.fp = self.tn = self.fn = 0

    def report(self, predicted: str, actual: str) -> None:
        if predicted == self.pos:
            if actual == self.pos:
                self.tp += 1
            else:
                self.fp += 1
        else:
            if actual == self.neg:
                self.tn += 1
            else:
                self.fn += 1

    def add_counts(self, tp: int, fp: int, tn: int, fn: int) -> None:
        self.tp += tp
        self.fp += fp
        self.tn += tn
        self.fn += fn

    @property
    def recall(self) -> int:
        return int(100 * self.tp / (self.tp + self.fn)) if self.tp + self.fn else 0

    @property
    def precision(self) -> int:
        return int(100 * self.tp / (self.tp + self.fp)) if self.tp + self.fp else 0

    @property
    def accuracy(self) -> int:
        t = self.tp + self.tn + self.fp + self.fn
        return int(100 * (self.tp + self.tn) / t) if t else 0

    def to_counters(self, counters: Counters) -> None:
        g = "Validation"
        counters.set(g, "TruePositive", self.tp)
        counters.set(g, "FalseNegative", self.fn)
        counters.set(g, "TrueNagative", self.tn)
        counters.set(g, "FalsePositive", self.fp)
        counters.set(g, "Accuracy", self.accuracy)
        counters.set(g, "Recall", self.recall)
        counters.set(g, "Precision", self.precision)


# ----------------------------------------------------------------------------------------------
# perfMetric equivalents (python/lib/mlutil.py:615-647), computed with torch on device
# ----------------------------------------------------------------------------------------------
def confusion(actual: torch.Tensor, pred: torch.Tensor, n_classes: int) -> torch.Tensor:
    a = actual.long().view(-1)
    p = pred.long().view(-1)
    ok = (a >= 0) & (a < n_classes) & (p >= 0) & (p < n_classes)
    idx = a[ok] * n_classes + p[ok]
    return torch.bincount(idx, minlength=n_classes * n_classes).view(n_classes, n_classes)


def accuracy(actual, pred) -> float:
    a, p = torch.as_tensor(actual).view(-1), torch.as_tensor(pred).view(-1)
    return float((a == p).float().mean()) if a.numel() else 0.0


def precision_recall_f1(actual, pred, pos: int = 1) -> tuple[float, float, float]:
    a, p = torch.as_tensor(actual).view(-1), torch.as_tensor(pred).view(-1)
    tp = float(((p == pos) & (a == pos)).sum())
    fp = float(((p == pos) & (a != pos)).sum())
    fn = float(((p != pos) & (a == pos)).sum())
    pr = tp / (tp + fp) if tp + fp else 0.0
    rc = tp / (tp + fn) if tp + fn else 0.0
    f1 = 2 * pr * rc / (pr + rc) if pr + rc else 0.0
    return pr, rc, f1


def roc_auc(actual, score) -> float:
    """AUC via sort + rank sum (Mann-Whitney), ties averaged."""
    a = torch.as_tensor(actual).view(-1).double()
    s = torch.as_tensor(score).view(-1).double()
    npos = float(a.sum())
    nneg = float(a.numel() - npos)
    if npos == 0 or nneg == 0:
        return math.nan
    order = torch.argsort(s)
    ss = s[order]
    ranks = torch.empty_like(s)
    r = torch.arange(1, s.numel() + 1, dtype=torch.float64, device=s.device)
    # average ranks over ties
    uniq, inv, cnt = torch.unique_consecutive(ss, return_inverse=True, return_counts=True)
    csum = torch.cumsum(cnt, 0).double()
    avg = csum - (cnt.double() - 1) / 2
    ranks[order] = avg[inv]
    del r, uniq
    return float((ranks[a > 0.5].sum() - npos * (npos + 1) / 2) / (npos * nneg))


def mse(actual, pred) -> float:
    a, p = torch.as_tensor(actual).double(), torch.as_tensor(pred).double()
    return float(((a - p) ** 2).mean())


def perf_metric(metric: str, actual: Sequence, pred: Sequence, pos: int = 1):
    m = metric.lower()
    if m in ("acc", "accuracy"):
        return accuracy(actual, pred)
    pr, rc, f1 = precision_recall_f1(actual, pred, pos)
    if m in ("prec", "precision"):
        return pr
    if m in ("rec", "recall"):
        return rc
    if m in ("f1", "fone"):
        return f1
    if m in ("auc", "roc"):
        return roc_auc(actual, pred)
    if m == "mse":
        return mse(actual, pred)
    if m == "rmse":
        return math.sqrt(mse(actual, pred))
    if m in ("mae",):
        return float((torch.as_tensor(actual).double() - torch.as_tensor(pred).double()).abs().mean())
    if m in ("confm", "confusion"):
        n = int(max(max(actual), max(pred))) + 1
        return confusion(torch.as_tensor(actual), torch.as_tensor(pred), n)
    raise ValueError(f"unknown metric {metric}")


class MetricsRegistry:
    """Counters (grouped, reference names), gauges and fixed-bucket histograms; ``snapshot()`` is a
    JSON-able dict, ``all_reduce`` sums counters / histograms and maxes gauges across ranks."""

    def __init__(self, buckets: Sequence[float] = (0.1, 0.5, 1, 5, 10, 50, 100, 500, 1000)):
        self.counters = Counters()
        self.gauges: dict[str, float] = {}
        self.buckets = list(buckets)
        self.hists: dict[str, list[int]] = {}

    def gauge(self, name: str, value: float) -> None:
        self.gauges[name] = float(value)

    def observe(self, name: str, value: float) -> None:
        h = self.hists.setdefault(name, [0] * (len(self.buckets) + 1))
        i = next((k for k, b in enumerate(self.buckets) if value <= b), len(self.buckets))
        h[i] += 1

    def snapshot(self) -> dict:
        return {"counters": self.counters.as_dict(), "gauges": dict(self.gauges),
                "histograms": {k: {"buckets": self.buckets, "counts": v} for k, v in self.hists.items()}}

    def all_reduce(self, comm) -> None:
        self.counters.all_reduce(comm)
        dev = comm.device if comm.backend == "nccl" else "cpu"
        names = comm.broadcast_object(sorted(self.hists))
        if names:
            t = torch.tensor([self.hists.get(n, [0] * (len(self.buckets) + 1)) for n in names], device=dev)
            comm.all_reduce(t)
            self.hists = {n: row for n, row in zip(names, t.tolist())}
        gnames = comm.broadcast_object(sorted(self.gauges))
        if gnames:
            g = torch.tensor([self.gauges.get(n, float("-inf")) for n in gnames], dtype=torch.float64, device=dev)
            comm.all_reduce(g, op="max")
            self.gauges = dict(zip(gnames, g.tolist()))

    def dumps(self) -> str:
        return json.dumps(self.snapshot(), indent=1, sort_keys=True)


METRICS = MetricsRegistry()
