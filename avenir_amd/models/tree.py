"""Decision trees, random forests and gradient-boosted trees on the GPU.

Reference behaviour (``J/tree``, ``J/model``, ``P/supv/rf.py``, ``P/supv/gbt.py``):

* ``DecisionTreeBuilder`` grows a tree level by level (one Hadoop job per level).  Candidate splits
  come from ``SplitManager``: numeric attributes split at multiples of ``splitScanInterval`` between
  ``min`` and ``max`` into up to ``maxSplit`` segments (``SplitManager.java:256-330``), categorical
  attributes are partitioned into 2..``maxSplit`` value groups (``:405-522``).  Each parent keeps
  the split with the minimum population-weighted entropy / gini of its children (``best``) or a
  random one among the top ``dtb.top.split.count`` (``randomAmongTop``)
  (``DecisionTreeBuilder.java:499-616``); ``DecisionPathStoppingStrategy`` stops a path by
  ``maxDepth`` / ``minInfoGain`` / ``minPopulation`` (``:57-70``); attributes per path are chosen
  ``all`` / ``notUsedYet`` / ``randomAll`` / ``randomNotUsedYet`` (``:365-381``); sub-sampling is
  ``withReplace`` / ``withoutReplace`` / ``none``.  The model is a JSON ``DecisionPathList``.
* ``DecisionTreeModel`` predicts with the first matching path (``DecisionTreeModel.java:56-93``);
  ``EnsemblePredictiveModel`` is a weighted majority vote (``EnsemblePredictiveModel.java:69-110``).

MI355X design: a level = ONE histogram kernel pass (``node_hist``: class counts per frontier node x
fine bin, where every candidate split of every attribute is a grouping of fine bins), split scoring
for all nodes x all candidate splits as batched tensor math on the device, and ONE row-assignment
kernel pass.  Data-parallel across ranks: the [A, C, TB] histogram is all-reduced once per level,
so every rank takes identical decisions (shared seeded RNG) and moves its own rows.

Documented divergence: the reference's multi-point numeric split emits an unbounded ``le`` for its
last interior segment (``SplitManager.java:620-660``, the segments then overlap); here every segment
is bounded (``attr le p2 p1`` = ``p1 < x <= p2``), which is what the predicate evaluation intends.
"""
from __future__ import annotations

import itertools
import json
import os
import math
import random
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Sequence

import numpy as np
import torch

from .. import _native
from ..data.table import MISSING, Table, pad16
from ..ops import tree_ops as T
from ..parallel.comm import Comm, get_comm
from ..utils.schema import FeatureField, FeatureSchema

ROOT = "$root"


# ================================================================================================
# Split space: per-attribute fine-bin encoding + candidate splits
# ================================================================================================
@dataclass
class Split:
    segmap: list[int]          # fine bin -> segment
    n_seg: int
    predicates: list[str]      # predicate string per segment (reference syntax)


@dataclass
class FeatureSplits:
    field: FeatureField
    kind: str                          # "cat" | "num"
    points: list[float] = field(default_factory=list)   # numeric split points (fine-bin edges)
    splits: list[Split] = field(default_factory=list)
    binary: bool = False               # binary threshold splits scored by prefix sums

    @property
    def n_bins(self) -> int:
        return len(self.field.cardinality) if self.kind == "cat" else len(self.points) + 1

    def encode(self, t: Table) -> torch.Tensor:
        """uint8 [ld] fine-bin codes of this attribute for table ``t`` (255 = missing)."""
        f = self.field
        if self.kind == "cat":
            j = [x.ordinal for x in t.binned_fields].index(f.ordinal)
            return t.codes[j]
        # numeric: need the raw column
        names = [x.ordinal for x in t.numeric_fields]
        if f.ordinal in names:
            x = t.numeric[names.index(f.ordinal)]
            pts = torch.tensor(self.points, dtype=torch.float32, device=x.device)
            b = torch.bucketize(x, pts, right=False)  # P[b-1] < x <= P[b]
            b = torch.where(torch.isnan(x), torch.full_like(b, MISSING), b)
            return b.clamp_max(MISSING).to(torch.uint8)
        j = [x.ordinal for x in t.binned_fields].index(f.ordinal)
        # bucketized column (bucketWidth): map bucket centre to fine bins (approximate)
        c = t.codes[j].long()
        lo = (c + f.bucket_offset).float() * f.bucket_width
        pts = torch.tensor(self.points, dtype=torch.float32, device=c.device)
        b = torch.bucketize(lo, pts, right=False)
        return torch.where(c >= MISSING, torch.full_like(b, MISSING), b).to(torch.uint8)

    def pred_value(self, v: float) -> str:
        if self.field.is_integer or float(v).is_integer():
            return str(int(round(v)))
        return repr(float(v))


def _set_partitions(values: list[str], k: int):
    """All partitions of ``values`` into exactly ``k`` non-empty groups (restricted growth strings),
    in a canonical order."""
    n = len(values)

    def rec(i, assign, m):
        if i == n:
            if m == k:
                yield list(assign)
            return
        if n - i < k - m:  # not enough elements left to open the remaining groups
            return
        for g in range(min(m + 1, k)):
            assign.append(g)
            yield from rec(i + 1, assign, max(m, g + 1))
            assign.pop()

    yield from rec(0, [], 0)


def categorical_splits(field: FeatureField, max_split: int | None = None, cap: int = 4096) -> list[Split]:
    card = list(field.cardinality)
    ms = max(2, max_split or field.max_split or 2)
    out = []
    for k in range(2, min(ms, len(card)) + 1):
        for assign in _set_partitions(card, k):
            groups = [[card[i] for i in range(len(card)) if assign[i] == g] for g in range(k)]
            preds = [f"{field.ordinal} in {':'.join(gv)}" for gv in groups]
            out.append(Split(list(assign), k, preds))
            if len(out) >= cap:
                return out
    return out


def numeric_points(field: FeatureField, values: torch.Tensor | None = None, max_bins: int = 32) -> list[float]:
    """Split points: multiples of splitScanInterval in (min, max) (reference), else data quantiles."""
    if field.min is not None and field.max is not None and field.split_scan_interval:
        lo, hi, step = field.min, field.max, field.split_scan_interval
        if int((hi - lo) / step) == 0:
            step = (hi - lo) / 2
        pts, p = [], lo + step
        while p < hi - 1e-12:
            pts.append(p)
            p += step
        return pts
    if values is None:
        raise ValueError(f"field {field.name}: no min/max/splitScanInterval and no data for quantiles")
    v = values[~torch.isnan(values)].float()
    if v.numel() == 0:
        return []
    qs = torch.linspace(0, 1, max_bins + 1, device=v.device)[1:-1]
    if v.numel() > 1 << 20:
        # bin edges from a strided 1M-value sample (deterministic; quantile error ~1e-3, far below
        # the 1/max_bins bin width) instead of a full sort of every column
        v = v[:: (v.numel() + (1 << 20) - 1) >> 20]
    pts = torch.unique(torch.quantile(v, qs)).cpu().tolist()
    return [float(p) for p in pts]


def numeric_splits(fs: FeatureSplits, max_split: int | None = None, cap: int = 4096) -> list[Split]:
    P = fs.points
    ms = max(2, max_split or fs.field.max_split or 2)
    out = []
    for m in range(1, ms):
        for combo in itertools.combinations(range(len(P)), m):
            pts = [P[i] for i in combo]
            # fine bin b covers (P[b-1], P[b]]: segment = #chosen points <= P[b-1]
            segmap = []
            for b in range(len(P) + 1):
                segmap.append(0 if b == 0 else sum(1 for i in combo if i <= b - 1))
            o = fs.field.ordinal
            pv = [fs.pred_value(p) for p in pts]
            preds = [f"{o} le {pv[0]}"]
            for i in range(1, len(pv)):
                preds.append(f"{o} le {pv[i]} {pv[i - 1]}")
            preds.append(f"{o} gt {pv[-1]}")
            out.append(Split(segmap, m + 1, preds))
            if len(out) >= cap:
                return out
    return out


def build_split_space(schema: FeatureSchema, t: Table | None = None, attrs: Sequence[int] | None = None,
                      binary: bool = False, max_bins: int = 32, comm=None) -> list[FeatureSplits]:
    """Candidate-split space over the feature attributes (reference SplitManager semantics, or
    binary threshold splits over ordered fine bins when ``binary``).  With ``comm`` distributed and
    row shards, data-quantile split points come from the values of ALL ranks (one all-gather per
    numeric column of at most 2^20 / world sampled values each), so every rank bins identically."""
    out = []
    gather = comm is not None and comm.is_distributed
    pre = _batched_points(schema, t, attrs, binary, max_bins) if (t is not None and not gather) else {}
    for f in schema.feature_fields:
        if attrs is not None and f.ordinal not in attrs:
            continue
        if f.ordinal in pre:
            fs = FeatureSplits(f, "num", points=pre[f.ordinal], binary=binary)
            if not binary:
                fs.splits = numeric_splits(fs)
            if fs.n_bins > 254:
                raise ValueError(f"attribute {f.name}: {fs.n_bins} fine bins > 254")
            out.append(fs)
            continue
        if f.is_categorical:
            fs = FeatureSplits(f, "cat", binary=binary)
            if not binary:
                fs.splits = categorical_splits(f)
        elif f.is_numeric:
            vals = None
            if t is not None:
                names = [x.ordinal for x in t.numeric_fields]
                if f.ordinal in names:
                    vals = t.numeric[names.index(f.ordinal), : t.n]
                    if gather and (binary or not (f.min is not None and f.max is not None
                                                  and f.split_scan_interval)):
                        vals = _gather_sample(vals, comm)
            if binary or not (f.min is not None and f.max is not None and f.split_scan_interval):
                pts = numeric_points(FeatureField(f.name, f.ordinal, f.data_type), vals, max_bins)
            else:
                pts = numeric_points(f, vals, max_bins)
            fs = FeatureSplits(f, "num", points=pts, binary=binary)
            if not binary:
                fs.splits = numeric_splits(fs)
        else:
            continue
        if fs.n_bins > 254:
            raise ValueError(f"attribute {f.name}: {fs.n_bins} fine bins > 254")
        out.append(fs)
    return out


def _batched_points(schema, t: Table, attrs, binary: bool, max_bins: int) -> dict[int, list[float]]:
    """Quantile split points of every data-quantile numeric feature in ONE batched quantile over a
    stacked [F, m] sample (one sort launch instead of one per column); identical to
    ``numeric_points`` per column.  Columns with NaNs are left to the per-column path."""
    names = [x.ordinal for x in t.numeric_fields]
    fields = [f for f in schema.feature_fields
              if (attrs is None or f.ordinal in attrs) and f.is_numeric and f.ordinal in names
              and (binary or not (f.min is not None and f.max is not None and f.split_scan_interval))]
    if len(fields) < 2 or t.n == 0:
        return {}
    V = t.numeric[[names.index(f.ordinal) for f in fields], : t.n].float()
    if bool(torch.isnan(V).any()):
        return {}
    if V.shape[1] > 1 << 20:
        V = V[:, :: (V.shape[1] + (1 << 20) - 1) >> 20]
    qs = torch.linspace(0, 1, max_bins + 1, device=V.device)[1:-1]
    Q = torch.quantile(V, qs, dim=1).t().contiguous().cpu()           # [F, nq]
    return {f.ordinal: [float(p) for p in torch.unique(Q[i]).tolist()] for i, f in enumerate(fields)}


def _gather_sample(vals: torch.Tensor, comm) -> torch.Tensor:
    """This rank's column values (strided to <= 2^20 / world when larger) gathered from all ranks."""
    cap = max(1, (1 << 20) // comm.world)
    v = vals[:: (vals.numel() + cap - 1) // cap] if vals.numel() > cap else vals
    dev = comm.device if comm.backend == "nccl" else torch.device("cpu")
    return comm.all_gather_v(v.float().contiguous().to(dev)).to(vals.device)


def _with_total_row(codes: torch.Tensor, n: int) -> torch.Tensor:
    tot = torch.full((1, codes.shape[1]), MISSING, dtype=torch.uint8, device=codes.device)
    tot[0, :n] = 0
    return torch.cat([codes, tot], 0)


def encode_for_tree(space: list[FeatureSplits], t: Table) -> torch.Tensor:
    ld = t.ld
    codes = torch.full((len(space), ld), MISSING, dtype=torch.uint8, device=t.device)
    names = [x.ordinal for x in t.numeric_fields]
    raw = [i for i, fs in enumerate(space) if fs.kind == "num" and fs.field.ordinal in names and len(fs.points) <= 254]
    if t.device.type == "cuda" and raw:
        # every raw numeric column in ONE fused bucketize launch (forest.hip bucketize_u8)
        from .. import _native
        X = t.numeric[[names.index(space[i].field.ordinal) for i in raw]].contiguous()
        edges = torch.tensor([p for i in raw for p in space[i].points], dtype=torch.float32, device=t.device)
        eoff = torch.tensor(list(itertools.accumulate([0] + [len(space[i].points) for i in raw])), dtype=torch.int32)
        out = torch.empty((len(raw), ld), dtype=torch.uint8, device=t.device)
        _native.C().bucketize_u8(X, int(t.n), edges, eoff, out)
        codes[raw, : t.n] = out[:, : t.n]
    for i, fs in enumerate(space):
        if t.device.type == "cuda" and i in raw:
            continue
        c = fs.encode(t)
        codes[i, : c.shape[0]] = c[:ld]
    codes[:, t.n:] = MISSING
    return codes


# ================================================================================================
# impurity
# ================================================================================================
def impurity(counts: torch.Tensor, algorithm: str) -> torch.Tensor:
    """Entropy (base 2) or gini over the last dim of class counts (InfoContentStat.processStat)."""
    tot = counts.sum(-1, keepdim=True).double()
    p = counts.double() / tot.clamp_min(1)
    if algorithm == "entropy":
        return -(torch.where(p > 0, p * torch.log2(p.clamp_min(1e-300)), torch.zeros_like(p))).sum(-1)
    if algorithm in ("giniIndex", "gini"):
        return 1.0 - (p * p).sum(-1)
    raise ValueError(f"unsupported split algorithm {algorithm}")


# ================================================================================================
# tree structure
# ================================================================================================
@dataclass
class Node:
    predicates: list[str]
    population: int
    info: float
    class_pr: list[float]
    depth: int
    stopped: bool = False
    feature: int = -1            # index into the split space (internal nodes)
    split: int = -1              # index of the chosen split
    segmap: list[int] | None = None
    children: list[int] = field(default_factory=list)   # per segment: node index or -1
    used_attrs: frozenset = frozenset()

    @property
    def is_leaf(self) -> bool:
        return self.feature < 0


class DecisionTree:
    """A built tree: node list (index 0 = root) + its split space and class values."""

    def __init__(self, nodes: list[Node], space: list[FeatureSplits], class_values: list[str]):
        self.nodes = nodes
        self.space = space
        self.class_values = class_values

    # -- reference JSON (DecisionPathList) ---------------------------------------------------------
    def to_decision_paths(self, total_population: int | None = None) -> dict:
        paths = []
        for nd in self.nodes:
            if not nd.is_leaf:
                continue
            preds = [{"attribute": 0, "predicateStr": ROOT, "operator": None, "valueInt": 0,
                      "valueDbl": 0.0, "categoricalValues": None, "otherBoundInt": None,
                      "otherBoundDbl": None}]
            for ps in nd.predicates:
                preds.append(_predicate_obj(ps, self._field_of(ps)))
            cp = {cv: p for cv, p in zip(self.class_values, nd.class_pr)}
            maj = max(cp.values()) if cp else 0.0
            mino = 1.0 - maj
            conf = min(maj / mino, 100.0) if mino > 0 else 100.0
            d = {"stopped": nd.stopped or True, "classValPr": cp, "infoContent": nd.info,
                 "predicates": preds, "population": nd.population,
                 "outputClassVal": max(cp, key=cp.get) if cp else "", "confidence": conf}
            if total_population:
                d["support"] = nd.population / total_population
            paths.append(d)
        return {"decisionPaths": paths}

    def _field_of(self, ps: str) -> FeatureField:
        o = int(ps.split()[0])
        for fs in self.space:
            if fs.field.ordinal == o:
                return fs.field
        raise KeyError(o)

    def save_json(self, path: str | Path, total_population: int | None = None) -> None:
        Path(path).write_text(json.dumps(self.to_decision_paths(total_population), indent=1))

    # -- native compact format ---------------------------------------------------------------------
    def state(self) -> dict:
        return {
            "class_values": self.class_values,
            "space": [{"ordinal": fs.field.ordinal, "kind": fs.kind, "points": fs.points,
                       "binary": fs.binary} for fs in self.space],
            "nodes": [{"predicates": n.predicates, "population": n.population, "info": n.info,
                       "class_pr": n.class_pr, "depth": n.depth, "stopped": n.stopped,
                       "feature": n.feature, "split": n.split, "segmap": n.segmap,
                       "children": n.children} for n in self.nodes],
        }

    @classmethod
    def from_state(cls, st: dict, schema: FeatureSchema) -> "DecisionTree":
        space = [FeatureSplits(schema.find_field_by_ordinal(s["ordinal"]), s["kind"], list(s["points"]),
                               binary=s.get("binary", False)) for s in st["space"]]
        nodes = [Node(n["predicates"], n["population"], n["info"], n["class_pr"], n["depth"], n["stopped"],
                      n["feature"], n["split"], n["segmap"], n["children"]) for n in st["nodes"]]
        return cls(nodes, space, st["class_values"])

    # -- rules ---------------------------------------------------------------------------------
    def rules(self) -> list[tuple[str, str, float]]:
        """(predicate conjunction, class, probability) per leaf."""
        out = []
        for nd in self.nodes:
            if nd.is_leaf:
                k = int(np.argmax(nd.class_pr)) if nd.class_pr else 0
                out.append((" and ".join([ROOT] + nd.predicates), self.class_values[k], nd.class_pr[k]))
        return out


class DecisionPathModel:
    """Inference straight from the reference's decision-path JSON (J/tree/DecisionTreeModel.java:
    56-144): a record takes the first path whose predicates all hold.  Predicates (``ord le v``,
    ``ord le v lower``, ``ord gt v``, ``ord in a:b``) are evaluated column-wise over all records
    (one tensor comparison per distinct predicate), the path matches are one ``[N, P]`` boolean
    matrix, and the first matching path per record is an argmax."""

    def __init__(self, js: dict):
        self.paths = js["decisionPaths"]
        self.class_values = sorted({c for p in self.paths for c in p.get("classValPr", {})})

    def _pred(self, cols, ps: str) -> torch.Tensor:
        it = ps.split()
        o, op = int(it[0]), it[1]
        if op == "in":
            c, vocab = cols.codes(o)
            ids = [vocab[v] for v in it[2].split(":") if v in vocab]
            return (torch.isin(c, torch.tensor(ids, dtype=torch.long, device=c.device)) if ids
                    else torch.zeros_like(c, dtype=torch.bool))
        x = cols.numeric(o)
        v = float(it[2])
        if op == "le":
            m = x <= v
            if len(it) > 3:
                m &= x > float(it[3])
            return m
        if op == "gt":
            m = x > v
            if len(it) > 3:
                m &= x <= float(it[3])
            return m
        if op == "lt":
            return x < v
        if op == "ge":
            return x >= v
        raise ValueError(f"unknown predicate operator in {ps!r}")

    def predict_proba_rows(self, rows) -> tuple[torch.Tensor, torch.Tensor]:
        """(class probabilities [N, C] of the matched path, matched path index [N] (-1 = none))."""
        from ..utils.rules import ColumnCache
        return self.predict_proba_cols(ColumnCache(rows))

    def predict_proba_cols(self, cols) -> tuple[torch.Tensor, torch.Tensor]:
        """:meth:`predict_proba_rows` over a column source with ``n``, ``device``, ``codes(o)`` ->
        (codes, {value: code}) and ``numeric(o)`` -> float64 values: ``utils.rules.ColumnCache``
        (split rows), :class:`TableColumns` (a schema Table) or ``RecordColumns`` (a native token
        table) — the last two keep every step on the table's device."""
        n, P = cols.n, len(self.paths)
        dev = cols.device
        # the first matching path per record: paths visited last to first, each a chain of 1-D
        # boolean ANDs and one select (no [N, P] match matrix: contiguous passes only)
        cache: dict[str, torch.Tensor] = {}
        first = torch.full((n,), P, dtype=torch.int32, device=dev)
        for j in range(P - 1, -1, -1):
            m = None
            for pr in self.paths[j]["predicates"]:
                ps = pr["predicateStr"]
                if ps == ROOT:
                    continue
                if ps not in cache:
                    cache[ps] = self._pred(cols, ps)
                m = cache[ps].clone() if m is None else m.logical_and_(cache[ps])
            first = torch.where(m, j, first) if m is not None else torch.full_like(first, j)
        first = first.long()
        first = torch.where(first < P, first, torch.full_like(first, -1))
        ci = {c: i for i, c in enumerate(self.class_values)}
        tab = torch.zeros((P + 1, len(ci)), dtype=torch.float64)
        for j, p in enumerate(self.paths):
            for c, v in p.get("classValPr", {}).items():
                tab[j, ci[c]] = float(v)
        return tab.to(dev)[torch.where(first >= 0, first, torch.full_like(first, P))], first


class TableColumns:
    """Column source of :meth:`DecisionPathModel.predict_proba_cols` over a schema Table (loaded
    with ``raw_numeric``): categorical codes with the schema dictionary, numeric columns widened to
    float64 — the predicate thresholds the builder writes come from the same float32 columns."""

    def __init__(self, t: Table):
        self.t, self.n, self.device = t, t.n, t.device

    def codes(self, o: int):
        for j, f in enumerate(self.t.binned_fields):
            if f.ordinal == o:
                return self.t.codes[j, : self.n].long(), {v: i for i, v in enumerate(f.cardinality or [])}
        raise KeyError(f"field {o} is not a binned field of the table")

    def numeric(self, o: int) -> torch.Tensor:
        for j, f in enumerate(self.t.numeric_fields):
            if f.ordinal == o:
                return self.t.numeric[j, : self.n].double()
        raise KeyError(f"field {o} is not a numeric field of the table")


def _predicate_obj(ps: str, f: FeatureField) -> dict:
    it = ps.split()
    d = {"attribute": int(it[0]), "predicateStr": ps, "operator": it[1], "valueInt": 0, "valueDbl": 0.0,
         "categoricalValues": None, "otherBoundInt": None, "otherBoundDbl": None}
    if it[1] == "in":
        d["categoricalValues"] = it[2].split(":")
    elif f.is_integer:
        d["valueInt"] = int(float(it[2]))
        if len(it) > 3:
            d["otherBoundInt"] = int(float(it[3]))
    else:
        d["valueDbl"] = float(it[2])
        if len(it) > 3:
            d["otherBoundDbl"] = float(it[3])
    return d


# ================================================================================================
# builder
# ================================================================================================
@dataclass
class TreeParams:
    algorithm: str = "giniIndex"                  # entropy | giniIndex
    stopping: str = "maxDepth"                    # maxDepth | minInfoGain | minPopulation
    max_depth: int = 3
    min_info_gain: float = 0.0
    min_population: int = 1
    attr_selection: str = "notUsedYet"            # all | notUsedYet | randomAll | randomNotUsedYet
    random_attr_count: int = 3
    split_selection: str = "best"                 # best | randomAmongTop
    top_split_count: int = 3
    sub_sampling: str = "none"                    # none | withReplace | withoutReplace
    sampling_rate: float = 100.0                  # percent, withoutReplace
    seed: int = 0
    binary: bool = False                          # binary threshold splits (RF / sklearn style)
    max_bins: int = 32

    @classmethod
    def from_config(cls, cfg) -> "TreeParams":
        """From a ``dtb.``-prefixed JobConfig (reference keys, R/detr.properties)."""
        p = cls()
        p.algorithm = cfg.get_str("split.algorithm", p.algorithm)
        p.stopping = cfg.get_str("path.stopping.strategy", "minInfoGain")
        if p.stopping == "maxDepth":
            p.max_depth = cfg.get_int("max.depth.limit")
        elif p.stopping == "minInfoGain":
            p.min_info_gain = cfg.get_float("min.info.gain.limit")
        elif p.stopping == "minPopulation":
            p.min_population = cfg.get_int("min.population.limit")
        p.attr_selection = cfg.get_str("split.attribute.selection.strategy", p.attr_selection)
        p.random_attr_count = cfg.get_int("random.split.set.size", p.random_attr_count)
        p.split_selection = cfg.get_str("split.select.strategy", p.split_selection)
        p.top_split_count = cfg.get_int("top.split.count", p.top_split_count)
        p.sub_sampling = cfg.get_str("sub.sampling.strategy", p.sub_sampling)
        p.sampling_rate = cfg.get_float("sub.sampling.rate", p.sampling_rate)
        p.seed = cfg.get_int("random.seed", p.seed)
        return p


class DecisionTreeBuilder:
    """Level-wise GPU tree builder (data parallel over ranks)."""

    def __init__(self, schema: FeatureSchema, params: TreeParams | None = None, comm: Comm | None = None,
                 space: list[FeatureSplits] | None = None):
        self.schema = schema
        self.p = params or TreeParams()
        self.comm = comm
        self.space = space
        self.level_times: list[float] = []

    # -- helpers -------------------------------------------------------------------------------
    def _weights(self, t: Table, rng_seed: int) -> torch.Tensor | None:
        p = self.p
        if p.sub_sampling == "none":
            return None
        comm = self.comm or get_comm()
        g = torch.Generator(device=t.device)
        g.manual_seed(rng_seed * 1000003 + comm.rank)
        if p.sub_sampling == "withReplace":
            w = torch.poisson(torch.ones(t.ld, device=t.device), generator=g).clamp_max(255)
        elif p.sub_sampling == "withoutReplace":
            w = (torch.rand(t.ld, generator=g, device=t.device) * 100.0 < p.sampling_rate).float()
        else:
            raise ValueError(f"unknown sub sampling strategy {p.sub_sampling}")
        w[t.n:] = 0
        return w.to(torch.uint8)

    def _candidate_attrs(self, nd: Node, F: int, rng: random.Random) -> list[int]:
        s = self.p.attr_selection
        allf = list(range(F))
        if s == "all":
            return allf
        remaining = [f for f in allf if f not in nd.used_attrs] or allf
        if s == "notUsedYet":
            return remaining
        if s == "randomAll":
            return sorted(rng.sample(allf, min(self.p.random_attr_count, F)))
        if s == "randomNotUsedYet":
            return sorted(rng.sample(remaining, min(self.p.random_attr_count, len(remaining))))
        raise ValueError(f"unknown attribute selection strategy {s}")

    def _should_stop(self, pop: int, info: float, parent_info: float, depth: int) -> bool:
        p = self.p
        if p.stopping == "maxDepth":
            return depth >= p.max_depth
        if p.stopping == "minInfoGain":
            return (parent_info - info) < p.min_info_gain
        if p.stopping == "minPopulation":
            return pop < p.min_population
        raise ValueError(f"invalid stopping strategy {p.stopping}")

    # -- build ---------------------------------------------------------------------------------
    def fit(self, t: Table, tree_seed: int | None = None, codes: torch.Tensor | None = None) -> DecisionTree:
        """One tree over this rank's rows (``sub.sampling`` weights from a seeded generator)."""
        comm = self.comm or get_comm()
        p = self.p
        seed = p.seed if tree_seed is None else tree_seed
        if self.space is None:
            self.space = build_split_space(self.schema, t, binary=p.binary, max_bins=p.max_bins, comm=comm)
        if codes is None:
            codes = encode_for_tree(self.space, t)
        node0 = torch.full((t.ld,), -1, dtype=torch.int32, device=t.device)
        node0[: t.n] = 0
        cls = list(t.class_field.cardinality) if t.class_field else ["_"]
        return self._grow(_with_total_row(codes, t.n), t.n, t.labels, self._weights(t, seed), node0,
                          [random.Random(seed)], t.n_classes, cls)[0]

    def fit_many(self, t: Table, seeds: Sequence[int], codes: torch.Tensor | None = None) -> list[DecisionTree]:
        """Several trees at once (a random forest with the reference's split semantics: multi-way
        numeric splits, categorical set partitions, ``notUsedYet`` / ``randomNotUsedYet``): every
        tree's bootstrap sample is a contiguous block of one row buffer (forest.hip bootstrap kernels:
        multiplicity = f(seed, tree, GLOBAL row), so samples do not depend on the device or the
        world size), every level of ALL trees is one histogram launch, one scoring pass and one
        host copy.  Tree i uses ``seeds[i]`` for its bootstrap and its attribute / split draws, so
        it equals the tree a one-tree build with that seed and sample would give."""
        from ..ops import forest_ops as FO
        comm = self.comm or get_comm()
        p = self.p
        if self.space is None:
            self.space = build_split_space(self.schema, t, binary=p.binary, max_bins=p.max_bins, comm=comm)
        if codes is None:
            codes = encode_for_tree(self.space, t)
        if p.sub_sampling not in FO.BOOT_MODES:
            raise ValueError(f"unknown sub sampling strategy {p.sub_sampling}")
        mode = FO.BOOT_MODES[p.sub_sampling]
        rate32 = min(int(min(max(p.sampling_rate, 0.0), 100.0) / 100.0 * 4294967296.0), 0xFFFFFFFF)
        keys = np.asarray([((s * 1000003 + 17) * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF for s in seeds],
                          dtype=np.uint64).view(np.int64)
        dev = t.device
        # the node-total slot row rides along the bootstrap (a copy of the input's codes, not of the
        # several-times larger bootstrap buffer)
        cb, lb, wb, cnt = FO.forest_bootstrap(_with_total_row(codes, t.n).contiguous(), t.labels.to(dev).contiguous(),
                                              t.n, keys, t.row_offset, mode, rate32)
        cnt_h = [int(x) for x in cnt.tolist()]
        R = sum(cnt_h)
        cb[-1, R:] = MISSING
        node0 = torch.full((cb.shape[1],), -1, dtype=torch.int32, device=dev)
        a = 0
        for i, c in enumerate(cnt_h):           # tree i's rows are one contiguous block
            node0[a:a + c] = i
            a += c
        cls = list(t.class_field.cardinality) if t.class_field else ["_"]
        starts = list(itertools.accumulate([0] + cnt_h))
        return self._grow(cb, R, lb, wb, node0, [random.Random(s) for s in seeds], t.n_classes, cls,
                          tree_rows=list(zip(starts[:-1], starts[1:])))

    def _grow(self, codes: torch.Tensor, n: int, labels: torch.Tensor, weight: torch.Tensor | None,
              node: torch.Tensor, rngs: list, C: int, cls: list[str],
              tree_rows: list[tuple[int, int]] | None = None) -> list[DecisionTree]:
        """Level-wise growth of ``len(rngs)`` trees whose rows are marked by ``node`` (row -> root
        slot = tree index, -1 = unused).  Per level, for every frontier node of every tree: ONE
        histogram launch (children whose parent is fully covered are derived by subtraction), the
        scores of every candidate split of every attribute as batched device tensor math, the
        segment counts of the chosen (or top-k) splits gathered on the device, and ONE host copy.
        The host then only creates node objects.  ``tree_rows``: tree i's rows are the block
        [lo, hi) (fit_many's bootstrap layout), so each histogram chunk scans only its trees' rows."""
        import time
        t_grow0 = time.perf_counter()
        comm = self.comm or get_comm()
        p = self.p
        space = self.space
        F = len(space)
        bins = [fs.n_bins for fs in space] + [1]
        offs = list(itertools.accumulate([0] + bins[:-1]))
        TBt = offs[F] + 1
        dev = codes.device
        NT = len(rngs)

        # ---- explicit (multi-way / categorical partition) splits of every feature, once ----------
        nb_f = [f for f, fs in enumerate(space) if not fs.binary and len(fs.splits)]
        Gmax = max([s.n_seg for f in nb_f for s in space[f].splits] + [2])
        Bmax = max([space[f].n_bins for f in nb_f] + [1])
        seg_np = {}
        nb_rows = []                              # (feature, split) of every explicit split, in order
        for f in nb_f:
            fs = space[f]
            S, B = len(fs.splits), fs.n_bins
            M = np.zeros((S, Gmax, B))
            for si, sp in enumerate(fs.splits):
                M[si, np.asarray(sp.segmap, dtype=np.int64), np.arange(len(sp.segmap))] = 1.0
            seg_np[f] = M
            nb_rows += [(f, s) for s in range(S)]
        seg_tensors = {f: torch.from_numpy(M).to(dev) for f, M in seg_np.items()}
        if nb_rows:
            # per explicit split: its [Gmax, Bmax] segment map and the histogram column of each bin
            # (TBt = an all-zero column appended for the padding bins)
            allseg = np.zeros((len(nb_rows), Gmax, Bmax))
            splitcol = np.full((len(nb_rows), Bmax), TBt, dtype=np.int64)
            r = 0
            for f in nb_f:
                S, B = seg_np[f].shape[0], space[f].n_bins
                allseg[r:r + S, :, :B] = seg_np[f]
                splitcol[r:r + S, :B] = np.arange(offs[f], offs[f] + B)
                r += S
            allseg, splitcol = torch.from_numpy(allseg).to(dev), torch.from_numpy(splitcol).to(dev)

        # binary-threshold features are scored together: one segmented cumsum over their bins
        bin_f = [f for f, fs in enumerate(space) if fs.binary]
        if bin_f:
            bcols = torch.cat([torch.arange(offs[f], offs[f] + bins[f]) for f in bin_f]).to(dev)
            bfeat = torch.cat([torch.full((bins[f],), f, dtype=torch.long) for f in bin_f]).to(dev)
            starts, pos = [], 0
            for f in bin_f:
                starts.append(pos)
                pos += bins[f]
            bstart = torch.cat([torch.full((bins[f],), st, dtype=torch.long) for f, st in zip(bin_f, starts)]).to(dev)
            bend = torch.cat([torch.full((bins[f],), st + bins[f] - 1, dtype=torch.long)
                              for f, st in zip(bin_f, starts)]).to(dev)
            bthr = torch.cat([torch.arange(bins[f]) for f in bin_f]).to(dev)      # threshold index within feature
            bvalid = bthr < torch.cat([torch.full((bins[f],), bins[f] - 1) for f in bin_f]).to(dev)
        NBc = int(bcols.numel()) if bin_f else 0
        # score column -> (feature, split): binary block first, then the explicit splits
        index: list[tuple[int, int]] = (list(zip(bfeat.tolist(), bthr.tolist())) if bin_f else []) + nb_rows

        # K7 device scoring (csrc/kernels/split.hip): every candidate of ``index`` is a row of one split
        # table — binary thresholds (the last one invalid) as two-segment maps, then the explicit
        # splits — scored, ranked and expanded into segment counts / impurities on the device
        use_k7 = (dev.type == "cuda" and os.environ.get("AVMI_TREE_K7", "1") != "0" and _native.C() is not None
                  and hasattr(_native.C(), "ref_split_score") and C <= 32 and max(Gmax, 2) <= 64 and len(index) > 0)
        if use_k7:
            sp_rows, seg_bytes = [], []
            for f, s_ in index:
                fs = space[f]
                if fs.binary:
                    sm, ns, valid = [0 if b <= s_ else 1 for b in range(bins[f])], 2, int(s_ < bins[f] - 1)
                else:
                    sp_ = fs.splits[s_]
                    sm, ns, valid = list(sp_.segmap), sp_.n_seg, 1
                sp_rows.append([f, offs[f], bins[f], ns, valid, len(seg_bytes)])
                seg_bytes += sm
            k7_sp = torch.tensor(sp_rows, dtype=torch.int32, device=dev)
            k7_seg = torch.tensor(seg_bytes, dtype=torch.int8, device=dev)
            k7_algo = {"entropy": 0, "giniIndex": 1, "gini": 1}.get(p.algorithm)
            use_k7 = k7_algo is not None
        # ---- roots: one histogram launch for every tree ------------------------------------------
        def rows_of(gis):
            if tree_rows is None:
                return None
            return torch.tensor([tree_rows[tree_of[g]] for g in gis], dtype=torch.long).to(dev, non_blocking=True)

        tree_of: list[int] = list(range(NT))
        hist = T.node_histogram(codes, n, labels, node, weight, bins, C, NT, rows_of(range(NT)))
        if comm.is_distributed:
            comm.all_reduce(hist)
        rc_all = hist[:, :, offs[F]].cpu()
        self.root_time = time.perf_counter() - t_grow0
        nodes: list[Node] = []
        for ti in range(NT):
            rc = rc_all[ti]
            pop = int(rc.sum())
            nodes.append(Node([], pop, float(impurity(rc.unsqueeze(0), p.algorithm)[0]),
                              (rc.double() / max(pop, 1)).tolist(), depth=0))   # depth = #predicates
        frontier = list(range(NT))   # global node indices; position = histogram slot
        while frontier:
            t0 = time.perf_counter()
            A = len(frontier)
            hist_t = hist.transpose(1, 2).double()                     # [A, TB, C]
            # ---- candidate attributes (per-tree RNG streams, frontier order) ----
            cand = np.zeros((A, F), dtype=bool)
            for a, gi in enumerate(frontier):
                cand[a, self._candidate_attrs(nodes[gi], F, rngs[tree_of[gi]])] = True
            cand_masks = torch.from_numpy(cand).to(dev)
            G2 = max(Gmax, 2)
            if use_k7:
                k = min(p.top_split_count, len(index)) if p.split_selection == "randomAmongTop" else 1
                top, topv, segc, cinfo = _native.C().ref_split_score(
                    hist.contiguous(), k7_sp, k7_seg, cand_masks.to(torch.uint8).contiguous(), k7_algo, k, G2)
            else:
                score_blocks = []
                if bin_f:
                    hb = hist_t[:, bcols, :]                                    # [A, NB, C]
                    cs = torch.cumsum(hb, 1)
                    base = torch.where((bstart > 0).view(1, -1, 1), cs[:, (bstart - 1).clamp_min(0), :],
                                       torch.zeros_like(cs))
                    left = cs - base
                    right = cs[:, bend, :] - base - left
                    bseg = torch.stack([left, right], 2)                        # [A, NB, 2, C]
                    cnt = bseg.sum(-1)
                    stat = impurity(bseg, p.algorithm)
                    wavg = (stat * cnt).sum(-1) / cnt.sum(-1).clamp_min(1)
                    ok = ((cnt > 0).sum(-1) >= 2) & bvalid.view(1, -1) & cand_masks[:, bfeat]
                    score_blocks.append(torch.where(ok, wavg, torch.full_like(wavg, math.inf)))
                for f in nb_f:
                    hb = hist_t[:, offs[f]: offs[f] + bins[f], :]               # [A, B, C]
                    seg = torch.einsum("sgb,abc->asgc", seg_tensors[f], hb)     # [A, S, G, C]
                    cnt = seg.sum(-1)
                    stat = impurity(seg, p.algorithm)
                    wavg = (stat * cnt).sum(-1) / cnt.sum(-1).clamp_min(1)     # [A, S]
                    nonempty = (cnt > 0).sum(-1) >= 2                           # a split must separate rows
                    score_blocks.append(torch.where(nonempty & cand_masks[:, f:f + 1], wavg,
                                                    torch.full_like(wavg, math.inf)))
                if not score_blocks:
                    break
                scores = torch.cat(score_blocks, 1)                             # [A, S_total]
                k = min(p.top_split_count, scores.shape[1]) if p.split_selection == "randomAmongTop" else 1
                # the k best by (score, index), as the device kernel ranks them
                top = torch.sort(scores, dim=1, stable=True).indices[:, :k]
                topv = torch.gather(scores, 1, top)
                # segment class counts of every top candidate, on the device: [A, k, Gmax', C]
                segc = torch.zeros((A, k, G2, C), dtype=torch.float64, device=dev)
                if bin_f:
                    isb = top < NBc
                    bsel = bseg[torch.arange(A, device=dev).view(-1, 1).expand(A, k), top.clamp_max(NBc - 1)]
                    segc[:, :, :2] = torch.where(isb.view(A, k, 1, 1), bsel, segc[:, :, :2])
                if nb_rows:
                    isn = top >= NBc
                    r = (top - NBc).clamp(0, len(nb_rows) - 1)
                    hpad = torch.cat([hist_t, torch.zeros((A, 1, C), dtype=hist_t.dtype, device=dev)], 1)
                    cols = splitcol[r]                                          # [A, k, Bmax]
                    hsel = torch.gather(hpad, 1, cols.view(A, -1, 1).expand(-1, -1, C)).view(A, k, Bmax, C)
                    nsel = torch.einsum("akgb,akbc->akgc", allseg[r], hsel)
                    segc[:, :, :Gmax] = torch.where(isn.view(A, k, 1, 1), nsel, segc[:, :, :Gmax])
                cinfo = impurity(segc, p.algorithm)                             # [A, k, G2]
            # ---- the ONE host copy of the level ----
            flat = torch.cat([top.double().view(-1), topv.double().view(-1), segc.round().view(-1),
                              cinfo.double().view(-1)]).cpu()
            top_h = flat[: A * k].long().view(A, k).tolist()
            topv_h = flat[A * k: 2 * A * k].view(A, k).tolist()
            o3 = 2 * A * k + A * k * G2 * C
            segc_np = flat[2 * A * k: o3].view(A, k, G2, C).numpy()
            pop_h = segc_np.sum(-1).astype(np.int64).tolist()                       # [A][k][G2]
            prob_h = (segc_np / np.maximum(segc_np.sum(-1, keepdims=True), 1)).tolist()
            cinfo_h = flat[o3:].view(A, k, G2).tolist()
            # ---- choose (randomAmongTop: per-tree RNG among the finite top-k) ----
            pick = [-1] * A
            for a in range(A):
                if k == 1:
                    pick[a] = 0 if math.isfinite(topv_h[a][0]) else -1
                else:
                    fin = [i for i in range(k) if math.isfinite(topv_h[a][i])]
                    pick[a] = rngs[tree_of[frontier[a]]].choice(fin) if fin else -1
            # ---- create children ----
            new_frontier: list[int] = []
            derived: list[tuple[int, int, list[int]]] = []   # (global child, parent slot, built sibling gis)
            max_bins = max(bins)
            max_seg = G2
            split_feat = np.full((A,), -1, dtype=np.int32)
            segmap = np.full((A, max_bins), -1, dtype=np.int16)
            child_of = np.full((A, max_seg), -1, dtype=np.int32)
            for a, gi in enumerate(frontier):
                nd = nodes[gi]
                if pick[a] < 0:
                    nd.stopped = True
                    continue
                f, s = index[top_h[a][pick[a]]]
                fs = space[f]
                if fs.binary:
                    sm = [0 if b <= s else 1 for b in range(fs.n_bins)]
                    o = fs.field.ordinal
                    if fs.kind == "num":
                        pv = fs.pred_value(fs.points[s])
                        preds = [f"{o} le {pv}", f"{o} gt {pv}"]
                    else:
                        card = fs.field.cardinality
                        preds = [f"{o} in {':'.join(card[: s + 1])}", f"{o} in {':'.join(card[s + 1:])}"]
                    ng = 2
                else:
                    sp = fs.splits[s]
                    sm, preds, ng = sp.segmap, sp.predicates, sp.n_seg
                pk = pick[a]
                nd.feature, nd.split, nd.segmap = f, s, list(sm)
                nd.children = []
                split_feat[a] = f
                segmap[a, : len(sm)] = sm
                kids = []
                for g in range(ng):
                    pop = pop_h[a][pk][g]
                    if pop == 0:
                        nd.children.append(-1)
                        continue
                    info = cinfo_h[a][pk][g]                         # segment impurity from the device
                    depth = nd.depth + 1   # parentPredicates.size() + 1 (DecisionTreeBuilder.java:606)
                    stop = self._should_stop(pop, info, nd.info, depth) or info == 0.0
                    child = Node(nd.predicates + [preds[g]], pop, info, prob_h[a][pk][g],
                                 depth, stopped=stop, used_attrs=nd.used_attrs | {f})
                    ci = len(nodes)
                    nodes.append(child)
                    tree_of.append(tree_of[gi])
                    nd.children.append(ci)
                    kids.append((g, ci, pop, stop))
                # histogram subtraction: when every row of the parent lands in a frontier child, the
                # most populated child's histogram is the parent's minus its built siblings'
                live = [kk for kk in kids if not kk[3]]
                whole = sum(kk[2] for kk in kids) == nd.population and len(live) == len(kids) and len(live) >= 2
                heavy = max(live, key=lambda kk: kk[2])[1] if whole else -1
                for g, ci, _, stop in kids:
                    if not stop and ci != heavy:
                        child_of[a, g] = len(new_frontier)
                        new_frontier.append(ci)
                if heavy >= 0:
                    derived.append((heavy, a, [ci for _, ci, _, _ in live if ci != heavy]))
            # derived children take the ids after the built ones: the histogram pass skips their rows
            slot = {ci: j for j, ci in enumerate(new_frontier)}
            m = len(new_frontier)
            for j, (ci, a, _) in enumerate(derived):
                g = nodes[frontier[a]].children.index(ci)
                child_of[a, g] = m + j
            T.tree_assign(codes, n, node, torch.from_numpy(split_feat).to(dev), torch.from_numpy(segmap).to(dev),
                          torch.from_numpy(child_of).to(dev))
            if new_frontier or derived:
                hs = T.node_histogram(codes, n, labels, node, weight, bins, C, m,   # built children only
                                      rows_of(new_frontier))
                if comm.is_distributed:
                    comm.all_reduce(hs)
                parts = [hs]
                if derived:
                    pa = torch.tensor([a for _, a, _ in derived], device=dev)
                    dh = hist[pa].clone()
                    jj = [j for j, (_, _, sibs) in enumerate(derived) for _ in sibs]
                    ss = [slot[sg] for _, _, sibs in derived for sg in sibs]
                    if jj:   # parent minus its built siblings, one scatter for the level
                        dh.index_add_(0, torch.tensor(jj, device=dev), hs[torch.tensor(ss, device=dev)], alpha=-1)
                    parts.append(dh)
                hist = torch.cat(parts) if len(parts) > 1 else hs
            frontier = new_frontier + [ci for ci, _, _ in derived]
            self.level_times.append(time.perf_counter() - t0)
        # ---- split the node list into one DecisionTree per tree (children re-indexed) ----
        per_tree: list[list[int]] = [[] for _ in range(NT)]
        for g, ti in enumerate(tree_of):
            per_tree[ti].append(g)
        out = []
        for ti in range(NT):
            gids = per_tree[ti]
            local = {g: j for j, g in enumerate(gids)}
            tn = []
            for g in gids:
                nd = nodes[g]
                nd.children = [local[c] if c >= 0 else -1 for c in nd.children]
                tn.append(nd)
            out.append(DecisionTree(tn, space, list(cls)))
        return out


# ================================================================================================
# inference (ModelPredictor / DecisionTreeModel / EnsemblePredictiveModel)
# ================================================================================================
def flatten_forest(trees: Sequence[DecisionTree], device, weights: Sequence[float] | None = None,
                   value_fn=None) -> dict:
    """Concatenate trees into the flat int32/int16/float32 arrays of ``tree_predict``.  All trees
    must share one split space (same encoded code rows)."""
    feat, seg_base, child_base, leaf_idx, child, segrows, values, roots = [], [], [], [], [], [], [], []
    max_bins = max((fs.n_bins for fs in trees[0].space), default=1)
    for tr in trees:
        base = len(feat)
        roots.append(base)
        for nd in tr.nodes:
            if nd.is_leaf or not nd.children:
                feat.append(-1)
                seg_base.append(0)
                child_base.append(0)
            else:
                feat.append(nd.feature)
                seg_base.append(len(segrows))
                row = [-1] * max_bins
                for b, g in enumerate(nd.segmap):
                    row[b] = g
                segrows.append(row)
                child_base.append(len(child))
                child.extend([c + base if c >= 0 else -1 for c in nd.children])
            leaf_idx.append(len(values))
            values.append(value_fn(nd) if value_fn else nd.class_pr)
    if not segrows:
        segrows = [[-1] * max_bins]
    if not child:
        child = [-1]
    dev = torch.device(device)
    out = {
        "feat": torch.tensor(feat, dtype=torch.int32, device=dev),
        "seg_base": torch.tensor(seg_base, dtype=torch.int32, device=dev),
        "segmap": torch.tensor(segrows, dtype=torch.int16, device=dev),
        "child_base": torch.tensor(child_base, dtype=torch.int32, device=dev),
        "child": torch.tensor(child, dtype=torch.int32, device=dev),
        "leaf_idx": torch.tensor(leaf_idx, dtype=torch.int32, device=dev),
        "values": torch.tensor(values, dtype=torch.float32, device=dev),
        "tree_root": torch.tensor(roots, dtype=torch.int32, device=dev),
    }
    if weights is not None:
        out["tree_w"] = torch.tensor(list(weights), dtype=torch.float32, device=dev)
    bn = _binary_nodes(trees)
    if bn is not None:
        out["bin_nodes"] = torch.tensor(bn, dtype=torch.int64).to(torch.int32).to(dev)
    return out


def _binary_nodes(trees: Sequence[DecisionTree]) -> list | None:
    """Packed [K, 2] records of ``forest_predict_bin_kernel`` when every internal node is a
    threshold split (segments 0..0 1..1 over the feature's bins, two children) and the forest fits
    the record fields (features < 255, bins <= 255, < 65536 nodes); None otherwise."""
    recs = []
    for tr in trees:
        base = len(recs)
        for nd in tr.nodes:
            if nd.is_leaf or not nd.children:
                recs.append([0xFF, 0])
                continue
            nb = tr.space[nd.feature].n_bins
            sm = list(nd.segmap)
            thr = sum(1 for g in sm if g == 0) - 1
            if (len(nd.children) != 2 or min(nd.children) < 0 or nd.feature >= 255 or nb > 255 or thr < 0
                    or sm != [0] * (thr + 1) + [1] * (len(sm) - thr - 1) or len(sm) != nb):
                return None
            left, right = nd.children[0] + base, nd.children[1] + base
            recs.append([nd.feature | (thr << 8) | (nb << 16), left | (right << 16)])
    if len(recs) > 65535:
        return None
    # int32 view of the unsigned record words
    return [[x - (1 << 32) if x >= (1 << 31) else x for x in r] for r in recs]


class TreeEnsemble:
    """Prediction over one or more trees (DecisionTreeModel; EnsemblePredictiveModel when more than
    one tree: weighted majority vote, optional minimum odds ratio -> ambiguous)."""

    def __init__(self, trees: Sequence[DecisionTree], weights: Sequence[float] | None = None):
        self.trees = list(trees)
        self.weights = list(weights) if weights is not None else None
        self._flat: dict | None = None

    @property
    def class_values(self) -> list[str]:
        return self.trees[0].class_values

    def encode(self, t: Table) -> torch.Tensor:
        return encode_for_tree(self.trees[0].space, t)

    def flat(self, device) -> dict:
        if self._flat is None or self._flat["feat"].device != torch.device(device):
            self._flat = flatten_forest(self.trees, device, self.weights)
        return self._flat

    def predict_proba(self, t: Table, codes: torch.Tensor | None = None) -> torch.Tensor:
        codes = self.encode(t) if codes is None else codes
        out = T.tree_predict(codes, t.n, self.flat(t.device), mode=0)
        tw = sum(self.weights) if self.weights else len(self.trees)
        return out / tw

    def predict_votes(self, t: Table, codes: torch.Tensor | None = None) -> torch.Tensor:
        codes = self.encode(t) if codes is None else codes
        return T.tree_predict(codes, t.n, self.flat(t.device), mode=1)

    def predict(self, t: Table, min_odds_ratio: float | None = None) -> torch.Tensor:
        """Class index per row; with an ensemble, majority vote (-1 = ambiguous when the top/second
        vote ratio is below ``min_odds_ratio``)."""
        if len(self.trees) == 1:
            return self.predict_proba(t).argmax(1)
        votes = self.predict_votes(t)
        top2 = torch.topk(votes, min(2, votes.shape[1]), dim=1)
        pred = top2.indices[:, 0]
        if min_odds_ratio is not None and votes.shape[1] > 1:
            ratio = top2.values[:, 0] / top2.values[:, 1].clamp_min(1e-9)
            pred = torch.where(ratio < min_odds_ratio, torch.full_like(pred, -1), pred)
        return pred


# ================================================================================================
# random forest (P/supv/rf.py parity: sklearn-style RF, and R/rafo.sh reference RF)
# ================================================================================================
class RandomForest:
    def __init__(self, schema: FeatureSchema, n_trees: int = 10, params: TreeParams | None = None,
                 max_features: str | int = "sqrt", comm: Comm | None = None, tree_parallel: bool = False):
        self.schema = schema
        self.n_trees = n_trees
        base = params or TreeParams(binary=True, stopping="maxDepth", max_depth=8,
                                    sub_sampling="withReplace", attr_selection="randomAll")
        self.params = base
        self.max_features = max_features
        self.comm = comm
        self.tree_parallel = tree_parallel
        self.trees: list[DecisionTree] = []

    def _k(self, F: int) -> int:
        mf = self.max_features
        if isinstance(mf, int):
            return max(1, min(F, mf))
        if mf == "sqrt":
            return max(1, int(math.sqrt(F)))
        if mf == "log2":
            return max(1, int(math.log2(F)))
        if mf in ("all", None, "auto"):
            return F
        return max(1, int(float(mf) * F))

    def fit(self, t: Table) -> "RandomForest":
        comm = self.comm or get_comm()
        # tree-parallel ranks hold every row; data-parallel ranks bin on globally gathered samples
        space = build_split_space(self.schema, t, binary=self.params.binary, max_bins=self.params.max_bins,
                                  comm=None if self.tree_parallel else comm)
        codes = encode_for_tree(space, t)
        import copy
        my_trees = range(self.n_trees)
        if self.tree_parallel and comm.is_distributed:
            my_trees = range(comm.rank, self.n_trees, comm.world)
        trees = []
        if self.params.binary and self.params.attr_selection != "notUsedYet":
            # all trees at once, rows resident and partitioned in HBM (models/forest.py)
            from .forest import ForestBuilder
            p = copy.copy(self.params)
            p.random_attr_count = self._k(len(space))
            fb = ForestBuilder(self.schema, self.n_trees, p, comm=_LocalComm() if self.tree_parallel else comm)
            trees = fb.fit(t, space=space, codes=codes, tree_ids=list(my_trees))
            self.build_stats = fb.stats
            my_trees = []
        if list(my_trees):
            # the reference's split semantics (multi-way numeric, categorical partitions,
            # notUsedYet): every tree of this rank grown together by the level-wise builder
            p = copy.copy(self.params)
            p.random_attr_count = self._k(len(space))
            b = DecisionTreeBuilder(self.schema, p, comm=_LocalComm() if self.tree_parallel else comm,
                                    space=space)
            trees = b.fit_many(t, [self.params.seed * 7919 + i for i in my_trees], codes=codes)
            self.build_stats = {"levels": len(b.level_times), "seconds": sum(b.level_times),
                                "root_seconds": getattr(b, "root_time", None),
                                "level_seconds": [round(x, 5) for x in b.level_times]}
        if self.tree_parallel and comm.is_distributed:
            states = comm.all_gather_object([tr.state() for tr in trees])
            allt = {}
            for r, sts in enumerate(states):
                for j, st in enumerate(sts):
                    allt[r + j * comm.world] = DecisionTree.from_state(st, self.schema)
            trees = [allt[i] for i in sorted(allt)]
        self.trees = trees
        return self

    def ensemble(self) -> TreeEnsemble:
        return TreeEnsemble(self.trees)

    def predict_proba(self, t: Table) -> torch.Tensor:
        return self.ensemble().predict_proba(t)

    def predict(self, t: Table) -> torch.Tensor:
        return self.predict_proba(t).argmax(1)


class _LocalComm:
    """Single-rank stand-in used for tree-parallel forests (each rank grows whole trees)."""
    is_distributed = False
    world = 1
    rank = 0

    def all_reduce(self, t, op="sum"):
        return t


# ================================================================================================
# gradient boosted trees (P/supv/gbt.py parity: sklearn GradientBoostingClassifier, deviance loss)
# ================================================================================================
@dataclass
class GBTParams:
    n_estimators: int = 120
    learning_rate: float = 0.12
    max_depth: int = 3
    min_samples_leaf: int = 1
    subsample: float = 1.0
    l2: float = 0.0
    max_bins: int = 64
    seed: int = 0


@dataclass
class _RegNode:
    value: float
    feature: int = -1
    threshold_bin: int = -1
    children: list[int] = field(default_factory=list)
    depth: int = 0


class GradientBoostedTrees:
    """Histogram GBT: per stage one regression tree per class on (g, h) with Newton leaves.

    Device-resident rounds (csrc/kernels/gbt.hip): every tree of depth D lives in static heap
    arrays (slot s of a level has children 2s / 2s+1), so a tree build is a fixed sequence of launches
    — per level one ``node_grad_hist`` pass (exact fixed-point sums; from level 1 only the left
    children, right = parent - left), the threshold scan as batched tensor math, and one
    ``gbt_assign`` pass that also adds ``lr * leaf value`` to the raw scores of rows reaching a
    leaf (no separate inference pass).  On a GPU that sequence is captured once in a HIP graph and
    replayed per tree; the per-round gradient kernel computes the previous round's training loss on
    the device.  Nothing is copied to the host until the fit ends (one copy of every tree), except
    when per-round checkpoints are written."""

    def __init__(self, schema: FeatureSchema, params: GBTParams | None = None, comm: Comm | None = None,
                 recovery=None):
        self.schema = schema
        self.p = params or GBTParams()
        self.comm = comm
        self.recovery = recovery          # per-round checkpoint / resume (utils/resilience)
        self.space: list[FeatureSplits] | None = None
        self.stages: list[list[DecisionTree]] = []
        self.init: torch.Tensor | None = None
        self.n_classes = 2
        self.train_loss: list[float] = []
        self.graph_used = False

    # ------------------------------------------------------------------------------------------
    def _build_tree(self, st: dict, k: int) -> None:
        """One regression tree for class ``k`` from the gradients in st["g"][k], st["h"][k]: writes
        the heap arrays st["feat"], st["thr"], st["val"] and updates the raw scores.  Static shapes
        and device-only work (graph-capturable)."""
        p = self.p
        comm = self.comm or get_comm()
        codes, n, bins, sc = st["codes"], st["n"], st["bins"], self._scan
        node, g, h = st["node"], st["g"][k], st["h"][k]
        feat, thr, val = st["feat"], st["thr"], st["val"]
        tb_tot = st["offs"][-1]
        feat.fill_(-1)
        thr.zero_()
        val.zero_()
        node[:n] = 0

        def grad_hist(A, even):
            hh = T.node_grad_histogram(codes, n, node, g, h, bins, A, even_only=even, bins_d=st["bins_d"],
                                       offs_d=st["offs_d"], tot_slot=tb_tot)
            if comm.is_distributed:
                comm.all_reduce(hh)
            return hh

        D = p.max_depth
        if codes.is_cuda:
            self._build_tree_device(st, k, grad_hist_raw=lambda A, even: self._grad_hist_raw(st, comm, g, h, A, even))
            return
        hist = grad_hist(1, False)
        for lvl in range(D):
            A = 1 << lvl
            hb, hc = A - 1, 2 * A - 1
            # node total: feature 0's bins + the slot of rows missing feature 0 (tot_slot)
            tot = hist[:, : bins[0], :].sum(1) + hist[:, tb_tot, :]
            G, H = tot[:, 0], tot[:, 1]
            if lvl == 0:
                val[0:1] = -G / (H + p.l2).clamp_min(1e-12)
            parent = G * G / (H + p.l2).clamp_min(1e-12)
            cs = torch.cumsum(hist[:, : sc["nb"], :].transpose(1, 2).contiguous(), 2).transpose(1, 2)  # [A, NB, 2]
            base = torch.where((sc["start"] > 0).view(1, -1, 1), cs[:, (sc["start"] - 1).clamp_min(0), :],
                               torch.zeros_like(cs))
            left = cs - base
            right = cs[:, sc["end"], :] - base - left
            gl, hl, gr, hr = left[..., 0], left[..., 1], right[..., 0], right[..., 1]
            gain = gl * gl / (hl + p.l2).clamp_min(1e-12) + gr * gr / (hr + p.l2).clamp_min(1e-12) \
                - parent.unsqueeze(1)
            ok = (hl > 1e-12) & (hr > 1e-12) & sc["valid"].view(1, -1)
            gain = torch.where(ok, gain, torch.full_like(gain, -math.inf))
            best_gain, best_pos = gain.max(1)
            bi = best_pos.view(-1, 1)
            cgl, chl = gl.gather(1, bi)[:, 0], hl.gather(1, bi)[:, 0]
            cgr, chr_ = gr.gather(1, bi)[:, 0], hr.gather(1, bi)[:, 0]
            split = torch.isfinite(best_gain) & (best_gain > 1e-12)
            feat[hb:hb + A] = torch.where(split, sc["feat"][best_pos], torch.full_like(best_pos, -1)).int()
            thr[hb:hb + A] = sc["thr"][best_pos].int()
            vl = -cgl / (chl + p.l2).clamp_min(1e-12)
            vr = -cgr / (chr_ + p.l2).clamp_min(1e-12)
            val[hc:hc + 2 * A] = torch.where(split.view(-1, 1), torch.stack([vl, vr], 1),
                                             torch.zeros_like(torch.stack([vl, vr], 1))).view(-1)
            last = lvl + 1 == D
            T.gbt_assign(codes, n, node, feat, thr, val, st["bins_t"], lvl, last, p.learning_rate, st["F"], k)
            if last:
                break
            if st["subtract"]:
                hl_ = grad_hist(A, True)                     # left children (even slots) only
                hist = torch.stack([hl_, hist - hl_], 1).view(2 * A, *hist.shape[1:])
            else:
                hist = grad_hist(2 * A, False)

    @staticmethod
    def _grad_hist_raw(st, comm, g, h, A, even):
        hh = T.node_grad_histogram(st["codes"], st["n"], st["node"], g, h, st["bins"], A, even_only=even,
                                   bins_d=st["bins_d"], offs_d=st["offs_d"], raw=True, tot_slot=st["offs"][-1])
        if comm.is_distributed:
            comm.all_reduce(hh)               # exact int64 fixed point
        return hh

    def _build_tree_device(self, st: dict, k: int, grad_hist_raw) -> None:
        """GPU levels: raw fixed-point histograms -> ONE split-scoring launch per level
        (gbt_split_kernel: sibling subtraction, prefix sums, gains, argmax, heap writes) -> the
        assign / leaf-update launch.  Same results as the tensor scan of ``_build_tree``."""
        p = self.p
        codes, n, sc = st["codes"], st["n"], self._scan
        node, feat, thr, val = st["node"], st["feat"], st["thr"], st["val"]
        tot = st["offs"][-1]
        D = p.max_depth
        hist, parent, left = grad_hist_raw(1, False), None, None
        for lvl in range(D):
            A = 1 << lvl
            last = lvl + 1 == D
            keep = st["subtract"] and not last          # this level's histogram is the next one's parent
            out_h = torch.empty((A, hist.shape[1] if hist is not None else left.shape[1], 2), dtype=torch.int64,
                                device=codes.device) if keep else None
            T.gbt_split(hist, parent, left, out_h, A, tot, sc, p.l2, lvl, feat, thr, val)
            T.gbt_assign(codes, n, node, feat, thr, val, st["bins_t"], lvl, last, p.learning_rate, st["F"], k)
            if last:
                break
            if st["subtract"]:
                hist, parent, left = None, out_h, grad_hist_raw(A, True)
            else:
                hist, parent, left = grad_hist_raw(2 * A, False), None, None

    def _trees_from_heaps(self, feat, thr, val) -> list[list[DecisionTree]]:
        """Host DecisionTrees from the [R, K, heap] arrays (nodes reachable from the root only)."""
        R, K, Hn = feat.shape
        bins = [fs.n_bins for fs in self.space]
        fl, tl, vl = feat.tolist(), thr.tolist(), val.tolist()
        seg_cache: dict[tuple[int, int], list[int]] = {}
        stages = []
        for r in range(R):
            stage = []
            for k in range(K):
                fr, trr, vr = fl[r][k], tl[r][k], vl[r][k]
                nodes: list[Node] = []
                idx_of = {0: 0}
                order = [0]
                nodes.append(Node([], 0, 0.0, [vr[0]], depth=0))
                q = 0
                while q < len(order):
                    i = order[q]
                    q += 1
                    f = fr[i]
                    if f < 0 or 2 * i + 2 >= Hn:
                        continue
                    # heap children of i: level l = floor(log2(i + 1)); slot s = i - (2^l - 1)
                    lvl = (i + 1).bit_length() - 1
                    s = i - ((1 << lvl) - 1)
                    cl = (2 << lvl) - 1 + 2 * s
                    nd = nodes[idx_of[i]]
                    th = trr[i]
                    sm = seg_cache.get((f, th))
                    if sm is None:
                        sm = seg_cache[(f, th)] = [0 if b <= th else 1 for b in range(bins[f])]
                    nd.feature, nd.split, nd.segmap = f, th, sm
                    nd.children = []
                    for c in (cl, cl + 1):
                        idx_of[c] = len(nodes)
                        nd.children.append(len(nodes))
                        nodes.append(Node([], 0, 0.0, [vr[c]], depth=nd.depth + 1))
                        order.append(c)
                stage.append(DecisionTree(nodes, self.space, ["value"]))
            stages.append(stage)
        return stages

    def fit(self, t: Table) -> "GradientBoostedTrees":
        import time as _time
        marks = [("start", _time.perf_counter())]
        comm = self.comm or get_comm()
        p = self.p
        if p.max_depth < 1 or p.max_depth > 16:
            raise ValueError("GBT max_depth must be in 1..16")
        self.space = build_split_space(self.schema, t, binary=True, max_bins=p.max_bins, comm=comm)
        codes = encode_for_tree(self.space, t)
        # + one slot: rows missing feature 0 (feature 0's bins + it = the node total)
        bins = [fs.n_bins for fs in self.space] + [1]
        n, dev = t.n, t.device
        ld = codes.shape[1]
        fb = bins[:-1]
        offs0 = list(itertools.accumulate([0] + fb[:-1]))
        offs = list(itertools.accumulate([0] + bins[:-1]))
        self._scan = {
            "nb": sum(fb),
            "feat": torch.cat([torch.full((b,), f, dtype=torch.long) for f, b in enumerate(fb)]).to(dev),
            "thr": torch.cat([torch.arange(b) for b in fb]).to(dev),
            "start": torch.cat([torch.full((b,), o, dtype=torch.long) for o, b in zip(offs0, fb)]).to(dev),
            "end": torch.cat([torch.full((b,), o + b - 1, dtype=torch.long) for o, b in zip(offs0, fb)]).to(dev),
            "valid": torch.cat([torch.arange(b) < b - 1 for b in fb]).to(dev),
        }
        sc = self._scan
        sc.update({"feat_i": sc["feat"].int(), "thr_i": sc["thr"].int(), "start_i": sc["start"].int(),
                   "end_i": sc["end"].int(), "valid_u8": sc["valid"].to(torch.uint8)})
        C = t.n_classes
        self.n_classes = C
        y = t.labels[:n].long().clamp_max(C - 1)
        K = 1 if C == 2 else C
        cnt = torch.bincount(y, minlength=C).double()
        if comm.is_distributed:
            comm.all_reduce(cnt)
        n_total = float(cnt.sum())
        prior = (cnt / cnt.sum()).clamp(1e-12, 1 - 1e-12)
        self.init = (torch.log(prior[1] / prior[0]).view(1) if K == 1 else torch.log(prior)).float()
        Hn = (2 << p.max_depth) - 1
        R = p.n_estimators
        missing = bool((codes[:, :n] == MISSING).any()) if n else False
        if comm.is_distributed:
            mt = torch.tensor([float(missing)])
            comm.all_reduce(mt, "max")
            missing = bool(mt[0] > 0)
        y8 = torch.zeros(ld, dtype=torch.uint8, device=dev)
        y8[:n] = y.to(torch.uint8)
        st = {
            "codes": codes, "n": n, "bins": bins, "offs": offs,
            "bins_d": torch.tensor(bins, dtype=torch.int32, device=dev),
            "offs_d": torch.tensor(offs, dtype=torch.int32, device=dev),
            "bins_t": torch.tensor(fb, dtype=torch.int32, device=dev),
            "node": torch.full((ld,), -1, dtype=torch.int32, device=dev),
            "g": torch.zeros((K, ld), dtype=torch.float32, device=dev),
            "h": torch.zeros((K, ld), dtype=torch.float32, device=dev),
            "feat": torch.full((Hn,), -1, dtype=torch.int32, device=dev),
            "thr": torch.zeros(Hn, dtype=torch.int32, device=dev),
            "val": torch.zeros(Hn, dtype=torch.float64, device=dev),
            "F": self.init.to(dev).view(1, K).expand(ld, K).contiguous(),
            "subtract": not missing,
        }
        feat_all = torch.full((R, K, Hn), -1, dtype=torch.int32, device=dev)
        thr_all = torch.zeros((R, K, Hn), dtype=torch.int32, device=dev)
        val_all = torch.zeros((R, K, Hn), dtype=torch.float64, device=dev)
        loss_all = torch.zeros(R + 1, dtype=torch.float64, device=dev)
        rate32 = 0xFFFFFFFF if p.subsample >= 1.0 else int(max(0.0, p.subsample) * 4294967296.0)
        # one boosting round = one resumable iteration.  The checkpoint is REPLICATED (rank 0 writes
        # the trees and the global loss sums), so a job resumes at any world size: each rank replays
        # the restored trees over its own rows to rebuild its raw scores (same gbt_assign launches
        # in the same order as the original rounds: bit-identical F).
        from ..utils.hipgraph import capturing
        from ..utils.resilience import IterationLoop
        lp = IterationLoop("gbt", self.recovery, comm, device=dev)
        r0, ck, meta = lp.restore(dev)
        if ck is not None:
            if tuple(ck["feat"].shape[1:]) != (K, Hn) or r0 > R:
                raise ValueError(f"gbt checkpoint shape {tuple(ck['feat'].shape)} does not match this model "
                                 f"(rounds {R}, classes {K}, heap {Hn})")
            feat_all[:r0], thr_all[:r0], val_all[:r0] = ck["feat"].to(dev), ck["thr"].to(dev), ck["val"].to(dev)
            if comm.rank == 0:                          # global sums: the final all-reduce adds zeros elsewhere
                loss_all[:r0] = ck["loss"].to(dev)[:r0]
            self._replay_scores(st, feat_all, thr_all, val_all, r0)
        use_graph = (dev.type == "cuda" and not comm.is_distributed and not lp.enabled
                     and os.environ.get("AVMI_GBT_GRAPH", "1") != "0")
        graphs: dict[int, Any] = {}

        def tree(k):
            if not use_graph:
                self._build_tree(st, k)
                return
            if k not in graphs:
                # warm up on a side stream (allocator pools, kernel selection), then capture
                s_ = torch.cuda.Stream(device=dev)
                s_.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(s_):
                    Fsave = st["F"].clone()
                    self._build_tree(st, k)
                    st["F"].copy_(Fsave)
                torch.cuda.current_stream(dev).wait_stream(s_)
                gr = torch.cuda.CUDAGraph()
                with capturing(gr, device=dev):      # no allocator flush per fit (utils/hipgraph.py)
                    self._build_tree(st, k)
                graphs[k] = gr
            graphs[k].replay()

        seed_base = (p.seed * 0x9E3779B97F4A7C15 + 0x632BE59BD9B4E019) & 0x7FFFFFFFFFFFFFFF
        timing = os.environ.get("AVMI_GBT_TIMING") == "1" and dev.type == "cuda"
        if timing:
            torch.cuda.synchronize(dev)
            marks.append(("setup", _time.perf_counter()))
        # Without subsampling a round does not depend on its index on the host side (the gradient's
        # subsample seed is unused), so the WHOLE round — gradients, every class's tree, the heap
        # copies into round slot rnd_dev (a device counter) and the loss — is one graph replayed
        # once per round: 1 host launch per round instead of ~5 (launch-bound at 64 k rows: the
        # fit's time follows host scheduling noise otherwise).  The first round runs eagerly
        # (warm-up), the capture records without executing.
        round_graph = None
        if use_graph and rate32 == 0xFFFFFFFF and R - r0 >= 3 and os.environ.get("AVMI_GBT_ROUND_GRAPH", "1") != "0":
            rnd_dev = torch.full((1,), r0, dtype=torch.long, device=dev)
            loss_slot = torch.zeros(1, dtype=torch.float64, device=dev)

            def round_body():
                loss_slot.zero_()
                for k in range(K):
                    T.gbt_grad(st["F"], k, y8, n, t.row_offset, seed_base, rate32, st["g"][k], st["h"][k],
                               loss_slot if k == 0 else None)
                for k in range(K):
                    self._build_tree(st, k)
                    feat_all[:, k].index_copy_(0, rnd_dev, st["feat"].view(1, Hn))
                    thr_all[:, k].index_copy_(0, rnd_dev, st["thr"].view(1, Hn))
                    val_all[:, k].index_copy_(0, rnd_dev, st["val"].view(1, Hn))
                loss_all.index_copy_(0, rnd_dev, loss_slot)
                rnd_dev.add_(1)

            with lp.step(r0, nbytes=float(codes.numel()) * p.max_depth):
                round_body()
            if timing:
                torch.cuda.synchronize(dev)
                marks.append(("round0", _time.perf_counter()))
            round_graph = torch.cuda.CUDAGraph()
            with capturing(round_graph, device=dev):
                round_body()
            if timing:
                torch.cuda.synchronize(dev)
                marks.append(("capture", _time.perf_counter()))
            for rnd in range(r0 + 1, R):
                with lp.step(rnd, nbytes=float(codes.numel()) * p.max_depth):
                    round_graph.replay()
        for rnd in range(r0, R if round_graph is None else r0):
            with lp.step(rnd, nbytes=float(codes.numel()) * p.max_depth):
                rseed = (seed_base ^ (rnd * 0xD1B54A32D192ED03)) & 0x7FFFFFFFFFFFFFFF
                for k in range(K):       # all gradients from the round's starting scores
                    T.gbt_grad(st["F"], k, y8, n, t.row_offset, rseed, rate32, st["g"][k], st["h"][k],
                               loss_all[rnd:rnd + 1] if k == 0 else None)
                for k in range(K):
                    tree(k)
                    feat_all[rnd, k].copy_(st["feat"])
                    thr_all[rnd, k].copy_(st["thr"])
                    val_all[rnd, k].copy_(st["val"])
            if lp.enabled:
                gl = loss_all[:rnd + 1].clone()
                if comm.is_distributed:
                    comm.all_reduce(gl)
                lp.commit(rnd, {"feat": feat_all[:rnd + 1], "thr": thr_all[:rnd + 1], "val": val_all[:rnd + 1],
                                "loss": gl}, {"rows": n_total})
        self.graph_used = bool(graphs) or round_graph is not None
        if timing:
            torch.cuda.synchronize(dev)
            marks.append(("rounds", _time.perf_counter()))
        self.train_loss = self._losses(loss_all, R, st, y8, n, t, n_total, comm)
        self.stages = self._trees_from_heaps(feat_all.cpu(), thr_all.cpu(), val_all.cpu())
        self._flat = None
        if timing:
            marks.append(("trees", _time.perf_counter()))
            import sys as _sys
            _sys.stderr.write("[gbt_timing] " + " ".join(f"{a}={b - marks[i][1]:.4f}" for i, (a, b) in
                                                         enumerate(marks[1:])) + "\n")
        return self

    def _replay_scores(self, st: dict, feat_all, thr_all, val_all, rounds: int) -> None:
        """Raw scores of this rank's rows after ``rounds`` restored rounds: every tree's levels
        re-run through ``gbt_assign`` exactly as the round that built it ran them."""
        n, D, lr = st["n"], self.p.max_depth, self.p.learning_rate
        K = st["F"].shape[1]
        for rnd in range(rounds):
            for k in range(K):
                st["node"][:n] = 0
                for lvl in range(D):
                    T.gbt_assign(st["codes"], n, st["node"], feat_all[rnd, k], thr_all[rnd, k], val_all[rnd, k],
                                 st["bins_t"], lvl, lvl + 1 == D, lr, st["F"], k)

    def _losses(self, loss_all, upto, st, y8, n, t, n_total, comm) -> list[float]:
        """train_loss[r] = mean deviance after round r: round r+1's gradient pass measured it; the
        last one is measured here.  One host copy."""
        last = torch.zeros(1, dtype=torch.float64, device=loss_all.device)
        K = st["F"].shape[1]
        gs = torch.zeros_like(st["g"][0])
        T.gbt_grad(st["F"], 0, y8, n, t.row_offset, 0, 0xFFFFFFFF, gs, torch.zeros_like(gs), last)
        tot = torch.cat([loss_all[1:upto], last])
        if comm.is_distributed:
            comm.all_reduce(tot)
        return (tot / max(n_total, 1.0)).tolist()

    def decision_function(self, t: Table) -> torch.Tensor:
        codes = encode_for_tree(self.space, t)
        K = 1 if self.n_classes == 2 else self.n_classes
        F = self.init.to(t.device).view(1, K).expand(t.n, K).clone()
        for k in range(K):
            trees = [st[k] for st in self.stages]
            if not trees:
                continue
            flat = flatten_forest(trees, t.device, value_fn=lambda nd: nd.class_pr)
            F[:, k] += self.p.learning_rate * T.tree_predict(codes, t.n, flat, mode=0)[:, 0]
        return F

    def predict_proba(self, t: Table) -> torch.Tensor:
        F = self.decision_function(t)
        if F.shape[1] == 1:
            p1 = torch.sigmoid(F[:, 0])
            return torch.stack([1 - p1, p1], 1)
        return torch.softmax(F, 1)

    def predict(self, t: Table) -> torch.Tensor:
        return self.predict_proba(t).argmax(1)
