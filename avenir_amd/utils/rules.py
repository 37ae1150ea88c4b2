"""Rule expressions over delimited records, evaluated column-wise on tensors.

Reference: ``J/util/RuleExpression.java:51-56`` (``cond > consequent``, split on the first '>'),
which extends chombo's ``AttributeFilter`` (conjunction of ``<ordinal> <op> <value>`` predicates;
chombo is not part of the reference tree, so the predicate grammar below — operators ``eq ne gt ge
lt le in notIn``, optional ``int:/double:/string:`` value type tags as in R/ovsa.properties
``pro.select.filter=8 eq int:1``, ``in`` value lists joined by ':' — is the documented
re-statement, parity unpinned).  The conjunct separator is configurable (``rue.cond.delim``,
``RuleEvaluator.java:100-115``); default ``" and "``.

Evaluation is vectorised: every referenced column is converted once into a float tensor (NaN when
not numeric) and a dictionary-code tensor, and each predicate is one tensor comparison, so a rule
costs O(#predicates) tensor ops over all records instead of a per-record interpreter.
"""
from __future__ import annotations

import math
import re
from dataclasses import dataclass, field
from typing import Sequence

import torch

_OPS = ("eq", "ne", "gt", "ge", "lt", "le", "in", "notIn", "notin")
_TYPES = ("int", "long", "double", "float", "string", "str", "categorical")


def _num(s: str) -> float | None:
    try:
        return float(s)
    except ValueError:
        return None


@dataclass
class Predicate:
    ordinal: int
    op: str
    values: list[str]
    numeric: bool

    @classmethod
    def parse(cls, text: str) -> "Predicate":
        parts = text.strip().split(None, 2)
        if len(parts) != 3 or parts[1] not in _OPS:
            raise ValueError(f"bad predicate {text!r}: expected '<ordinal> <op> <value>' with op in {_OPS}")
        ordn, op, val = int(parts[0]), parts[1], parts[2].strip()
        typ = None
        m = re.match(r"^(%s):(.*)$" % "|".join(_TYPES), val)
        if m:
            typ, val = m.group(1), m.group(2)
        vals = val.split(":") if op in ("in", "notIn", "notin") else [val]
        numeric = typ in ("int", "long", "double", "float") or (typ is None and all(_num(v) is not None for v in vals))
        return cls(ordn, "notIn" if op == "notin" else op, vals, numeric)


@dataclass
class RuleExpression:
    predicates: list[Predicate]
    consequent: str | None = None
    text: str = ""

    @classmethod
    def create_rule(cls, rule: str, cond_delim: str = " and ") -> "RuleExpression":
        """``cond > consequent`` (split on the first '>')."""
        if ">" in rule:
            cond, cons = rule.split(">", 1)
            cons = cons.strip()
        else:
            cond, cons = rule, None
        return cls.from_condition(cond, cond_delim, cons)

    @classmethod
    def from_condition(cls, cond: str, cond_delim: str = " and ", consequent: str | None = None) -> "RuleExpression":
        preds = [Predicate.parse(p) for p in cond.split(cond_delim) if p.strip()]
        return cls(preds, consequent, cond.strip())

    @property
    def ordinals(self) -> list[int]:
        return sorted({p.ordinal for p in self.predicates})

    def evaluate(self, cols: "ColumnCache") -> torch.Tensor:
        m = torch.ones(cols.n, dtype=torch.bool, device=cols.device)
        for p in self.predicates:
            m &= cols.compare(p)
        return m

    def evaluate_rows(self, rows: Sequence[Sequence[str]], device="cpu") -> torch.Tensor:
        return self.evaluate(ColumnCache(rows, device))


class ColumnCache:
    """Lazily tensorised columns of a list of split records."""

    def __init__(self, rows: Sequence[Sequence[str]], device="cpu"):
        self.rows = rows
        self.n = len(rows)
        self.device = torch.device(device)
        self._num: dict[int, torch.Tensor] = {}
        self._codes: dict[int, tuple[torch.Tensor, dict[str, int]]] = {}

    def numeric(self, o: int) -> torch.Tensor:
        if o not in self._num:
            v = []
            for r in self.rows:
                x = _num(r[o]) if o < len(r) else None
                v.append(math.nan if x is None else x)
            self._num[o] = torch.tensor(v, dtype=torch.float64, device=self.device)
        return self._num[o]

    def codes(self, o: int) -> tuple[torch.Tensor, dict[str, int]]:
        if o not in self._codes:
            vocab: dict[str, int] = {}
            c = [vocab.setdefault(r[o].strip() if o < len(r) else "", len(vocab)) for r in self.rows]
            self._codes[o] = (torch.tensor(c, dtype=torch.long, device=self.device), vocab)
        return self._codes[o]

    def compare(self, p: Predicate) -> torch.Tensor:
        if p.numeric and p.op in ("gt", "ge", "lt", "le", "eq", "ne"):
            x = self.numeric(p.ordinal)
            v = float(p.values[0])
            r = {"eq": x == v, "ne": x != v, "gt": x > v, "ge": x >= v, "lt": x < v, "le": x <= v}[p.op]
            return r & ~torch.isnan(x) if p.op != "ne" else r
        c, vocab = self.codes(p.ordinal)
        if p.op in ("in", "notIn", "eq", "ne"):
            ids = [vocab[v] for v in p.values if v in vocab]
            hit = torch.isin(c, torch.tensor(ids, dtype=torch.long, device=c.device)) if ids else \
                torch.zeros_like(c, dtype=torch.bool)
            return hit if p.op in ("in", "eq") else ~hit
        # lexicographic order comparison on strings
        inv = sorted(vocab, key=vocab.get)
        v = p.values[0]
        lut = torch.tensor([{"gt": s > v, "ge": s >= v, "lt": s < v, "le": s <= v}[p.op] for s in inv],
                           dtype=torch.bool, device=c.device)
        return lut[c] if len(inv) else torch.zeros_like(c, dtype=torch.bool)


class RecordColumns(ColumnCache):
    """ColumnCache's interface over a native token table (data/records.Records): ``codes(o)`` are
    the table's dictionary codes of field ``o`` (read with mode 'd', trimmed), ``numeric(o)`` its
    parsed doubles — the table's own numbers for fields read with mode 'n' (``num_fields``), else
    the numeric value of each dictionary string; everything stays on the table's device, no
    Python string per record."""

    def __init__(self, rec, num_fields=None):
        self.rec, self.n, self.device = rec, rec.n_lines, rec.device
        self.num_fields = None if num_fields is None else set(num_fields)
        self._vocab: dict[str, int] | None = None
        self._lut = None
        self._num, self._codes = {}, {}

    def numeric(self, o: int) -> torch.Tensor:
        if self.rec.nums is not None and (self.num_fields is None or o in self.num_fields):
            return self.rec.field(o, numeric=True)
        if self._lut is None:
            from ..data.records import numeric_lut
            self._lut = numeric_lut(self.rec.vocab, self.device)
        c = self.rec.field(o).long()
        if self._lut.numel() == 0:
            return torch.full(c.shape, math.nan, dtype=torch.float64, device=self.device)
        return torch.where(c >= 0, self._lut[c.clamp_min(0)], torch.full(c.shape, math.nan, dtype=torch.float64,
                                                                            device=self.device))

    def codes(self, o: int):
        if self._vocab is None:
            self._vocab = {}
            for i, v in enumerate(self.rec.vocab):
                self._vocab.setdefault(v, i)
        return self.rec.field(o).long(), self._vocab


def rule_field_modes(rules, extra: dict | None = None) -> dict[int, str]:
    """Tokenizer mode per field referenced by ``rules``: 'n' when every predicate on the field
    compares numerically, else 'd' (``extra`` adds / overrides fields)."""
    m: dict[int, str] = {}
    for r in rules:
        for p in r.predicates:
            num = p.numeric and p.op in ("gt", "ge", "lt", "le", "eq", "ne")
            m[p.ordinal] = "n" if num and m.get(p.ordinal, "n") == "n" else "d"
    m.update(extra or {})
    return m


def rules_from_config(cfg, names_key: str = "rule.names", rule_prefix: str = "rule.",
                      cond_delim_key: str = "cond.delim") -> dict[str, RuleExpression]:
    """``rue.rule.names=a,b`` + ``rue.rule.a=<cond> > <consequent>`` (RuleEvaluator.java:100-115)."""
    delim = cfg.get_str(cond_delim_key, None) or " and "
    names = cfg.get_list(names_key)
    return {n: RuleExpression.create_rule(cfg.get_str(rule_prefix + n), delim) for n in names}
