"""Grab-bag helpers (``P/lib/util.py``, ``P/lib/weighted_rec_sampler.py``, ``P/app/comp_learn.py``).

ID / date / geo generators for fixtures, typed list parsing, keyed counters, ``StepFunction``,
``DummyVarGenerator`` (one-hot rows of delimited text), weighted record sampling (the reference
script is Python 2 and does not run; here it is a device multinomial draw), and PAC-learning
sample-complexity formulas (comp_learn.py: m >= (ln|H| + ln(1/delta)) / epsilon).
"""
from __future__ import annotations

import math
import random
import string
from collections import Counter, defaultdict
from datetime import datetime, timedelta
from itertools import combinations
from typing import Iterable, Sequence

import torch

_ALNUM = string.ascii_uppercase + string.digits


def gen_id(size: int = 10, rng: random.Random | None = None) -> str:
    r = rng or random
    return "".join(r.choice(_ALNUM) for _ in range(size))


def gen_ids(n: int, size: int = 10, seed: int = 0) -> list[str]:
    r = random.Random(seed)
    out, seen = [], set()
    while len(out) < n:
        s = gen_id(size, r)
        if s not in seen:
            seen.add(s)
            out.append(s)
    return out


def gen_name_initial(rng: random.Random | None = None) -> str:
    r = rng or random
    return r.choice(string.ascii_uppercase) + r.choice(string.ascii_uppercase)


def rand_date(start: datetime, days: int, rng: random.Random | None = None) -> datetime:
    r = rng or random
    return start + timedelta(seconds=r.randint(0, days * 86400))


def epoch_to_str(epoch: float, fmt: str = "%Y-%m-%d %H:%M:%S") -> str:
    return datetime.fromtimestamp(epoch).strftime(fmt)


def rand_location(lat: float, lon: float, radius_miles: float, n: int = 1, seed: int = 0) -> torch.Tensor:
    """Uniform points within a radius of (lat, lon): [n, 2] degrees."""
    g = torch.Generator().manual_seed(seed)
    r = radius_miles * torch.sqrt(torch.rand(n, generator=g, dtype=torch.float64))
    th = 2 * math.pi * torch.rand(n, generator=g, dtype=torch.float64)
    dlat = r * torch.cos(th) / 69.0
    dlon = r * torch.sin(th) / (69.0 * math.cos(math.radians(lat)))
    return torch.stack([lat + dlat, lon + dlon], 1)


def str_to_int_list(s: str, delim: str = ",") -> list[int]:
    return [int(v) for v in s.split(delim)] if s else []


def str_to_float_list(s: str, delim: str = ",") -> list[float]:
    return [float(v) for v in s.split(delim)] if s else []


def is_number(s: str) -> bool:
    try:
        float(s)
        return True
    except ValueError:
        return False


def keyed_list(pairs: Iterable[tuple]) -> dict:
    d = defaultdict(list)
    for k, v in pairs:
        d[k].append(v)
    return dict(d)


def count_keys(items: Iterable) -> dict:
    return dict(Counter(items))


class StepFunction:
    """Piecewise-constant lookup over (lo, hi, value) intervals; below / above the range returns the
    first / last value; values are looked up for a whole tensor at once."""

    def __init__(self, *points: tuple[float, float, float]):
        self.points = list(points)
        self.lo = torch.tensor([p[0] for p in points], dtype=torch.float64)
        self.hi = torch.tensor([p[1] for p in points], dtype=torch.float64)
        self.val = torch.tensor([p[2] for p in points], dtype=torch.float64)

    def find(self, x):
        xt = torch.as_tensor(x, dtype=torch.float64)
        scalar = xt.dim() == 0
        xt = xt.view(-1, 1)
        inside = (xt >= self.lo) & (xt < self.hi)
        y = torch.where(inside.any(1), (inside.double() * self.val).sum(1), torch.zeros(xt.shape[0], dtype=torch.float64))
        y = torch.where(xt.view(-1) < self.lo[0], self.val[0], y)
        y = torch.where(xt.view(-1) > self.hi[-1], self.val[-1], y)
        return float(y[0]) if scalar else y


class DummyVarGenerator:
    """Expand categorical columns of delimited rows into true/false indicator columns."""

    def __init__(self, row_size: int, cat_values: dict[int, Sequence[str]], true_val: str = "1",
                 false_val: str = "0", delim: str = ","):
        self.row_size, self.cat_values = row_size, {int(k): list(v) for k, v in cat_values.items()}
        self.true_val, self.false_val, self.delim = true_val, false_val, delim
        self.new_row_size = row_size - len(cat_values) + sum(len(v) for v in cat_values.values())

    def processRow(self, row: str) -> str:
        items = row.split(self.delim)
        if len(items) != self.row_size:
            raise ValueError(f"row does not have expected number of columns {len(items)}")
        out = []
        for i, v in enumerate(items):
            if i in self.cat_values:
                out += [self.true_val if v == c else self.false_val for c in self.cat_values[i]]
            else:
                out.append(v)
        return self.delim.join(out)


def weighted_record_sample(lines: Sequence[str], weight_index: int, n: int | None = None, seed: int = 0,
                           delim: str = ",") -> list[str]:
    """Sample records with replacement proportionally to the weight column (output sorted by
    position, like the reference script)."""
    w = torch.tensor([float(l.split(delim)[weight_index]) for l in lines], dtype=torch.float64)
    g = torch.Generator().manual_seed(seed)
    idx = torch.multinomial(w / w.sum(), n or len(lines), replacement=True, generator=g)
    return [lines[i] for i in sorted(idx.tolist())]


# ------------------------------------------------------------------------------------------------
# PAC learning sample complexity (comp_learn.py)
# ------------------------------------------------------------------------------------------------
def pac_num_samples(num_hyp: float, error: float, delta: float) -> int:
    return int(math.log(num_hyp / delta) / error)


def pac_num_samples_ln(num_hyp_ln: float, error: float, delta: float) -> int:
    return int((num_hyp_ln + math.log(1.0 / delta)) / error)


def terms_hyp_space(feature_card: Sequence[int], class_card: int) -> int:
    n = 1
    for f in feature_card:
        n *= f + 1
    return n * class_card


def value_combinations(feature_card: Sequence[int], num_vars: int) -> int:
    """Number of value assignments of ``num_vars`` distinct features (the reference's nested loops
    enumerate ordered index triples with overlapping ranges; here: unordered distinct subsets)."""
    if num_vars == len(feature_card):
        return math.prod(feature_card)
    return sum(math.prod(c) for c in combinations(feature_card, num_vars))


def disjunctive_hyp_space(feature_card: Sequence[int], class_card: int, c_size: int, d_size: int) -> int:
    """k-term DNF: choose ``d_size`` conjunctions of ``c_size`` literals."""
    m = value_combinations(feature_card, c_size)
    return math.comb(m, d_size) * class_card


def conjunctive_hyp_space_ln(feature_card: Sequence[int], class_card: int, d_size: int) -> float:
    """k-CNF: ln |H| ~ (#clauses) ln 2 + ln |classes|."""
    m = value_combinations(feature_card, d_size)
    return m * math.log(2) + math.log(class_card)
