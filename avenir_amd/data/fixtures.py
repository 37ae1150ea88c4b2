"""Tutorial data-set generators (the reference's ``P/app/*.py`` fixture scripts), vectorised.

Every tutorial in the reference starts by running a small Python-2 generator that loops per
record, draws each field from a sampler and prints a CSV line.  Here each generator draws all
records at once with a seeded ``numpy.random.Generator`` (so a fixture is reproducible from its
seed, and 10^7 rows take seconds) and returns the CSV lines in the reference's field order and
number formats.  Time-stamped generators take an explicit ``end_time`` (epoch seconds) instead
of the wall clock, for reproducibility.

Samplers used by the reference and their equivalents here:
* ``GaussianRejectSampler(m, s)`` (rejection within m ± 3s)            -> ``_tnorm``
* ``NonParamRejectSampler(lo, width, *w)`` (histogram density)        -> ``_nonparam``
* ``CategoricalRejectSampler((v, w), ...)``                           -> ``_cat``
* ``AncestralSampler`` (class first, then class-conditional features) -> ``_ancestral``
* ``genID`` / ``genNumID`` (token alphabet with digits twice)         -> ``ids`` / ``num_ids``
* ``addNoiseNum`` / ``addNoiseCat``                                   -> ``_noise_num`` / ``_noise_cat``

``FIXTURES`` maps the reference script name to its generator; ``python -m avenir_amd genData
<name> ...`` prints one (cli.py).
"""
from __future__ import annotations

import math
from typing import Callable, Sequence

import numpy as np

_TOKENS = np.array(list("0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789"))   # P/lib/util.py:35-36
_DIGITS = np.array(list("0123456789"))
DAY_S, HOUR_S = 86400, 3600
DAY_MS, WEEK_MS = 86400 * 1000, 7 * 86400 * 1000
DEFAULT_END = 1_700_000_000     # fixed "now" (epoch s) so fixtures are reproducible


# ---------------------------------------------------------------------------------------------
# vectorised samplers
# ---------------------------------------------------------------------------------------------
def rng_of(seed: int | np.random.Generator) -> np.random.Generator:
    return seed if isinstance(seed, np.random.Generator) else np.random.default_rng(seed)


def ids(rng, n: int, size: int) -> np.ndarray:
    """``genID``: ``size`` tokens from the 46-token alphabet (digits twice as likely)."""
    pick = rng.integers(0, len(_TOKENS), size=(n, size))
    return np.array(["".join(r) for r in _TOKENS[pick]]) if n else np.array([], dtype=str)


def num_ids(rng, n: int, size: int) -> np.ndarray:
    pick = rng.integers(0, 10, size=(n, size))
    return np.array(["".join(r) for r in _DIGITS[pick]]) if n else np.array([], dtype=str)


def _tnorm(rng, mean, sd, n: int) -> np.ndarray:
    """Normal truncated to mean ± 3 sd (GaussianRejectSampler); mean / sd may be arrays [n]."""
    mean = np.broadcast_to(np.asarray(mean, dtype=np.float64), (n,))
    sd = np.broadcast_to(np.asarray(sd, dtype=np.float64), (n,))
    z = rng.standard_normal(n)
    bad = np.abs(z) > 3
    while bad.any():
        z[bad] = rng.standard_normal(int(bad.sum()))
        bad = np.abs(z) > 3
    return mean + sd * z


def _nonparam(rng, lo: float, width: float, weights: Sequence[float], n: int) -> np.ndarray:
    """Histogram density: bin by weight, uniform inside the bin (NonParamRejectSampler)."""
    w = np.asarray(weights, dtype=np.float64)
    k = rng.choice(len(w), size=n, p=w / w.sum())
    return lo + (k + rng.random(n)) * width


def _cat(rng, values: Sequence, weights: Sequence[float], n: int) -> np.ndarray:
    w = np.asarray(weights, dtype=np.float64)
    return np.asarray(values)[rng.choice(len(w), size=n, p=w / w.sum())]


def _uniform_pick(rng, values: Sequence, n: int) -> np.ndarray:
    return np.asarray(values)[rng.integers(0, len(values), n)]


def _event(rng, pct: float, n: int) -> np.ndarray:
    """``isEventSampled(pct)``: randint(0, 100) < pct."""
    return rng.integers(0, 101, n) < pct


def _noise_num(rng, x: np.ndarray, sd: float) -> np.ndarray:
    """``addNoiseNum``: x * (1 + N(0, sd)) (multiplicative noise)."""
    return x * (1.0 + _tnorm(rng, 0.0, sd, len(x))) if sd > 0 else x


def _noise_cat(rng, x: np.ndarray, values: Sequence, pct: float) -> np.ndarray:
    """``addNoiseCat``: with probability ``pct`` replace by a random other value."""
    if pct <= 0:
        return x
    flip = rng.random(len(x)) < pct
    return np.where(flip, _uniform_pick(rng, values, len(x)), x)


def _step(x: np.ndarray, steps: Sequence[tuple[float, float, float]]) -> np.ndarray:
    """``StepFunction((lo, hi, v), ...).find``: v where lo <= x < hi, else 0."""
    out = np.zeros(len(x))
    for lo, hi, v in steps:
        out = np.where((x >= lo) & (x < hi), v, out)
    return out


def _ancestral(rng, class_values, class_weights, feats: Sequence[tuple], n: int):
    """Class first, then every feature from its class-conditional sampler.  ``feats[j]`` maps
    class value -> ("cat", values, weights) | ("num", mean, sd) | ("np", lo, width, weights)."""
    y = _cat(rng, class_values, class_weights, n)
    cols = []
    for spec in feats:
        col = np.empty(n, dtype=object)
        for cv in class_values:
            m = y == cv
            k = int(m.sum())
            s = spec[cv]
            if s[0] == "cat":
                col[m] = _cat(rng, s[1], s[2], k)
            elif s[0] == "num":
                col[m] = _tnorm(rng, s[1], s[2], k)
            else:
                col[m] = _nonparam(rng, s[1], s[2], s[3], k)
        cols.append(col)
    return y, cols


def _fmt(v, prec: int = 3) -> str:
    if isinstance(v, (float, np.floating)):
        return f"{v:.{prec}f}"
    return str(v)


def _rows(*cols, delim: str = ",") -> list[str]:
    return [delim.join(r) for r in zip(*cols)]


def _s(col, fmt: str | None = None) -> list[str]:
    if fmt is None:
        return [str(v) for v in col]
    return [fmt % v for v in col]


def dummy_vars(lines: Sequence[str], cat_vars: dict[int, Sequence[str]], true: str = "1", false: str = "0",
               delim: str = ",") -> list[str]:
    """``DummyVarGenerator.processRow`` (P/lib/util.py:1120): every categorical column listed in
    ``cat_vars`` (index -> values) is replaced in place by one true/false column per value."""
    out = []
    for ln in lines:
        items = ln.strip().split(delim)
        new = []
        for i, it in enumerate(items):
            if i in cat_vars:
                new.extend(true if it == v else false for v in cat_vars[i])
            else:
                new.append(it)
        out.append(delim.join(new))
    return out


# ---------------------------------------------------------------------------------------------
# generators (one per reference script)
# ---------------------------------------------------------------------------------------------
def advt(num_apps: int, num_models: int, num_advt: int, num_zip: int, num_days: int, seed=0,
         end_time: int = DEFAULT_END) -> list[str]:
    """Ad impressions: impression id, os, device model, app, advert, zip, tapped (20 %) every
    5–30 s over ``num_days`` days (P/app/advt.py:26-60)."""
    rng = rng_of(seed)
    apps, adverts, zips = ids(rng, num_apps, 8), ids(rng, num_advt, 10), num_ids(rng, num_zip, 5)
    models = {"Android": ids(rng, int(num_models * 0.6), 8), "iOS": ids(rng, int(num_models * 0.4), 8)}
    span = (num_days + 1) * DAY_S
    n = int(span / 17.5 * 1.1) + 16
    t = np.cumsum(rng.integers(5, 31, n))
    n = int(np.searchsorted(t, span))
    os_ = _uniform_pick(rng, ["Android", "iOS"], n)
    model = np.where(os_ == "Android", _uniform_pick(rng, models["Android"], n), _uniform_pick(rng, models["iOS"], n))
    tapped = _event(rng, 20, n).astype(int)
    return _rows(ids(rng, n, 16), os_, model, _uniform_pick(rng, apps, n), _uniform_pick(rng, adverts, n),
                 _uniform_pick(rng, zips, n), _s(tapped))


def atm_xaction(num_atm: int, history_days: int, bucket: int, seed=0, end_time: int = DEFAULT_END) -> list[str]:
    """Daily ATM transaction totals, weekday N(40,10) vs weekend N(60,15), bucketed
    (P/app/atm_xaction.py:24-56).  Rows: atm id, time ms, transactions."""
    rng = rng_of(seed)
    atms = ids(rng, num_atm, 12)
    now = end_time * 1000
    past = (now - history_days * DAY_MS) // DAY_MS * DAY_MS
    days = np.arange(past, now, DAY_MS)
    T = np.repeat(days, num_atm)
    A = np.tile(atms, len(days))
    weekday = ((T % WEEK_MS) // DAY_MS) < 5
    x = np.where(weekday, _tnorm(rng, 40, 10, len(T)), _tnorm(rng, 60, 15, len(T)))
    trans = (x + bucket).astype(np.int64) // bucket * bucket
    return _rows(A, _s(T), _s(trans))


def call_hangup(n: int, seed=0) -> list[str]:
    from .synth import call_hangup_lines
    return call_hangup_lines(n, seed if isinstance(seed, int) else 0)


def cs_escalate(n: int, noise: float, key_len: int | None = None, seed=0) -> list[str]:
    """Customer-service escalation, ancestral sampler with 8 class-conditional features
    (P/app/cs_escalate.py:28-104)."""
    rng = rng_of(seed)
    feats = [
        {"1": ("np", 1, 1, [15, 20, 15, 30, 40, 55, 80, 120, 170]), "0": ("np", 1, 1, [120, 90, 70, 30, 10])},
        {"1": ("np", 0, 1, [20, 35, 80]), "0": ("np", 0, 1, [120, 80, 20])},
        {"1": ("num", 16, 2), "0": ("num", 4, 1)},
        {"1": ("np", 0, 1, [15, 35, 70]), "0": ("np", 0, 1, [120, 60])},
        {"1": ("num", 16, 4), "0": ("num", 8, 2)},
        {"1": ("num", 24, 2), "0": ("num", 12, 1)},
        {"1": ("np", 0, 1, [20, 40, 70]), "0": ("np", 0, 1, [100, 40])},
        {"1": ("cat", ["0", "1"], [20, 80]), "0": ("cat", ["0", "1"], [90, 10])},
    ]
    y, cols = _ancestral(rng, ["1", "0"], [30, 70], feats, n)
    out = [_s(_noise_num(rng, c.astype(np.float64), noise).astype(np.int64)) for c in cols[:7]]
    out.append(list(_noise_cat(rng, cols[7].astype(str), ["1", "0"], noise)))
    cl = _noise_cat(rng, y, ["1", "0"], noise)
    rows = _rows(*out, cl)
    if key_len:
        rows = [f"{k},{r}" for k, r in zip(ids(rng, n, key_len), rows)]
    return rows


def cust_seg(n: int, noise_level: int, seed=0) -> list[str]:
    """Three customer segments + noise (P/app/cust_seg.py:28-76).  Rows: id, visits, visit
    duration, time of visit, transactions, amount."""
    rng = rng_of(seed)
    pop = 100 - noise_level
    th = [pop * 40 // 100, pop * 70 // 100, pop]
    case = rng.integers(1, 101, n)
    seg = np.select([case < th[0], case < th[1], case < th[2]], [0, 1, 2], 3)
    nv = np.select([seg == 0, seg == 1, seg == 2],
                   [_tnorm(rng, 15, 3, n), _tnorm(rng, 8, 2, n), _tnorm(rng, 20, 5, n)], rng.integers(1, 31, n))
    vd = np.select([seg == 0, seg == 1, seg == 2],
                   [_tnorm(rng, 10, 2, n), _tnorm(rng, 20, 3, n), _tnorm(rng, 10, 3, n)], rng.integers(2, 41, n))
    tv = np.select([seg == 0], [2], np.where(seg == 3, rng.integers(0, 4, n), 3))
    u, u2 = rng.random(n), rng.random(n)
    frac = np.select([seg == 0, seg == 1, seg == 2], [0.4 + u * 0.2, 0.3 + u * 0.3, 0.5 + u * 0.2], 0.3 + u * 0.5)
    nx = (nv * frac).astype(np.int64)
    amt = nx * np.select([seg == 0, seg == 1, seg == 2],
                         [80 * (0.4 + u2 * 0.3), 100 * (0.9 + u2 * 0.5), 50 * (0.5 + u2 * 0.5)], 50 * (0.2 + u2 * 0.6))
    cid = 1000001 + np.arange(n)
    return _rows(_s(cid), _s(nv.astype(np.int64)), _s(vd.astype(np.int64)), _s(tv), _s(nx), _s(amt, "%.3f"))


def cust_value(n: int, seed=0) -> list[str]:
    """Customer value: 70 % random profiles (20 % high value), 30 % high-value archetypes
    (P/app/cust_value.py:24-64).  Rows: id, gender, zip, visit frequency, value T/F."""
    rng = rng_of(seed)
    genders, freqs = ["F", "F", "M", "M"], ["H", "M", "L", "M"]
    zip_groups = [num_ids(rng, int(rng.integers(10, 31)), 5) for _ in range(4)]
    all_zip = np.concatenate(zip_groups + [num_ids(rng, max(n // 10, 1), 5)])
    rand = rng.integers(1, 101, n) < 70
    c = rng.integers(0, 4, n)
    gender = np.where(rand, _uniform_pick(rng, genders, n), np.asarray(genders)[c])
    zg = np.array([_uniform_pick(rng, zip_groups[k], 1)[0] for k in c]) if n else np.array([], dtype=str)
    zc = np.where(rand, _uniform_pick(rng, all_zip, n), zg)
    fq = np.where(rand, _uniform_pick(rng, freqs, n), np.asarray(freqs)[c])
    value = np.where(rand, np.where(rng.integers(1, 101, n) < 80, "F", "T"), "T")
    return _rows(ids(rng, n, 8), gender, zc, fq, value)


def elearn(n: int, seed=0, as_int: bool = False) -> list[str]:
    """E-learning activity with a failure probability built from per-feature thresholds
    (P/app/elearn.py:26-105).  Rows: user id, 9 activity features, P/F.  The script prints the
    features as floats; ``as_int`` rounds them to the int fields of resource/elearnActivity.json."""
    rng = rng_of(seed)
    spec = [(300, 100), (80, 40), (40, 20), (10, 6), (50, 30), (60, 40), (100, 60), (60, 40), (12, 8)]
    f = [_tnorm(rng, m, s, n) for m, s in spec]
    for j in (0, 1, 2, 3, 6, 7, 8):
        f[j] = np.maximum(f[j], 0)
    f[4], f[5] = np.clip(f[4], 10, 100), np.clip(f[5], 10, 100)
    p = np.full(n, 10.0)
    p += np.select([f[0] < 100, f[0] < 150], [10, 6], 0)
    p += np.select([f[1] < 30, f[1] < 50], [8, 4], 0)
    p += np.where(f[1] < 10, 5, 0)                    # reference tests discussTime here (elearn.py:53)
    p += np.where(f[3] < 3, 6, 0)
    p += np.select([f[4] < 30, f[4] < 40, f[4] < 50], [34, 20, 14], 0)
    p += np.select([f[5] < 35, f[5] < 50, f[5] < 60], [28, 18, 10], 0)
    p += np.where(f[6] < 20, 4, 0)
    p += np.select([f[7] < 15, f[7] < 30], [7, 3], 0)
    p += np.where(f[8] < 4, 8, 0)
    status = np.where(rng.integers(0, 101, n) < p, "F", "P")
    uid = 1000000 + rng.integers(0, 1000001, n)
    if as_int:
        return _rows(_s(uid), *[_s(np.rint(c).astype(np.int64)) for c in f], status)
    return _rows(_s(uid), *[[repr(float(v)) for v in c] for c in f], status)


def exp_prod_price_discounts(num_prods: int, lead_times=(3, 5), discounts=(5, 10), seed=0) -> list[str]:
    """Perishable-product decision space: one ``pid,leadTime:discount`` row per combination
    (P/app/exp_prod_price.py ``createDiscounts``)."""
    rng = rng_of(seed)
    return [f"{p},{l}:{d}" for p in ids(rng, num_prods, 8) for l in lead_times for d in discounts]


def exp_prod_price_model(discount_lines: Sequence[str], lead_times=(3, 5), discounts=(5, 10), seed=0) -> list[str]:
    """Per product cost / price and inventory / demand distributions per (lead time, discount)
    (``createDistrModel``)."""
    rng = rng_of(seed)
    out, stat, last = [], {}, None
    max_lt = lead_times[-1]
    for ln in discount_lines:
        pid, ld = ln.split(",")[:2]
        lt, dc = (int(v) for v in ld.split(":"))
        if pid != last:
            cost = rng.uniform(10.0, 50.0)
            price = cost * rng.uniform(1.03, 1.08)
            max_inv = rng.uniform(500.0, 1000.0)
            stat = {}
            for l in lead_times:
                im = max_inv * rng.uniform(0.95, 1.05) * l / max_lt
                isd = rng.uniform(50.0, 100.0)
                for d in discounts:
                    stat[(l, d)] = (im, isd, im * rng.uniform(0.9, 1.1), rng.uniform(20.0, 150.0))
            last = pid
        im, isd, dm, dsd = stat[(lt, dc)]
        out.append(f"{pid},{ld.strip()},{cost:.3f},{price:.3f},{im:.3f},{isd:.3f},{dm:.3f},{dsd:.3f}")
    return out


def exp_prod_price_reward(model_lines: Sequence[str], decision_lines: Sequence[str], seed=0) -> list[str]:
    """Sampled profit of a (product, leadTime:discount) decision (``sampleReward``)."""
    rng = rng_of(seed)
    m = {}
    for ln in model_lines:
        it = ln.split(",")
        m[(it[0], it[1])] = tuple(float(v) for v in it[2:8])
    out = []
    for ln in decision_lines:
        pid, ld = (v.strip() for v in ln.split(",")[:2])
        cost, price, im, isd, dm, dsd = m[(pid, ld)]
        inv, dem = int(_tnorm(rng, im, isd, 1)[0]), int(_tnorm(rng, dm, dsd, 1)[0])
        unit = price - cost
        profit = inv * unit if dem > inv else dem * unit - (inv - dem) * cost
        out.append(f"{pid},{ld},{profit + 8000:.2f}")
    return out


def freq_items(item_count: int, triplet_count: int, n: int, seed=0, end_time: int = DEFAULT_END) -> list[str]:
    """Transactions seeded with frequent triplets (40 %), pairs (10 %) and singles (10 %) plus
    random fill (P/app/freq_items.py:25-94).  Rows: id, time, items..."""
    rng = rng_of(seed)
    items = ids(rng, item_count, 10)
    triplets = [list(_uniform_pick(rng, items, 3)) for _ in range(triplet_count)]
    pairs = [[t[i], t[j]] for t in triplets for i in range(3) for j in range(i + 1, 3)]
    pairs += [list(_uniform_pick(rng, items, 2)) for _ in range(5)]
    singles = [p[k] for p in pairs for k in (0, 1)] + list(_uniform_pick(rng, items, 10))
    t = end_time - 30 * DAY_S + np.cumsum(rng.integers(10, 301, n))
    r = rng.integers(0, 101, n)
    size = 3 + rng.integers(0, 11, n)
    out = []
    xid = ids(rng, n, 12)
    for i in range(n):
        if r[i] < 40:
            seed_items = triplets[rng.integers(len(triplets))]
        elif r[i] < 50:
            seed_items = pairs[rng.integers(len(pairs))]
        elif r[i] < 60:
            seed_items = [singles[rng.integers(len(singles))]]
        else:
            seed_items = []
        rest = list(_uniform_pick(rng, items, max(int(size[i]) - len(seed_items), 0)))
        out.append(",".join([xid[i], str(int(t[i]))] + list(seed_items) + rest))
    return out


def heart_disease(n: int, noise: float, key_len: int | None = None, seed=0) -> list[str]:
    """Heart disease, ancestral sampler over 10 features (P/app/heart_disease.py:26-112)."""
    rng = rng_of(seed)
    sex, smoker, diet, eth = ["M", "F"], ["NS", "SS", "SM"], ["BA", "AV", "GO"], ["WH", "BL", "SA", "EA"]
    feats = [
        {"1": ("cat", sex, [60, 40]), "0": ("cat", sex, [50, 50])},
        {"1": ("np", 30, 10, [10, 20, 35, 60, 90]), "0": ("np", 30, 10, [15, 20, 25, 30, 30])},
        {"1": ("num", 190, 8), "0": ("num", 150, 15)},
        {"1": ("np", 100, 10, [20, 25, 25, 30, 35, 45, 60, 75]), "0": ("np", 100, 10, [20, 30, 40, 20, 12, 8, 6, 4])},
        {"1": ("np", 60, 10, [20, 20, 25, 35, 50, 70]), "0": ("np", 60, 10, [20, 20, 25, 18, 12, 7])},
        {"1": ("cat", smoker, [20, 35, 60]), "0": ("cat", smoker, [40, 20, 15])},
        {"1": ("cat", diet, [60, 35, 20]), "0": ("cat", diet, [15, 40, 45])},
        {"1": ("num", 5, 1), "0": ("num", 15, 2)},
        {"1": ("num", 11, 2), "0": ("num", 17, 1)},
        {"1": ("cat", eth, [30, 40, 50, 20]), "0": ("cat", eth, [50, 20, 16, 20])},
    ]
    y, c = _ancestral(rng, ["1", "0"], [25, 75], feats, n)
    out = [list(_noise_cat(rng, c[0].astype(str), sex, noise)),
           [f"{float(v):.3f}" for v in c[1]],
           _s(_noise_num(rng, c[2].astype(np.float64), noise).astype(np.int64)),
           [f"{float(v):.3f}" for v in c[3]], [f"{float(v):.3f}" for v in c[4]],
           list(_noise_cat(rng, c[5].astype(str), smoker, noise)), list(_noise_cat(rng, c[6].astype(str), diet, noise)),
           _s(_noise_num(rng, c[7].astype(np.float64), noise).astype(np.int64)),
           _s(_noise_num(rng, c[8].astype(np.float64), noise).astype(np.int64)),
           list(_noise_cat(rng, c[9].astype(str), eth, noise))]
    rows = _rows(*out, _noise_cat(rng, y, ["1", "0"], noise))
    if key_len:
        rows = [f"{k},{r}" for k, r in zip(ids(rng, n, key_len), rows)]
    return rows


HEART_DISEASE_DUMMY = {0: ["M", "F"], 5: ["NS", "SS", "SM"], 6: ["BA", "AV", "GO"], 9: ["WH", "BL", "SA", "EA"]}


def lead_time(n: int, seed=0) -> list[str]:
    """Order lines with high lead time (T/F) from product, month and quantity scores
    (P/app/lead_time.py:24-64).  Rows: order id, product, quantity, month, status."""
    rng = rng_of(seed)
    prods = ids(rng, 50, 10)
    slow = rng.integers(0, 101, 50) < 30
    out, i = [], 0
    while i < n:
        k = min(int(rng.integers(5, 16)), n - i)
        oid, month = ids(rng, 1, 12)[0], int(rng.integers(1, 13))
        p = rng.integers(0, 50, k)
        q = rng.integers(100, 1001, k)
        score = rng.integers(5, 11, k) + np.where(slow[p], 40, 0) + (30 if month in (8, 10, 11) else 0) \
            + np.select([q > 800, q > 500], [30, 20], 0)
        for j in range(k):
            out.append(f"{oid},{prods[p[j]]},{q[j]},{month:02d},{'T' if score[j] > 60 else 'F'}")
        i += k
    return out


def loan_approve(n: int, seed=0) -> list[str]:
    from .generators import loan_approval
    return loan_approval().lines(n, seed if isinstance(seed, int) else 0)


def machine_op(n: int, seed=0) -> list[str]:
    """Machine failure from age, maintenance, breakdowns and vibration spectra
    (P/app/machine_op.py:24-80).  Label 1 / -1."""
    rng = rng_of(seed)
    age, maint = _tnorm(rng, 60, 15, n), _tnorm(rng, 6, 2, n)
    brk = np.where(rng.integers(0, 101, n) > 80, rng.integers(0, 3, n), 0)
    hi = rng.integers(0, 101, n) > 90
    f1 = np.where(hi, _tnorm(rng, 6000, 200, n), _tnorm(rng, 3000, 200, n))
    f2 = np.where(hi, _tnorm(rng, 8000, 100, n), _tnorm(rng, 4400, 100, n))
    a1, a2 = _tnorm(rng, 1.2, 0.2, n), _tnorm(rng, 1.2, 0.2, n)   # the reference samples both from the first
    pr = np.select([age > 90, age > 80], [10, 6], 0) + np.select([maint > 10, maint > 8], [8, 6], 0) \
        + np.where(brk > 0, 20, 0) + np.select([f1 > 6200, f1 > 5800], [26, 18], 0) + np.where(a1 > 1.4, 12, 0) \
        + np.select([f2 > 8200, f2 > 7800], [20, 16], 0) + np.where(a2 > 1.1, 8, 0)
    status = np.where(pr > rng.integers(40, 51, n), 1, -1)
    return _rows(ids(rng, n, 12), _s(age, "%.3f"), _s(maint, "%.3f"), _s(brk), _s(f1, "%.3f"), _s(a1, "%.3f"),
                 _s(f2, "%.3f"), _s(a2, "%.3f"), _s(status))


def pat(n: int, seed=0) -> list[str]:
    """Patient demographics with age-conditional income (P/app/pat.py:27-56)."""
    rng = rng_of(seed)
    sex = _cat(rng, ["1", "0"], [55, 45], n)
    married = _cat(rng, ["1", "0"], [40, 60], n)
    age = _cat(rng, ["Y", "M", "O"], [25, 35, 40], n)
    inc = np.empty(n, dtype=object)
    for a, w in (("Y", [75, 20, 5]), ("M", [10, 80, 10]), ("O", [10, 20, 70])):
        m = age == a
        inc[m] = _cat(rng, ["L", "M", "H"], w, int(m.sum()))
    eth = _cat(rng, ["WH", "BL", "SA", "EA"], [60, 20, 10, 10], n)
    return _rows(sex, married, age, inc.astype(str), eth)


PAT_DUMMY = {2: ["Y", "M", "O"], 3: ["L", "M", "H"], 4: ["WH", "BL", "SA", "EA"]}


def power(days_past: int, seed=0, end_time: int = DEFAULT_END) -> list[str]:
    """Hourly power usage: mean + trend + month and hour cycles + N(0, .05)
    (P/app/power.py:26-60)."""
    from datetime import datetime, timezone
    rng = rng_of(seed)
    year_c = np.array([0.75, 0.48, 0.22, -0.6, -0.08, 0.19, 0.40, 0.68, 0.41, 0.12, 0.39, .72])
    day_c = np.array([-0.10, -0.12, -0.16, -0.24, -0.28, -0.13, -0.08, 0.12, 0.25, 0.37, 0.45, 0.53, 0.42, 0.34,
                      0.26, 0.21, 0.16, 0.12, 0.10, 0.06, -0.01, -0.05, -0.08, -0.10])
    start = (end_time - (days_past + 1) * DAY_S) // HOUR_S * HOUR_S
    t = np.arange(start, end_time, HOUR_S)
    month = ((t % (365 * DAY_S)) // (30 * DAY_S)).clip(0, 11)
    usage = 3.0 + np.arange(len(t)) * (0.5 / (365 * 24)) + year_c[month] + day_c[(t % DAY_S) // HOUR_S] \
        + _tnorm(rng, 0.0, 0.05, len(t))
    ts = [datetime.fromtimestamp(int(v), timezone.utc).strftime("%Y-%m-%d %H:%M:%S") for v in t]
    return [f"{a},{u:.3f}" for a, u in zip(ts, usage)]


def price_opt(prod_count: int, seed=0) -> tuple[list[str], list[str]]:
    """Price-revenue curves per product (P/app/price_opt.py ``create_price``): returns (price
    rows ``prod,price,0,0,0``, stat rows ``prod,price,revenue`` with a revenue peak)."""
    rng = rng_of(seed)
    prices, stats = [], []
    for _ in range(1, prod_count):
        pid = int(rng.integers(1000000, 8000000))
        k, dp, p = int(rng.integers(6, 12)), int(rng.integers(2, 4)), int(rng.integers(10, 80))
        rev, dr = int(rng.integers(10000, 30000)), int(rng.integers(500, 1500))
        half = k // 2 + int(rng.integers(-2, 2))
        for pr in range(1, k):
            prices.append(f"{pid},{p},0,0,0")
            stats.append(f"{pid},{p},{rev}")
            p += dp
            rev += (dr + int(rng.integers(-20, 20))) * (1 if pr < half else -1)
    return prices, stats


def prot_seq(num_seq: int, min_len: int, max_len: int, mut_percent: int, seed=0) -> list[str]:
    """Divergent protein sequences: 10 % random seeds, each output a mutated, resized clone
    (P/app/prot_seq.py ``divergent``).  Rows: id, residues joined by ':'."""
    rng = rng_of(seed)
    aa = np.array(list("ACDEFGHIKLMNPQRSTVWY"))
    seeds = [aa[rng.integers(0, 20, int(rng.integers(min_len, max_len + 1)))] for _ in range(max(int(num_seq * 0.1), 1))]
    out = []
    keys = ids(rng, num_seq, 12)
    for i in range(num_seq):
        s = seeds[rng.integers(len(seeds))]
        ch = int(rng.integers(1, 7))
        s = np.concatenate([s, aa[rng.integers(0, 20, ch)]]) if rng.random() < 0.5 else s[:-ch].copy()
        if len(s):
            nm = int(len(s) * mut_percent / 100.0) + int(rng.integers(0, 11))
            s[rng.integers(0, len(s), nm)] = aa[rng.integers(0, 20, nm)]
        out.append(f"{keys[i]}," + ":".join(s))
    return out


def prsale_stats(num_prods: int, mean_tg=(300, 600), sd_tg=(30, 60), mean_qu=(2, 6), sd_qu=(1, 2), seed=0) -> list[str]:
    """Per product inter-sale gap and quantity distributions (P/app/prsale.py ``stat``)."""
    rng = rng_of(seed)
    return [f"{p},{rng.uniform(*mean_tg):.3f},{rng.uniform(*sd_tg):.3f}, {rng.uniform(*mean_qu):.3f}, "
            f"{rng.uniform(*sd_qu):.3f}" for p in ids(rng, num_prods, 12)]


def prsale(stat_lines: Sequence[str], start_days_past: int, end_days_past: int = 0, seed=0,
           end_time: int = DEFAULT_END) -> list[str]:
    """Sales events per product: gaps from N(tg), 8–16x longer before 6 am, quantity >= 1
    (P/app/prsale.py ``gen``).  Rows: product, time, quantity."""
    rng = rng_of(seed)
    start, stop = end_time - (start_days_past + 1) * DAY_S, end_time - end_days_past * DAY_S
    out = []
    for ln in stat_lines:
        it = [v.strip() for v in ln.split(",")]
        pid, mtg, stg, mqu, squ = it[0], *(float(v) for v in it[1:5])
        t = start
        while t < stop:
            k = 4096
            tg = _tnorm(rng, mtg, stg, k)
            qu = np.maximum(_tnorm(rng, mqu, squ, k).astype(np.int64), 1)
            for j in range(k):
                g = tg[j] * (int(rng.integers(8, 17)) if (t % DAY_S) < 6 * HOUR_S else 1)
                t += g
                if t >= stop:
                    break
                out.append(f"{pid},{int(t)},{qu[j]}")
    return out


def ranproj(num_dim: int, num_vecs: int, seed=0) -> list[str]:
    """Sparse random projection vectors: ~sqrt(d) N(0,1) entries (P/app/ranproj.py:25-41)."""
    rng = rng_of(seed)
    nz = int(math.sqrt(num_dim) + 0.5)
    nz = num_dim - 1 if nz == num_dim else nz
    out = []
    for _ in range(num_vecs):
        v = np.zeros(num_dim)
        v[rng.choice(num_dim, nz, replace=False)] = _tnorm(rng, 0.0, 1.0, nz)
        out.append(",".join(f"{x:.6f}" for x in v))
    return out


def retarget(n: int, seed=0) -> list[str]:
    """Retargeting conversions by customer type (P/app/retarget.py:7-23)."""
    rng = rng_of(seed)
    conv = {"1C": 75, "1S": 60, "1N": 50, "2C": 60, "2S": 40, "2N": 30, "3C": 20, "3S": 20, "3N": 15}
    types = np.array(list(conv))
    t = types[rng.integers(0, 9, n - 1)] if n > 1 else np.array([], dtype=str)
    p = np.array([conv[v] for v in t])
    c = np.where(rng.integers(1, 101, len(t)) < p, "Y", "N")
    return _rows(_s(1000000 + rng.integers(0, 1000000, len(t))), t, _s(20 + rng.integers(0, 301, len(t))), c)


def sales_lead(n: int, seed=0) -> list[str]:
    """Sales-lead conversion scored from 10 fields, converted if score > 116 (95 %)
    (P/app/sales_lead.py:25-82)."""
    rng = rng_of(seed)
    src = _cat(rng, ["tradeShow", "webDownload", "referral", "advertisement"], [80, 60, 100, 40], n)
    ct = _cat(rng, ["canReccommend", "canDecide"], [100, 40], n)
    cs = _cat(rng, ["small", "medium", "large"], [40, 100, 60], n)
    days = np.maximum(_tnorm(rng, 60, 30, n).astype(np.int64), 5)
    meet = np.maximum(_tnorm(rng, 5, 2, n).astype(np.int64), 0)
    mail = np.maximum(_tnorm(rng, 10, 3, n).astype(np.int64), 0)
    web = np.maximum(_tnorm(rng, 5, 2, n).astype(np.int64), 0)
    demo = np.maximum(_tnorm(rng, 3, 1, n).astype(np.int64), 0)
    rev = np.maximum(_tnorm(rng, 50000, 10000, n), 30000)
    prop = _cat(rng, ["Y", "N"], [40, 100], n)
    score = np.vectorize({"tradeShow": 12, "webDownload": 10, "referral": 20, "advertisement": 6}.get)(src) \
        + np.where(ct == "canDecide", 25, 15) + np.vectorize({"small": 7, "medium": 12, "large": 15}.get)(cs) \
        + _step(days, [(1, 20, 2), (20, 50, 5), (50, 80, 7), (80, 120, 8)]) \
        + _step(meet, [(0, 1, 1), (1, 5, 8), (5, 15, 9)]) + _step(mail, [(0, 1, 1), (1, 7, 6), (7, 18, 8)]) \
        + _step(web, [(0, 1, 1), (1, 5, 5), (5, 12, 7)]) + _step(demo, [(0, 1, 1), (1, 3, 15), (3, 5, 20)]) \
        + _step(rev, [(1, 30000, 16), (30000, 60000, 13), (60000, 100000, 10)]) + np.where(prop == "Y", 18, 7)
    conv = np.where((score > 116) & (rng.integers(0, 101, n) > 5), "1", "0")
    return _rows(ids(rng, n, 10), src, ct, cs, _s(days), _s(meet), _s(mail), _s(web), _s(demo),
                 _s(rev.astype(np.int64)), prop, conv)


SALES_LEAD_DUMMY = {1: ["tradeShow", "webDownload", "referral", "advertisement"], 2: ["canReccommend", "canDecide"],
                    3: ["small", "medium", "large"], 10: ["Y", "N"]}


def supplier(num_prod: int, history_weeks: int, seed=0, end_time: int = DEFAULT_END) -> list[str]:
    """Weekly order fulfilment level F / P / L per product (P/app/supplier.py:24-52)."""
    rng = rng_of(seed)
    prods = ids(rng, num_prod, 12)
    mean, sd = rng.integers(50, 81, num_prod), rng.integers(10, 21, num_prod)
    now = end_time * 1000
    t = (now - (history_weeks + 5) * WEEK_MS) // WEEK_MS * WEEK_MS
    out = []
    while t < now:
        full = rng.integers(0, 101, num_prod) > 40
        f = np.where(full, 100, np.clip(_tnorm(rng, mean, sd, num_prod), 20, 100))
        lvl = np.select([f == 100, f > 60], ["F", "P"], "L")
        out.extend(f"{p},{t},{l}" for p, l in zip(prods, lvl))
        t += WEEK_MS + int(rng.integers(-10, 11))
    return out


def telecom_churn(n: int, churn_rate: int, error_rate: int, seed=0, plan_id: bool = True) -> list[str]:
    """Telecom churn with three churn archetypes and label noise (P/app/telecom_churn.py:26-102).
    Rows: plan, minutes, data, cs calls, cs emails, network size, churn."""
    rng = rng_of(seed)
    thr = 100 - error_rate
    plan = rng.integers(1, 3, n)
    churned = rng.integers(1, 101, n) < churn_rate
    case = rng.integers(1, 5, n)
    minu = [_tnorm(rng, 600, 50, n), _tnorm(rng, 1200, 300, n)]
    data = [_tnorm(rng, 200, 50, n), _tnorm(rng, 500, 150, n)]
    call = [_tnorm(rng, 4, 1, n), _tnorm(rng, 8, 2, n)]
    mail = [_tnorm(rng, 6, 2, n), _tnorm(rng, 10, 3, n)]
    net = [_tnorm(rng, 3, 1, n), _tnorm(rng, 6, 2, n)]
    c14, c2 = churned & ((case == 1) | (case == 4)), churned & (case == 2)
    c3 = churned & (case == 3)
    plan = np.select([c14, c2 | c3], [1, 2], plan)
    keep = ~churned
    pm = plan - 1
    m = np.select([c14, c2, c3], [minu[1], minu[0], minu[0] + 200], np.where(pm == 0, minu[0], minu[1]))
    d = np.select([c14, c2, c3], [data[1], data[0], data[0] + 100], np.where(pm == 0, data[0], data[1]))
    cc = np.select([c2, keep], [np.maximum(call[1], 6), np.minimum(call[0], 2)], call[0])
    ce = np.select([c2, keep], [np.maximum(mail[1], 8), np.minimum(mail[0], 3)], mail[0])
    nw = np.where(c3, net[0], net[1])
    ok = rng.integers(1, 101, n) < thr
    label = np.where(churned, np.where(ok, 1, 0), np.where(ok, 0, 1))
    p = _s(plan) if plan_id else list(np.where(plan == 1, "plan A", "plan B"))
    return _rows(p, *[_s(v.astype(np.int64)) for v in (m, d, cc, ce, nw)], _s(label))


def visit_history(n: int, conv_rate: int, label: bool = False, seed=0) -> list[str]:
    """Web session histories of converting / non-converting users as elapsed+duration symbols
    (P/app/visit_history.py:25-84)."""
    rng = rng_of(seed)
    out = []
    uids = ids(rng, n, 12)
    for i in range(n):
        conv = rng.integers(0, 101) < conv_rate
        row = [uids[i]]
        if label:
            row.append(("T" if rng.integers(0, 101) < 90 else "F") if conv else ("F" if rng.integers(0, 101) < 90 else "T"))
        k = int(rng.integers(2, 21 if conv else 13))
        a, b = rng.integers(0, 101, k), rng.integers(0, 101, k)
        if conv:
            el = np.select([a <= 15, a <= 40], ["H", "M"], "L")
            du = np.select([b <= 15, b <= 40], ["L", "M"], "H")
        else:
            el = np.select([a <= 20, a <= 45], ["L", "M"], "H")
            du = np.select([b <= 20, b <= 45], ["H", "M"], "L")
        row.extend(e + d for e, d in zip(el, du))
        out.append(",".join(row))
    return out


def lat_long(n: int, lat1: float, long1: float, lat2: float, long2: float, seed=0) -> list[str]:
    """Uniform points in a lat/long box (P/app/gen_samples.py ``genLatLong``)."""
    rng = rng_of(seed)
    lat, lon = lat1 + (lat2 - lat1) * rng.random(n), long1 + (long2 - long1) * rng.random(n)
    return [f"{a:.5f}, {b:.5f}" for a, b in zip(lat, lon)]


def id_list(n: int, size: int, seed=0) -> list[str]:
    """P/app/id_gen.py, gen_samples.py ``genId``."""
    return list(ids(rng_of(seed), n, size))


# ---------------------------------------------------------------------------------------------
# resource/*.rb generators and transforms.  lib/util.rb is not part of the reference, so its
# samplers follow their use in the scripts: NumericalFieldRange(lo..hi, w, ...) = a range picked
# by weight, then a uniform integer inside it; CategoricalField(v, w, ...) = a value picked by
# weight; IdGenerator.generate(k) = a random k-token id.
# ---------------------------------------------------------------------------------------------
def _ranges(rng, spec: Sequence[tuple[tuple[int, int], float]], n: int) -> np.ndarray:
    lo = np.array([r[0] for r, _ in spec], dtype=np.int64)
    hi = np.array([r[1] for r, _ in spec], dtype=np.int64)
    w = np.array([w for _, w in spec], dtype=np.float64)
    k = rng.choice(len(spec), size=n, p=w / w.sum())
    return rng.integers(lo[k], hi[k] + 1)


def hosp_readmit(n: int, seed=0) -> list[str]:
    """Hospital readmission (resource/hosp_readmit.rb): id, age, weight, height, employment,
    family status, diet, exercise, follow-up, smoking, alcohol, readmitted (Y/N) with probability
    20 % plus the script's risk increments.  (The script's follow-up 'average' branch tests the
    misspelt 'avearge' and never fires; kept.)"""
    rng = rng_of(seed)
    pid = ids(rng, n, 12)
    age = _ranges(rng, [((10, 20), 2), ((21, 30), 3), ((31, 40), 6), ((41, 50), 10), ((51, 60), 14),
                        ((61, 70), 19), ((71, 80), 25), ((81, 90), 21)], n)
    wt = _ranges(rng, [((130, 140), 9), ((141, 150), 13), ((151, 160), 16), ((161, 170), 20), ((171, 180), 23),
                       ((181, 190), 20), ((191, 200), 17), ((201, 211), 14), ((211, 220), 10), ((221, 230), 7),
                       ((231, 240), 5), ((241, 250), 3)], n)
    ht = _ranges(rng, [((50, 55), 9), ((56, 60), 12), ((61, 65), 16), ((66, 70), 23), ((71, 75), 14)], n)
    p = 20 + np.select([age > 80, age > 70, age > 60], [10, 5, 3], 0)
    p += np.where((wt > 200) & (ht < 70), 5, np.where((wt > 180) & (ht < 60), 3, 0))
    emp = _cat(rng, ["employed", "unemployed", "retired"], [10, 1, 3], n)
    emp = np.where((age > 68) & (rng.integers(0, 10, n) < 8), "retired", emp)
    p += np.select([emp == "unemployed", emp == "retired"], [6, 4], 0)
    fam = _cat(rng, ["alone", "with partner"], [10, 15], n)
    p += np.where(fam == "alone", 9, 0)
    diet = _cat(rng, ["average", "poor", "good"], [10, 4, 2], n)
    diet = np.where((emp == "unemployed") & (rng.integers(0, 10, n) < 7), "poor", diet)
    p += np.select([diet == "poor", diet == "average"], [4, 2], 0)
    ex = _cat(rng, ["average", "low", "high"], [10, 12, 4], n)
    p += np.select([ex == "low", ex == "average"], [3, 1], 0)
    fu = _cat(rng, ["average", "low", "high"], [10, 14, 3], n)
    p += np.where(fu == "low", 8, 0)
    smoking = _cat(rng, ["non smoker", "smoker"], [10, 3], n)
    p += np.where(smoking == "smoker", 6, 0)
    alcohol = _cat(rng, ["average", "low", "high"], [10, 16, 4], n)
    p += np.select([alcohol == "high", alcohol == "average"], [5, 2], 0)
    readmit = np.where(rng.integers(0, 100, n) < p, "Y", "N")
    return _rows(_s(pid), _s(age), _s(wt), _s(ht), _s(emp), _s(fam), _s(diet), _s(ex), _s(fu), _s(smoking),
                 _s(alcohol), _s(readmit))


def disease(n: int, seed=0) -> list[str]:
    """Disease risk (resource/disease.rb): id, age 20-79, race, weight 120-239, diet, family
    history, domestic life, status Yes/No with risk 15 % scaled by age band, race, diet, family
    history and living alone (capped at 99 %)."""
    rng = rng_of(seed)
    pid = ids(rng, n, 12)
    age = 20 + rng.integers(0, 60, n)
    race = _cat(rng, ["EUA", "AFA", "LAA", "ASA"], [10, 3, 1, 1], n)
    weight = 120 + rng.integers(0, 120, n)
    diet = _cat(rng, ["LF", "REG", "HF"], [2, 8, 4], n)
    fam = _cat(rng, ["NFH", "FH"], [5, 1], n)
    dom = _cat(rng, ["S", "DP"], [2, 4], n)
    pr = 15.0 * np.select([age < 40, age < 50, age < 60, age < 70], [1.0, 1.05, 1.15, 1.4], 1.5)
    pr *= np.select([race == "AFA", race == "ASA", race == "LAA"], [1.2, 0.9, 0.95], 1.0)
    pr *= np.where(diet == "HF", 1.15, 1.0) * np.where(fam == "FH", 1.2, 1.0) * np.where(dom == "S", 1.2, 1.0)
    pr = np.minimum(pr, 99)
    status = np.where(rng.integers(0, 100, n) < pr, "Yes", "No")
    return _rows(_s(pid), _s(age), _s(race), _s(weight), _s(diet), _s(fam), _s(dom), _s(status))


EVENT_STATES = ["SL", "SS", "SM", "ML", "MS", "MM", "LL", "LS", "LM"]


def event_seq(n: int, seed=0) -> list[str]:
    """Customer event sequences (resource/event_seq.rb): 5-24 events from 9 states; after each
    event, with probability 0.3, a burst of 1-3 events from the same first-letter group (the
    script's first two members of the group)."""
    rng = rng_of(seed)
    cid = ids(rng, n, 10)
    ne = 5 + rng.integers(0, 20, n)
    B = int(ne.sum())
    base = rng.integers(0, 9, B)
    blen = np.where(rng.integers(0, 10, B) < 3, 1 + rng.integers(0, 3, B), 0)
    rep = np.repeat(np.arange(B), 1 + blen)
    first = np.r_[0, np.cumsum(1 + blen)[:-1]]
    pos = np.arange(len(rep)) - first[rep]
    ev = np.where(pos == 0, base[rep], (base[rep] // 3) * 3 + rng.integers(0, 2, len(rep)))
    per_cust = np.bincount(np.repeat(np.arange(n), ne), weights=1 + blen, minlength=n).astype(np.int64)
    names = np.asarray(EVENT_STATES)[ev]
    cuts = np.r_[0, np.cumsum(per_cust)]
    return [f"{cid[i]}," + ",".join(names[cuts[i]:cuts[i + 1]]) for i in range(n)]


def buy_xaction(cust_count: int, days: int, visitor_percent: float, seed=0, start_date: str = "2013-01-01",
                start_xid: int = DEFAULT_END) -> list[str]:
    """Purchase transactions (resource/buy_xaction.rb): every day visitor_percent x customers x
    U(85, 115) % transactions by customers drawn with replacement; a first purchase is 40-219,
    later ones depend on the days since and the amount of the customer's previous purchase.
    Rows: customer id, transaction id, date, amount.  Vectorised per day; repeat picks of a
    customer within a day are applied in pick order (rank rounds)."""
    rng = rng_of(seed)
    cids = ids(rng, cust_count, 10)
    last_day = np.full(cust_count, -1, dtype=np.int64)
    last_amt = np.zeros(cust_count, dtype=np.int64)
    day0 = np.datetime64(start_date, "D")
    out, xid = [], start_xid
    for d in range(days):
        m = int(visitor_percent * cust_count * (85 + rng.integers(0, 30)) / 100)
        pick = rng.integers(0, cust_count, m)
        order = np.argsort(pick, kind="stable")
        sp = pick[order]
        grp_start = np.r_[0, np.flatnonzero(np.diff(sp)) + 1]
        rank_sorted = np.arange(m) - np.repeat(grp_start, np.diff(np.r_[grp_start, m]))
        rank = np.empty(m, dtype=np.int64)
        rank[order] = rank_sorted
        amt = np.zeros(m, dtype=np.int64)
        for r in range(int(rank.max()) + 1 if m else 0):
            sel = np.flatnonzero(rank == r)
            c = pick[sel]
            k = len(sel)
            gap = d - last_day[c]
            la = last_amt[c]
            a = np.where(la < 40, 50 + rng.integers(0, 20, k) - 10, 30 + rng.integers(0, 10, k) - 5)
            a = np.where(gap >= 30, np.where(la < 80, 100 + rng.integers(0, 40, k) - 20,
                                             60 + rng.integers(0, 20, k) - 10), a)
            a = np.where(gap >= 60, np.where(la < 150, 180 + rng.integers(0, 60, k) - 30,
                                             120 + rng.integers(0, 40, k) - 20), a)
            a = np.where(last_day[c] < 0, 40 + rng.integers(0, 180, k), a)
            amt[sel] = a
            last_day[c] = d
            last_amt[c] = a
        date = str(day0 + d)
        out.extend(f"{cids[c]},{xid + 1 + i},{date},{a}" for i, (c, a) in enumerate(zip(pick, amt)))
        xid += m
    return out


def _xaction_state(prev_date, prev_amt, date, amt, short_days: int) -> str:
    dd = (date - prev_date).astype(np.int64)
    d = np.where(dd < short_days, "S", np.where(dd < 60, "M", "L"))
    a = np.where(prev_amt < 0.9 * amt, "L", np.where(prev_amt < 1.1 * amt, "E", "G"))
    return np.char.add(d, a)


def _group_xactions(lines: Sequence[str]) -> dict[str, tuple[np.ndarray, np.ndarray]]:
    hist: dict[str, list] = {}
    for ln in lines:
        it = ln.strip().split(",")
        hist.setdefault(it[0], []).append((it[2], it[3]))
    return {c: (np.array([np.datetime64(d, "D") for d, _ in h]), np.array([int(a) for _, a in h]))
            for c, h in hist.items()}


def xaction_seq(xaction_lines: Sequence[str]) -> list[str]:
    """Transaction -> state sequence per customer (resource/xaction_seq.rb): a state per pair of
    consecutive purchases, days gap S < 15 <= M < 60 <= L and amount change L / E / G at +-10 %;
    customers with more than one state."""
    out = []
    for c, (dates, amts) in _group_xactions(xaction_lines).items():
        if len(dates) < 2:
            continue
        seq = _xaction_state(dates[:-1], amts[:-1], dates[1:], amts[1:], 15)
        if len(seq) > 1:
            out.append(f"{c}," + ",".join(seq))
    return out


def xaction_state(history_lines: Sequence[str]) -> list[str]:
    """Per-customer history rows ``cid,date,amt,date,amt,...`` -> state sequences
    (resource/xaction_state.rb; gap thresholds 30 / 60 days), for rows with >= 2 purchases."""
    out = []
    for ln in history_lines:
        it = ln.strip().split(",")
        if len(it) < 5:
            continue
        dates = np.array([np.datetime64(x, "D") for x in it[1::2]])
        amts = np.array([int(x) for x in it[2::2]])
        seq = _xaction_state(dates[:-1], amts[:-1], dates[1:], amts[1:], 30)
        out.append(f"{it[0]}," + ",".join(seq))
    return out


MARK_STATES = ["SL", "SE", "SG", "ML", "ME", "MG", "LL", "LE", "LG"]


def mark_plan(xaction_lines: Sequence[str], model_rows: Sequence[Sequence[int]]) -> list[str]:
    """Next marketing date per customer (resource/mark_plan.rb): the last purchase-pair state
    (gap thresholds 30 / 60) -> most likely next state in the 9 x 9 transition count model ->
    last purchase date + 15 / 45 / 90 days.  Rows ``cid, date`` as the script prints them."""
    model = np.asarray(model_rows, dtype=np.int64)
    out = []
    for c, (dates, amts) in _group_xactions(xaction_lines).items():
        if len(dates) < 2:
            continue
        last = str(_xaction_state(dates[-2:-1], amts[-2:-1], dates[-1:], amts[-1:], 30)[0])
        nxt = MARK_STATES[int(np.argmax(model[MARK_STATES.index(last)]))]
        out.append(f"{c}, {dates[-1] + {'S': 15, 'M': 45, 'L': 90}[nxt[0]]}")
    return out


FIXTURES: dict[str, Callable] = {
    "advt": advt, "atm_xaction": atm_xaction, "call_hangup": call_hangup, "cs_escalate": cs_escalate,
    "cust_seg": cust_seg, "cust_value": cust_value, "elearn": elearn,
    "exp_prod_price": exp_prod_price_discounts, "freq_items": freq_items, "heart_disease": heart_disease,
    "lead_time": lead_time, "loan_approve": loan_approve, "machine_op": machine_op, "pat": pat, "power": power,
    "prot_seq": prot_seq, "prsale": prsale_stats, "ranproj": ranproj, "retarget": retarget,
    "sales_lead": sales_lead, "supplier": supplier, "telecom_churn": telecom_churn,
    "visit_history": visit_history, "lat_long": lat_long, "id_gen": id_list,
    # resource/*.rb
    "hosp_readmit": hosp_readmit, "disease": disease, "event_seq": event_seq, "buy_xaction": buy_xaction,
}
