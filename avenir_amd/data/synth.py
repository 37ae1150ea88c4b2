"""Seeded synthetic data generators (test fixtures and benchmark inputs).

Re-specified (not ported) from the reference's generators, keeping their planted signal:

* ``churn``       — mobile-churn usage data for ``resource/churn.json`` (``resource/usage.rb``):
  categorical usage levels, churn probability multiplied up by risk factors.
* ``call_hangup`` — call-centre hang-up data for ``resource/call_hangup.json``
  (``python/app/call_hangup.py``).
* ``supervised``  — generic per-class feature distributions (``SupvLearningDataGenerator``,
  ``python/lib/mlutil.py:263-369``).

Each generator can emit CSV lines (host) or device tensors directly (``*_device``) so benchmarks can
build multi-GB inputs on the GPU without touching the host.
"""
from __future__ import annotations

import json
import random
import string
from pathlib import Path

import numpy as np
import torch

CHURN_SCHEMA = {
    "fields": [
        {"name": "id", "ordinal": 0, "id": True, "dataType": "string"},
        {"name": "minUsed", "ordinal": 1, "dataType": "categorical",
         "cardinality": ["low", "med", "high", "overage"], "feature": True},
        {"name": "dataUsed", "ordinal": 2, "dataType": "categorical",
         "cardinality": ["low", "med", "high"], "feature": True},
        {"name": "CSCalls", "ordinal": 3, "dataType": "categorical",
         "cardinality": ["low", "med", "high"], "feature": True},
        {"name": "payment", "ordinal": 4, "dataType": "categorical",
         "cardinality": ["poor", "average", "good"], "feature": True},
        {"name": "acctAge", "ordinal": 5, "dataType": "categorical",
         "cardinality": ["1", "2", "3", "4", "5"], "feature": True},
        {"name": "status", "ordinal": 6, "dataType": "categorical", "cardinality": ["open", "closed"]},
    ]
}

# value weights and churn-risk multipliers (usage.rb)
_CHURN_W = [
    ([2, 5, 3, 2], [1.2, 1.0, 1.4, 1.8]),
    ([4, 6, 2], [1.1, 1.3, 1.6]),
    ([6, 3, 1], [1.0, 1.2, 1.6]),
    ([2, 5, 4], [1.3, 1.0, 1.0]),
    ([0, 1, 1, 1, 1], [1.0, 1.0, 1.05, 1.2, 1.3]),  # acctAge = rand(4)+1 (never 5... kept as-is)
]


def _id(rng: random.Random, k: int = 12) -> str:
    return "".join(rng.choice(string.ascii_uppercase + string.digits) for _ in range(k))


def churn_lines(n: int, seed: int = 0) -> list[str]:
    rng = random.Random(seed)
    card = [f["cardinality"] for f in CHURN_SCHEMA["fields"][1:6]]
    out = []
    for _ in range(n):
        vals, pr = [], 25.0
        for (w, mult), c in zip(_CHURN_W, card):
            k = rng.choices(range(len(w)), weights=w)[0]
            vals.append(c[k])
            pr *= mult[k]
        pr = min(pr, 99.0)
        status = "closed" if rng.random() * 100 < pr else "open"
        out.append(",".join([_id(rng)] + vals + [status]))
    return out


def write_churn(path: str | Path, n: int, seed: int = 0, schema_path: str | Path | None = None) -> None:
    Path(path).write_text("\n".join(churn_lines(n, seed)) + "\n")
    if schema_path:
        Path(schema_path).write_text(json.dumps(CHURN_SCHEMA, indent=2))


def churn_device(n: int, seed: int = 0, device="cuda", ld: int | None = None):
    """Churn columns generated directly on ``device``: (codes uint8 [5, ld], labels uint8 [ld]).
    Same distributions as ``churn_lines`` (inverse-CDF sampling with torch's Philox RNG)."""
    ld = ld or max(16, ((n + 15) // 16) * 16)
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    codes = torch.full((5, ld), 255, dtype=torch.uint8, device=device)
    risk = torch.full((n,), 25.0, dtype=torch.float32, device=device)
    for f, (w, mult) in enumerate(_CHURN_W):
        p = torch.tensor(w, dtype=torch.float32, device=device)
        cdf = torch.cumsum(p / p.sum(), 0)
        u = torch.rand(n, generator=g, device=device)
        k = torch.searchsorted(cdf, u).clamp_max(len(w) - 1)
        codes[f, :n] = k.to(torch.uint8)
        risk *= torch.tensor(mult, dtype=torch.float32, device=device)[k]
    risk.clamp_(max=99.0)
    u = torch.rand(n, generator=g, device=device) * 100
    labels = torch.full((ld,), 255, dtype=torch.uint8, device=device)
    labels[:n] = (u < risk).to(torch.uint8)
    return codes, labels


def write_churn_native(path: str | Path, n: int, seed: int = 0, nthreads: int = 8) -> int:
    """Write ``n`` churn records as CSV through the native multi-threaded writer
    (``avh::write_coded_csv``): the ``churn_device`` distributions sampled on the host, ids
    ``C<row>``.  Used for the ingest-inclusive benchmark (10^8-row files in seconds).
    Returns the bytes written."""
    from .. import _native
    C = _native.host()
    if C is None or not hasattr(C, "write_coded_csv"):
        raise RuntimeError("write_churn_native needs the native host module (avenir_amd._C)")
    codes, labels = churn_device(n, seed=seed, device="cpu")
    cols = torch.cat([codes, labels[None]], 0).contiguous()
    vocab = [list(f["cardinality"]) for f in CHURN_SCHEMA["fields"][1:7]]
    return int(C.write_coded_csv(str(path), cols, n, vocab, "C", ",", nthreads))


# ----------------------------------------------------------------------------------------------
CALL_HANGUP_SCHEMA = {
    "fields": [
        {"name": "id", "ordinal": 0, "id": True, "dataType": "string"},
        {"name": "customer type", "ordinal": 1, "dataType": "categorical", "feature": True,
         "maxSplit": 2, "cardinality": ["business", "residence"]},
        {"name": "issue", "ordinal": 3, "dataType": "categorical", "feature": True, "maxSplit": 2,
         "cardinality": ["internet", "cable", "billing", "other"]},
        {"name": "time of day", "ordinal": 4, "dataType": "categorical", "feature": True,
         "maxSplit": 2, "cardinality": ["AM", "PM"]},
        {"name": "hold time", "ordinal": 5, "dataType": "int", "feature": True, "bucketWidth": 60,
         "min": 0, "max": 600, "splitScanInterval": 60},
        {"name": "hungup", "ordinal": 6, "dataType": "categorical", "cardinality": ["T", "F"]},
    ]
}


def call_hangup_lines(n: int, seed: int = 0) -> list[str]:
    """Hang-up probability rises with hold time, residence callers and PM calls about billing."""
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        ct = rng.choices(["business", "residence"], weights=[4, 6])[0]
        area = rng.choice(["408", "650", "415", "510", "925"])
        issue = rng.choices(["internet", "cable", "billing", "other"], weights=[3, 3, 3, 1])[0]
        tod = rng.choice(["AM", "PM"])
        hold = int(max(0, min(599, rng.gauss(200 if issue != "billing" else 300, 120))))
        p = 0.1 + 0.6 * hold / 600
        p *= 1.3 if ct == "residence" else 0.8
        p *= 1.2 if tod == "PM" else 1.0
        hung = "T" if rng.random() < min(p, 0.95) else "F"
        out.append(",".join([_id(rng, 10), ct, area, issue, tod, str(hold), hung]))
    return out


# ----------------------------------------------------------------------------------------------
def supervised(n: int, n_features: int = 8, n_classes: int = 2, seed: int = 0, sep: float = 1.0,
               device="cpu") -> tuple[torch.Tensor, torch.Tensor]:
    """Gaussian blobs per class: X float32 [n, D], y int64 [n] (SupvLearningDataGenerator)."""
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    centers = torch.randn(n_classes, n_features, generator=g) * 2.0 * sep
    y = torch.randint(0, n_classes, (n,), generator=g)
    x = centers[y] + torch.randn(n, n_features, generator=g)
    return x.to(device), y.to(device)


def markov_sequences(n: int, n_states: int, length: int, n_classes: int = 2, seed: int = 0):
    """State sequences from class-specific random transition matrices: (states int16 [n, L],
    labels uint8 [n], trans float64 [C, S, S])."""
    rng = np.random.default_rng(seed)
    trans = rng.dirichlet(np.ones(n_states) * 0.5, size=(n_classes, n_states))
    labels = rng.integers(0, n_classes, n)
    states = np.zeros((n, length), dtype=np.int16)
    states[:, 0] = rng.integers(0, n_states, n)
    u = rng.random((n, length))
    for j in range(1, length):
        cdf = np.cumsum(trans[labels, states[:, j - 1]], axis=1)
        states[:, j] = np.minimum((u[:, j:j + 1] > cdf).sum(1), n_states - 1)
    return torch.from_numpy(states), torch.from_numpy(labels.astype(np.uint8)), torch.from_numpy(trans)
