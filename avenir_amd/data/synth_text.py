"""Synthetic files in the reference's non-schema text layouts, written at memory speed (numpy byte
matrices of fixed-width fields), for the ingest-inclusive job benchmarks (benchmarks/bench_ingest.py,
``bench.py`` extras).  Formats (the jobs' docstrings):

* state sequences  ``id,[class,]s1,...,sL``        (markovStateTransitionModel, R/conv.sh)
* transactions     ``tid,item,...,item``           (frequentItemsApriori, R/fit.sh)
* tagged tokens    ``id,obs:state,...``            (hiddenMarkovModelBuilder)
* match pairs      ``src,trg,srcRec..,trgRec..,rank`` (topMatchesByClass)
* knn pairs        ``trainId,testId,dist,trainClass,testClass`` (nearestNeighbor)
* events           ``key,time,state``              (stateTransitionRate)
"""
from __future__ import annotations

from pathlib import Path

import numpy as np


def _digits(v: np.ndarray, width: int) -> np.ndarray:
    """[n, width] uint8 ASCII of non-negative ints, zero padded."""
    v = v.astype(np.int64)
    out = np.empty((v.shape[0], width), dtype=np.uint8)
    for j in range(width - 1, -1, -1):
        out[:, j] = 48 + (v % 10)
        v = v // 10
    return out


def _id(prefix: str, v: np.ndarray, width: int) -> np.ndarray:
    p = np.frombuffer(prefix.encode(), dtype=np.uint8)
    return np.concatenate([np.broadcast_to(p, (v.shape[0], p.size)), _digits(v, width)], axis=1)


def _pick(vocab: list[str], idx: np.ndarray) -> np.ndarray:
    """[n, w] bytes of vocab[idx] (every vocab entry must have the same length)."""
    w = len(vocab[0])
    if any(len(x) != w for x in vocab):
        raise ValueError("fixed-width vocabulary required")
    table = np.frombuffer("".join(vocab).encode(), dtype=np.uint8).reshape(len(vocab), w)
    return table[idx]


def _write(path, cols: list[np.ndarray], chunk: int = 1 << 20) -> int:
    """Join fixed-width byte columns with ',' and newline-terminate each row; returns bytes."""
    n = cols[0].shape[0]
    total = 0
    with open(path, "wb") as fh:
        for a in range(0, n, chunk):
            b = min(n, a + chunk)
            parts = []
            for j, c in enumerate(cols):
                parts.append(c[a:b])
                parts.append(np.full((b - a, 1), ord(",") if j < len(cols) - 1 else ord("\n"), dtype=np.uint8))
            blk = np.ascontiguousarray(np.concatenate(parts, axis=1))
            fh.write(blk.tobytes())
            total += blk.size
    return total


STATES = ["LNL", "LNN", "LHL", "MNS", "MHS", "MNN", "HNL", "HHS", "HNN"]


def state_sequences(path, n: int, seq_len: int = 10, states=STATES, classes=("T", "F"), seed: int = 0) -> int:
    rng = np.random.default_rng(seed)
    S = len(states)
    cols = [_id("C", np.arange(n), 9)]
    if classes:
        cols.append(_pick(list(classes), rng.integers(0, len(classes), n)))
    # a sticky chain: stay with prob 1/2, else move uniformly
    cur = rng.integers(0, S, n)
    for _ in range(seq_len):
        cols.append(_pick(list(states), cur))
        move = rng.random(n) < 0.5
        cur = np.where(move, rng.integers(0, S, n), cur)
    return _write(path, cols)


def transactions(path, n: int, n_items: int = 1000, per_tx: int = 8, seed: int = 0) -> int:
    """Items drawn from a Zipf-like law (a few frequent items); duplicates inside a row allowed."""
    rng = np.random.default_rng(seed)
    w = len(str(n_items - 1))
    p = 1.0 / np.arange(1, n_items + 1) ** 1.1
    p /= p.sum()
    cols = [_id("T", np.arange(n), 9)]
    for _ in range(per_tx):
        cols.append(_id("i", rng.choice(n_items, size=n, p=p), w))
    return _write(path, cols)


def tagged_sequences(path, n: int, seq_len: int = 8, obs=("a", "b", "c", "d"), states=("S", "T", "U"),
                     seed: int = 0) -> int:
    rng = np.random.default_rng(seed)
    cols = [_id("s", np.arange(n), 9)]
    st = rng.integers(0, len(states), n)
    for _ in range(seq_len):
        o = (st + rng.integers(0, 2, n)) % len(obs)
        tok = np.concatenate([_pick(list(obs), o), np.full((n, 1), ord(":"), np.uint8), _pick(list(states), st)], 1)
        cols.append(tok)
        st = np.where(rng.random(n) < 0.3, rng.integers(0, len(states), n), st)
    return _write(path, cols)


def observation_sequences(path, n: int, seq_len: int = 8, obs=("a", "b", "c", "d"), states=("S", "T", "U"),
                          seed: int = 0) -> int:
    """``id,o1,...,oL``: the observations of ``tagged_sequences`` without their state tags
    (viterbiStatePredictor input)."""
    rng = np.random.default_rng(seed)
    cols = [_id("s", np.arange(n), 9)]
    st = rng.integers(0, len(states), n)
    for _ in range(seq_len):
        cols.append(_pick(list(obs), (st + rng.integers(0, 2, n)) % len(obs)))
        st = np.where(rng.random(n) < 0.3, rng.integers(0, len(states), n), st)
    return _write(path, cols)


def match_pairs(path, n_pairs: int, n_entities: int, classes=("A", "B"), seed: int = 0) -> int:
    """``src,trg,srcId,srcClass,trgId,trgClass,rank`` (record = id, class; tmc.class.attr.ord=1)."""
    rng = np.random.default_rng(seed)
    w = len(str(n_entities - 1))
    s = rng.integers(0, n_entities, n_pairs)
    t = rng.integers(0, n_entities, n_pairs)
    cls = np.arange(n_entities) % len(classes)
    sid, tid = _id("e", s, w), _id("e", t, w)
    return _write(path, [sid, tid, sid, _pick(list(classes), cls[s]), tid, _pick(list(classes), cls[t]),
                         _digits(rng.integers(0, 10000, n_pairs), 4)])


def knn_pairs(path, n_test: int, k: int = 64, n_train: int = 100000, classes=("A", "B"), seed: int = 0) -> int:
    """``trainId,testId,dist,trainClass,testClass``: ``k`` candidate training records per test."""
    rng = np.random.default_rng(seed)
    n = n_test * k
    test = np.repeat(np.arange(n_test), k)
    train = rng.integers(0, n_train, n)
    tcls = test % len(classes)
    near = rng.random(n) < 0.7
    trcls = np.where(near, tcls, rng.integers(0, len(classes), n))
    return _write(path, [_id("r", train, len(str(n_train - 1))), _id("q", test, len(str(n_test - 1))),
                         _digits(rng.integers(0, 100000, n), 5), _pick(list(classes), trcls),
                         _pick(list(classes), tcls)])


def events(path, n: int, n_keys: int = 100000, states=("A", "B", "C", "D"), seed: int = 0) -> int:
    """``key,timeMs,state``: per key a time-ordered random walk, keys interleaved."""
    rng = np.random.default_rng(seed)
    key = rng.integers(0, n_keys, n)
    t = 1_600_000_000_000 + np.cumsum(rng.integers(1, 60_000, n))
    st = rng.integers(0, len(states), n)
    return _write(path, [_id("k", key, len(str(n_keys - 1))), _digits(t, 13), _pick(list(states), st)])


FORMATS = {"obs": observation_sequences, "mst": state_sequences, "apriori": transactions, "hmm": tagged_sequences, "tmc": match_pairs,
           "nen": knn_pairs, "str": events}


def write(fmt: str, path: str | Path, n: int, seed: int = 0) -> int:
    """``n`` records of format ``fmt`` (one of FORMATS) at ``path``; returns the byte count."""
    if fmt == "tmc":
        return match_pairs(path, n, max(16, n // 32), seed=seed)
    if fmt == "nen":
        return knn_pairs(path, max(1, n // 64), 64, seed=seed)
    return FORMATS[fmt](path, n, seed=seed)
