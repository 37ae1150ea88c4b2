"""Apriori / association rule tests against a brute-force oracle."""
import itertools
import random

import pytest
import torch

from avenir_amd.models.association import Apriori, association_rules, build_bitsets, mark_infrequent

from _dist import run_world


def _transactions(n=400, n_items=12, seed=0):
    rng = random.Random(seed)
    items = [f"i{k}" for k in range(n_items)]
    tx = []
    for _ in range(n):
        base = rng.sample(items, rng.randint(1, 5))
        if rng.random() < 0.4:
            base += ["i1", "i2"]
        if rng.random() < 0.3:
            base += ["i1", "i2", "i3"]
        tx.append(sorted(set(base)))
    return tx


def _brute(tx, thr, max_len):
    items = sorted({i for t in tx for i in t})
    out = {}
    sets = [set(t) for t in tx]
    for k in range(1, max_len + 1):
        for c in itertools.combinations(items, k):
            cnt = sum(1 for s in sets if set(c) <= s)
            if cnt > thr * len(tx):
                out[c] = cnt
    return out


def test_apriori_matches_bruteforce():
    tx = _transactions()
    fi = Apriori(0.08, max_len=4).fit_transactions(tx)
    ref = _brute(tx, 0.08, 4)
    got = {tuple(fi.items[i] for i in s): c for lvl in fi.levels.values() for s, c in lvl}
    assert got == ref
    rules = association_rules(fi, 0.6)
    assert any(a == ["i3"] and "i1" in c for a, c, _, _ in rules)
    marked = mark_infrequent([["i1", "zzz"]], fi)
    assert marked == [["i1", "*"]]


def test_bitsets_roundtrip():
    b = build_bitsets(torch.tensor([0, 1, 63, 64, 130]), torch.tensor([0, 0, 1, 1, 2], dtype=torch.int32), 131, 3)
    assert b.shape == (3, 3)
    assert int(b[0, 0]) == 3 and int(b[1, 1]) == 1 and int(b[2, 2]) == 4


def _rank_apriori(rank, world, tx):
    from avenir_amd.parallel.comm import get_comm
    n = len(tx)
    part = tx[rank * n // world:(rank + 1) * n // world]
    fi = Apriori(0.08, max_len=4, comm=get_comm()).fit_transactions(part)
    return {tuple(fi.items[i] for i in s): c for lvl in fi.levels.values() for s, c in lvl}


def test_apriori_world_size_equivalence():
    tx = _transactions(301, seed=3)
    ref = _brute(tx, 0.08, 4)
    for got in run_world(_rank_apriori, 2, tx):
        assert got == ref


@pytest.mark.gpu
def test_apriori_gpu(cuda):
    tx = _transactions(5000, 20, seed=5)
    cpu = Apriori(0.05, max_len=4).fit_transactions(tx)
    gpu = Apriori(0.05, max_len=4).fit_transactions(tx, device=cuda)
    assert cpu.levels == gpu.levels
