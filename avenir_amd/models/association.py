"""Frequent itemsets (Apriori), infrequent-item marking and association rules (``J/association``,
``S/association/FrequentItemsApriori.scala``).

Reference: one MR job per itemset length k; mappers test every candidate against every transaction
and emit (itemset -> transId or 1), combiners dedup/sum, reducers keep sets with support above
``fia.support.threshold`` (``J/association/FrequentItemsApriori.java:133-343``); ``AssociationRuleMiner``
emits antecedent/consequent splits and keeps rules above ``arm.conf.threshold``.

MI355X: transactions become item bit rows ([I, T/64] uint64, built on device), every frequent
(k-1)-itemset keeps its transaction bitset, and a level is ONE support kernel over all candidates
(AND + popcount, K17) + one all-reduce of the support vector when transactions are sharded.
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass

import torch

from .. import _native
from ..parallel.comm import Comm, get_comm
from ..utils.resilience import IterationLoop, RecoveryConfig


def _popcount64(x: torch.Tensor) -> torch.Tensor:
    """CPU popcount of int64 words (reference path)."""
    v = x.clone()
    c = torch.zeros_like(v)
    for _ in range(64):
        c += v & 1
        v = torch.bitwise_right_shift(v, 1) & 0x7FFFFFFFFFFFFFFF
    return c


def build_bitsets(tx: torch.Tensor, item: torch.Tensor, n_tx: int, n_items: int) -> torch.Tensor:
    if tx.is_cuda:
        return _native.C().build_bitsets(tx.long().contiguous(), item.int().contiguous(), int(n_tx), int(n_items))
    W = max(1, (n_tx + 63) // 64)
    bits = torch.zeros((n_items, W), dtype=torch.int64)
    ok = (item >= 0) & (item < n_items) & (tx >= 0) & (tx < n_tx)
    # distinct (item, tx) pairs: adding distinct powers of two is OR (two's-complement wrap at bit 63)
    key = torch.unique(item[ok].long() * n_tx + tx[ok].long())
    i, t = key // n_tx, key % n_tx
    bits.view(-1).index_add_(0, i * W + t // 64, torch.bitwise_left_shift(torch.ones_like(t), t % 64))
    return bits


def itemset_support(P: torch.Tensor, items: torch.Tensor, cand_prefix: torch.Tensor,
                    cand_item: torch.Tensor) -> torch.Tensor:
    if P.is_cuda:
        return _native.C().itemset_support(P, items, cand_prefix.int().contiguous(), cand_item.int().contiguous())
    return _popcount64(P[cand_prefix.long()] & items[cand_item.long()]).sum(1)


@dataclass
class FrequentItemsets:
    items: list[str]
    levels: dict[int, list[tuple[tuple[int, ...], int]]]   # k -> [(itemset as item ids, support count)]
    n_transactions: int

    def support(self, itemset: tuple[int, ...]) -> int | None:
        for s, c in self.levels.get(len(itemset), []):
            if s == itemset:
                return c
        return None

    def as_names(self, k: int) -> list[tuple[list[str], float]]:
        return [([self.items[i] for i in s], c / self.n_transactions) for s, c in self.levels.get(k, [])]


class Apriori:
    def __init__(self, support_threshold: float = 0.1, max_len: int = 5, comm: Comm | None = None,
                 recovery: RecoveryConfig | None = None):
        self.threshold = support_threshold
        self.max_len = max_len
        self.comm = comm
        self.recovery = recovery        # per-level checkpoint / resume (utils/resilience)

    def fit_transactions(self, transactions: list[list[str]], device="cpu", tx_base: int = 0,
                         items: list[str] | None = None) -> FrequentItemsets:
        """Transactions as item-name lists (this rank's shard)."""
        comm = self.comm or get_comm()
        if items is None:
            local = sorted({i for tr in transactions for i in tr})
            allv = comm.all_gather_object(local) if comm.is_distributed else [local]
            items = sorted({i for lst in allv for i in lst})
        idx = {v: k for k, v in enumerate(items)}
        tx, it = [], []
        for t, tr in enumerate(transactions):
            for v in set(tr):
                if v in idx:
                    tx.append(t)
                    it.append(idx[v])
        dev = torch.device(device)
        bits = build_bitsets(torch.tensor(tx, dtype=torch.long, device=dev),
                             torch.tensor(it, dtype=torch.int32, device=dev), len(transactions), len(items))
        return self.fit_bitsets(bits, len(transactions), items)

    def fit_records(self, rec, skip: int = 0) -> FrequentItemsets:
        """Transactions from a CSR record table (data/records.py) whose first ``skip`` fields were
        tokenized as 'x' (transaction ids), so every dictionary entry is an item and the (merged)
        dictionary is the global item set.  Items are ordered by name (as ``fit_transactions``);
        (transaction, item) pairs go straight from the token table to the device bit rows."""
        items = sorted(rec.vocab)
        order = {v: k for k, v in enumerate(items)}
        dev = rec.device
        lut = torch.tensor([order[v] for v in rec.vocab] or [0], dtype=torch.int32, device=dev)
        ok = rec.codes >= 0
        tx = rec.line_of_token()[ok]
        it = lut[rec.codes[ok].long()] if len(rec.vocab) else rec.codes[ok]
        bits = build_bitsets(tx, it, rec.n_lines, len(items))
        return self.fit_bitsets(bits, rec.n_lines, items)

    def fit_bitsets(self, bits: torch.Tensor, n_tx: int, items: list[str]) -> FrequentItemsets:
        comm = self.comm or get_comm()
        total = torch.tensor([n_tx], dtype=torch.int64, device=bits.device)
        if comm.is_distributed:
            comm.all_reduce(total)
        N = int(total)
        min_count = self.threshold * N
        I = bits.shape[0]
        ones = torch.full((1, bits.shape[1]), -1, dtype=torch.int64, device=bits.device)
        # level 1: support of every item = popcount(ones & item row)
        sup = itemset_support(ones, bits, torch.zeros(I, dtype=torch.int32, device=bits.device),
                              torch.arange(I, dtype=torch.int32, device=bits.device))
        if comm.is_distributed:
            comm.all_reduce(sup)
        sup_l = sup.cpu().tolist()
        freq = [((i,), sup_l[i]) for i in range(I) if sup_l[i] > min_count]
        levels = {1: freq}
        P = bits[[s[0][0] for s in freq]] if freq else bits[:0]
        k = 1
        lp = IterationLoop("apriori", self.recovery, comm, device=bits.device)
        _, st, meta = lp.restore(bits.device)
        if st is not None:                  # resume after level ``meta['k']``: rebuild the level
            k = int(meta["k"])              # lists and the prefix bitsets of the last level
            levels = {}
            for j in range(1, k + 1):
                if f"l{j}_sets" not in st:
                    continue
                sets_t, sup_t = st[f"l{j}_sets"].tolist(), st[f"l{j}_sup"].tolist()
                levels[j] = [(tuple(a), b) for a, b in zip(sets_t, sup_t)]
            freq = levels.get(k, [])
            P = bits[[s[-1] for s, _ in freq]] if freq else bits[:0]
            if freq:
                idx = torch.tensor([s for s, _ in freq], dtype=torch.long, device=bits.device)
                for c in range(k - 1):
                    P = P & bits[idx[:, c]]
        while freq and k < self.max_len:
            k += 1
            with lp.step(k):
                sets = [s for s, _ in freq]
                setidx = {s: j for j, s in enumerate(sets)}
                cp, ci, cands = [], [], []
                # join (k-1)-sets sharing their first k-2 items; prune by the Apriori property
                by_pref: dict[tuple, list[int]] = {}
                for j, s in enumerate(sets):
                    by_pref.setdefault(s[:-1], []).append(j)
                for grp in by_pref.values():
                    for a, b in itertools.combinations(grp, 2):
                        sa, sb = sets[a], sets[b]
                        cand = sa + (sb[-1],) if sa[-1] < sb[-1] else sb + (sa[-1],)
                        if any(sub not in setidx for sub in itertools.combinations(cand, k - 1)):
                            continue
                        base = a if sa[-1] < sb[-1] else b
                        cp.append(base)
                        ci.append(cand[-1])
                        cands.append(cand)
                if not cands:
                    break
                dev = bits.device
                cpt = torch.tensor(cp, dtype=torch.int32, device=dev)
                cit = torch.tensor(ci, dtype=torch.int32, device=dev)
                sup = itemset_support(P, bits, cpt, cit)
                if comm.is_distributed:
                    comm.all_reduce(sup)
                sup_l = sup.cpu().tolist()
                keep = [m for m in range(len(cands)) if sup_l[m] > min_count]
                freq = [(cands[m], sup_l[m]) for m in keep]
                if freq:
                    kt = torch.tensor(keep, dtype=torch.long, device=dev)
                    P = P[cpt.long()[kt]] & bits[cit.long()[kt]]
                    order = sorted(range(len(freq)), key=lambda m: freq[m][0])
                    freq = [freq[m] for m in order]
                    P = P[torch.tensor(order, dtype=torch.long, device=dev)]
                    levels[k] = freq
            if lp.enabled:
                lp.commit(k, _levels_state(levels), {"k": k})
        lp.close()
        return FrequentItemsets(items, levels, N)


def _levels_state(levels) -> dict[str, torch.Tensor]:
    out = {}
    for j, lv in levels.items():
        out[f"l{j}_sets"] = (torch.tensor([e[0] for e in lv], dtype=torch.long) if lv
                             else torch.zeros((0, j), dtype=torch.long))
        out[f"l{j}_sup"] = torch.tensor([e[1] for e in lv], dtype=torch.long)
    return out


def association_rules(fi: FrequentItemsets, conf_threshold: float = 0.5, min_len: int = 2):
    """(antecedent names, consequent names, support, confidence) for every rule above threshold."""
    sup = {s: c for lvl in fi.levels.values() for s, c in lvl}
    out = []
    for k, lvl in fi.levels.items():
        if k < min_len:
            continue
        for s, c in lvl:
            for r in range(1, k):
                for ante in itertools.combinations(s, r):
                    a = sup.get(ante)
                    if not a:
                        continue
                    conf = c / a
                    if conf > conf_threshold:
                        cons = tuple(x for x in s if x not in ante)
                        out.append(([fi.items[i] for i in ante], [fi.items[i] for i in cons],
                                    c / fi.n_transactions, conf))
    return out


def mark_infrequent(transactions: list[list[str]], fi: FrequentItemsets, marker: str = "*"):
    """InfrequentItemMarker: replace items not among the frequent 1-itemsets by ``marker``."""
    keep = {fi.items[s[0]] for s, _ in fi.levels.get(1, [])}
    return [[v if v in keep else marker for v in tr] for tr in transactions]
