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
import math

import torch

from .. import _native
from ..parallel.comm import Comm, get_comm
from ..utils.resilience import IterationLoop, RecoveryConfig


_POP8 = torch.tensor([bin(i).count("1") for i in range(256)], dtype=torch.int64)


def _popcount64(x: torch.Tensor) -> torch.Tensor:
    """CPU popcount of int64 words (reference path): a 256-entry byte table over the 8 bytes."""
    return _POP8[x.contiguous().view(torch.uint8).long()].view(*x.shape, 8).sum(-1)


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
    out = torch.empty(cand_prefix.numel(), dtype=torch.int64)
    step = max(1, (1 << 22) // max(1, P.shape[1]))             # bounded temporaries
    for a in range(0, cand_prefix.numel(), step):
        b = min(cand_prefix.numel(), a + step)
        out[a:b] = _popcount64(P[cand_prefix[a:b].long()] & items[cand_item[a:b].long()]).sum(1)
    return out


class FrequentItemsets:
    """Frequent item sets per length: ``sets[k]`` int64 [N_k, k] item ids (rows sorted
    lexicographically, items ascending within a row) and ``sups[k]`` int64 [N_k] support counts, on
    the device that mined them; ``levels`` is the list view ({k: [(item-id tuple, count)]})."""

    def __init__(self, items: list[str], levels: dict | None = None, n_transactions: int = 0,
                 sets: dict | None = None, sups: dict | None = None):
        self.items = items
        self.n_transactions = n_transactions
        self.sets: dict[int, torch.Tensor] = dict(sets or {})
        self.sups: dict[int, torch.Tensor] = dict(sups or {})
        if levels is not None:
            for k, lv in levels.items():
                self.sets[k] = (torch.tensor([e[0] for e in lv], dtype=torch.long) if lv
                                else torch.zeros((0, k), dtype=torch.long))
                self.sups[k] = torch.tensor([e[1] for e in lv], dtype=torch.long)
        self._levels = None

    @property
    def levels(self) -> dict[int, list[tuple[tuple[int, ...], int]]]:
        if self._levels is None:
            self._levels = {k: [(tuple(a), int(b)) for a, b in zip(self.sets[k].tolist(), self.sups[k].tolist())]
                            for k in sorted(self.sets)}
        return self._levels

    def support(self, itemset: tuple[int, ...]) -> int | None:
        for s, c in self.levels.get(len(itemset), []):
            if s == itemset:
                return c
        return None

    def as_names(self, k: int) -> list[tuple[list[str], float]]:
        return [([self.items[i] for i in s], c / self.n_transactions) for s, c in self.levels.get(k, [])]


def _set_keys(S: torch.Tensor, base: int) -> torch.Tensor:
    """Order-preserving int64 key of every row (item ids ascending): exact mixed radix ``base``
    when base^k < 2^62, else a 64-bit polynomial hash (membership is then verified row-wise)."""
    k = S.shape[1]
    key = torch.zeros(S.shape[0], dtype=torch.long, device=S.device)
    if k * math.log2(max(base, 2)) < 62:
        for j in range(k):
            key = key * base + S[:, j]
        return key
    for j in range(k):
        key = key * 1000003 + S[:, j] + 1
        key = key ^ (key >> 29)
    return key


def _lookup(S: torch.Tensor, Q: torch.Tensor, base: int) -> torch.Tensor:
    """Row index of every row of ``Q`` in the row set ``S`` (-1 when absent), exact."""
    if S.shape[0] == 0 or Q.shape[0] == 0:
        return torch.full((Q.shape[0],), -1, dtype=torch.long, device=Q.device)
    ks = _set_keys(S, base)
    order = torch.argsort(ks)
    kss = ks[order]
    kq = _set_keys(Q, base)
    pos = torch.searchsorted(kss, kq).clamp_max(kss.numel() - 1)
    row = order[pos]
    hit = (kss[pos] == kq) & (S[row] == Q).all(1)
    return torch.where(hit, row, torch.full_like(row, -1))


def candidates(S: torch.Tensor, n_items: int) -> tuple[torch.Tensor, torch.Tensor]:
    """Apriori candidate generation on the device (S/association/FrequentItemsApriori.scala:222-262):
    the frequent (k-1)-sets ``S`` [N, k-1] (sorted rows) joined with every later row of the same
    (k-2)-prefix group — a segmented expansion, the K18 self-join pattern — then every candidate
    whose other (k-1)-subsets are not all frequent is pruned by an exact sorted-key lookup.
    Returns (prefix row a [M], candidates [M, k]) in lexicographic order."""
    N, km1 = S.shape
    dev = S.device
    if N < 2:
        return torch.zeros(0, dtype=torch.long, device=dev), torch.zeros((0, km1 + 1), dtype=torch.long, device=dev)
    if km1 == 1:
        gstart = torch.zeros(N, dtype=torch.long, device=dev)
        gend = torch.full((N,), N, dtype=torch.long, device=dev)
    else:
        pre = S[:, :-1]
        new = torch.ones(N, dtype=torch.bool, device=dev)
        new[1:] = (pre[1:] != pre[:-1]).any(1)
        gid = torch.cumsum(new.long(), 0) - 1
        starts = torch.nonzero(new).view(-1)
        ends = torch.cat([starts[1:], torch.tensor([N], device=dev)])
        gend = ends[gid]
    cnt = gend - torch.arange(N, device=dev) - 1                 # later rows of the same group
    a = torch.repeat_interleave(torch.arange(N, device=dev), cnt)
    first = torch.cumsum(cnt, 0) - cnt
    b = a + 1 + (torch.arange(a.numel(), device=dev) - first[a])
    cand = torch.cat([S[a], S[b][:, -1:]], 1)
    if km1 >= 2 and cand.shape[0]:
        ok = torch.ones(cand.shape[0], dtype=torch.bool, device=dev)
        k = km1 + 1
        for drop in range(k - 2):                # subsets without item `drop` (the last two are S[b], S[a])
            sub = torch.cat([cand[:, :drop], cand[:, drop + 1:]], 1)
            ok &= _lookup(S, sub, n_items) >= 0
        a, cand = a[ok], cand[ok]
    return a, cand


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
        """Level-wise mining with every level on the device: candidate join + prune
        (:func:`candidates`), ONE support kernel (AND + popcount of the (k-1)-prefix bit rows with
        the last item's row, K17), the support vector all-reduced across transaction shards, and a
        device filter.  The host sees only the level sizes (and the sets at the end)."""
        comm = self.comm or get_comm()
        dev = bits.device
        total = torch.tensor([n_tx], dtype=torch.int64, device=dev)
        if comm.is_distributed:
            comm.all_reduce(total)
        N = int(total)
        min_count = self.threshold * N
        I = bits.shape[0]
        ones = torch.full((1, bits.shape[1]), -1, dtype=torch.int64, device=dev)
        # level 1: support of every item = popcount(ones & item row)
        sup = itemset_support(ones, bits, torch.zeros(I, dtype=torch.int32, device=dev),
                              torch.arange(I, dtype=torch.int32, device=dev))
        if comm.is_distributed:
            comm.all_reduce(sup)
        keep = torch.nonzero(sup > min_count).view(-1)
        sets = {1: keep.view(-1, 1)}
        sups = {1: sup[keep].long()}
        S = sets[1]
        P = bits[keep]
        k = 1
        lp = IterationLoop("apriori", self.recovery, comm, device=dev)
        _, st, meta = lp.restore(dev)
        if st is not None:                  # resume after level ``meta['k']``: rebuild the level
            k = int(meta["k"])              # tensors and the prefix bitsets of the last level
            sets, sups = {}, {}
            for j in range(1, k + 1):
                if f"l{j}_sets" in st:
                    sets[j], sups[j] = st[f"l{j}_sets"].to(dev).long(), st[f"l{j}_sup"].to(dev).long()
            S = sets.get(k, torch.zeros((0, k), dtype=torch.long, device=dev))
            P = bits[S[:, -1]] if S.shape[0] else bits[:0]
            for c in range(k - 1):
                P = P & bits[S[:, c]]
        while S.shape[0] and k < self.max_len:
            k += 1
            with lp.step(k):
                a, cand = candidates(S, I)
                if cand.shape[0] == 0:
                    break
                sup = itemset_support(P, bits, a.int(), cand[:, -1].int())
                if comm.is_distributed:
                    comm.all_reduce(sup)
                keep = torch.nonzero(sup > min_count).view(-1)
                if keep.numel() == 0:
                    break
                S = cand[keep]
                P = P[a[keep]] & bits[cand[keep, -1]]
                sets[k], sups[k] = S, sup[keep].long()
            if lp.enabled:
                lp.commit(k, _levels_state(sets, sups), {"k": k})
        lp.close()
        return FrequentItemsets(items, None, N, sets, sups)


def _levels_state(sets, sups) -> dict[str, torch.Tensor]:
    out = {}
    for j in sets:
        out[f"l{j}_sets"] = sets[j].cpu()
        out[f"l{j}_sup"] = sups[j].cpu()
    return out


def association_rules(fi: FrequentItemsets, conf_threshold: float = 0.5, min_len: int = 2,
                      max_ante: int | None = None):
    """(antecedent names, consequent names, support, confidence) of every rule above the threshold
    (J/association/AssociationRuleMiner.java:111-196): per set length k and antecedent size r, the
    C(k, r) antecedents of all sets are gathered as one [N_k, C, r] tensor, their supports joined
    from level r by an exact sorted-key lookup, and the confidences filtered on the device; the
    host formats only the surviving rules (ordered by set, antecedent size, combination)."""
    out = []
    I = max(1, len(fi.items))
    for k in sorted(fi.sets):
        if k < min_len:
            continue
        S, cs = fi.sets[k], fi.sups[k]
        if S.shape[0] == 0:
            continue
        dev = S.device
        found = []            # (set idx, r, combo idx, ante cols, cons cols, conf)
        for r in range(1, k if max_ante is None else min(k, max_ante + 1)):
            if r not in fi.sets:
                continue
            combos = list(itertools.combinations(range(k), r))
            cidx = torch.tensor(combos, dtype=torch.long, device=dev)                 # [C, r]
            ante = S[:, cidx]                                                            # [N, C, r]
            row = _lookup(fi.sets[r], ante.reshape(-1, r), I).view(S.shape[0], len(combos))
            sa = torch.where(row >= 0, fi.sups[r][row.clamp_min(0)], torch.zeros_like(row))
            conf = cs.view(-1, 1).double() / torch.where(sa > 0, sa.double(), torch.ones_like(sa, dtype=torch.float64))
            ok = (row >= 0) & (sa > 0) & (conf > conf_threshold)
            si, ci = torch.nonzero(ok, as_tuple=True)
            if si.numel():
                found.append((si, torch.full_like(si, r), ci, conf[si, ci]))
        if not found:
            continue
        si = torch.cat([f[0] for f in found])
        rr = torch.cat([f[1] for f in found])
        ci = torch.cat([f[2] for f in found])
        cf = torch.cat([f[3] for f in found])
        key = (si * (k + 1) + rr) * (1 << 20) + ci
        o = torch.argsort(key)
        sets_l = S.tolist()
        sup_l = cs.tolist()
        combo_cache = {r: list(itertools.combinations(range(k), r)) for r in range(1, k)}
        for s_, r_, c_, f_ in zip(si[o].tolist(), rr[o].tolist(), ci[o].tolist(), cf[o].tolist()):
            ids = sets_l[s_]
            pos = combo_cache[r_][c_]
            ante = [fi.items[ids[p]] for p in pos]
            cons = [fi.items[ids[p]] for p in range(k) if p not in pos]
            out.append((ante, cons, sup_l[s_] / fi.n_transactions, f_))
    return out


def mark_infrequent(transactions: list[list[str]], fi: FrequentItemsets, marker: str = "*"):
    """InfrequentItemMarker: replace items not among the frequent 1-itemsets by ``marker``."""
    keep = {fi.items[s[0]] for s, _ in fi.levels.get(1, [])}
    return [[v if v in keep else marker for v in tr] for tr in transactions]
