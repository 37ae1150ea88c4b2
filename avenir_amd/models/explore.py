"""Exploratory analytics and categorical encodings (``J/explore``, ``S/explore``, ``J/util``).

All statistics here are functions of class-conditional (K2) and pair (K3) count tables, built in one
GPU pass each and all-reduced once across ranks:

* ``MutualInformation`` — MI(feature; class), MI(feature pair), MI(pair; class), pair-class joint
  entropy, class-conditional pair MI, and the greedy feature rankings MIM, MIFS, JMI, DISR, mRMR
  (``J/explore/MutualInformation.java:701-926``, ``J/explore/MutualInformationScore.java``).
* ``ContingencyStats`` — Cramér index, concentration coefficient (Goodman-Kruskal tau), uncertainty
  coefficient (``J/util/ContingencyMatrix.java:86-185``), used by ``CramerCorrelation`` and
  ``HeterogeneityReductionCorrelation``.
* ``NumericalCorrelation`` — Pearson matrix via one centred covariance GEMM (``XᵀX``).
* ``CategoricalClassAffinity`` — oddsRatio / distrDiff / minRisk / klDiff per value.
* encodings — supervised ratio / weight of evidence (``J/explore/CategoricalContinuousEncoding``,
  ``S/explore/CategoricalContinuousEncoding.scala``), leave-one-out, feature hashing, binary dummy
  variables, linear map.
* ``RuleEvaluator`` — per-rule class counts -> support and confidence.
* ``kolmogorov_smirnov_drift``, ``event_time_distribution``.
"""
from __future__ import annotations

import hashlib
import math
from dataclasses import dataclass
from typing import Sequence

import torch

from ..data.table import MISSING, Table
from ..ops import histogram as H
from ..parallel.comm import Comm, get_comm


def _reduce(comm: Comm | None, *ts: torch.Tensor) -> None:
    comm = comm or get_comm()
    if comm.is_distributed:
        for t in ts:
            comm.all_reduce(t)


def _plogp_sum(p: torch.Tensor) -> torch.Tensor:
    return -(torch.where(p > 0, p * torch.log(p.clamp_min(1e-300)), torch.zeros_like(p))).sum()


# ================================================================================================
# mutual information
# ================================================================================================
@dataclass
class MIResult:
    feature_class: dict[int, float]
    feature_pair: dict[tuple[int, int], float]
    pair_class: dict[tuple[int, int], float]
    pair_class_entropy: dict[tuple[int, int], float]
    pair_class_cond: dict[tuple[int, int], float]
    class_entropy: float


class MutualInformation:
    def __init__(self, redundancy_factor: float = 1.0, comm: Comm | None = None):
        self.redundancy_factor = redundancy_factor
        self.comm = comm

    def fit(self, t: Table) -> MIResult:
        n, C = t.n, t.n_classes
        bins = t.bins
        ords = [f.ordinal for f in t.binned_fields]
        fc = H.class_histogram(t.codes, n, bins, t.labels, C, count_labels=True)   # [C, TB+1]
        pairs = [(a, b) for a in range(len(bins)) for b in range(a + 1, len(bins))]
        pc = H.pair_histogram(t.codes, n, bins, pairs, t.labels, C)                 # [C, Ba, Bb] each
        flat = torch.cat([fc.view(-1)] + [x.reshape(-1) for x in pc]) if pc else fc.view(-1).clone()
        _reduce(self.comm, flat)
        fc = flat[: fc.numel()].view(fc.shape).double()
        o = fc.numel()
        pcs = []
        for x in pc:
            pcs.append(flat[o:o + x.numel()].view(x.shape).double())
            o += x.numel()
        self.class_feature_counts = fc                     # [C, TB + 1] (last column: class counts)
        cls_cnt = fc[:, -1]
        total = cls_cnt.sum()
        pc_ = cls_cnt / total
        res = MIResult({}, {}, {}, {}, {}, float(_plogp_sum(pc_)))
        off = 0
        feat_p = []
        for j, b in enumerate(bins):
            joint = fc[:, off:off + b] / total            # [C, B]
            pf = joint.sum(0)
            feat_p.append(pf)
            m = joint > 0
            mi = (joint[m] * torch.log(joint[m] / (pf.unsqueeze(0).expand_as(joint)[m] *
                                                    pc_.unsqueeze(1).expand_as(joint)[m]))).sum()
            res.feature_class[ords[j]] = float(mi)
            off += b
        for (a, b), cnt in zip(pairs, pcs):
            key = (ords[a], ords[b])
            jab = cnt.sum(0) / total                       # [Ba, Bb]
            m = jab > 0
            pa, pb = jab.sum(1), jab.sum(0)
            res.feature_pair[key] = float((jab[m] * torch.log(jab[m] / (pa.unsqueeze(1) * pb.unsqueeze(0))[m])).sum())
            jabc = cnt / total                             # [C, Ba, Bb]
            m3 = jabc > 0
            denom = (jab.unsqueeze(0) * pc_.view(-1, 1, 1)).expand_as(jabc)
            res.pair_class[key] = float((jabc[m3] * torch.log(jabc[m3] / denom[m3])).sum())
            res.pair_class_entropy[key] = float(_plogp_sum(jabc))
            # class-conditional pair MI: sum_c P(c) I(Fa; Fb | c)
            cm = 0.0
            for c in range(cnt.shape[0]):
                nc = cnt[c].sum()
                if nc <= 0:
                    continue
                pj = cnt[c] / nc
                qa, qb = pj.sum(1), pj.sum(0)
                mm = pj > 0
                cm += float(nc / total) * float((pj[mm] * torch.log(pj[mm] / (qa.unsqueeze(1) * qb.unsqueeze(0))[mm])).sum())
            res.pair_class_cond[key] = cm
        self.result = res
        return res

    # -- greedy feature scores (MutualInformationScore) ------------------------------------------
    def class_conditional_lines(self, t: Table, delim: str = ",") -> list[str]:
        """``featOrd,classVal,featVal,P(featVal|class)`` lines — the feature class-conditional
        distribution output (MutualInformation.java:560-583) that CategoricalClassAffinity reads."""
        fc = self.class_feature_counts
        cls_vals = t.label_values_all() if hasattr(t, "label_values_all") else t.class_field.cardinality
        out, off = [], 0
        for f in t.binned_fields:
            b = f.num_bins
            for c, cv in enumerate(cls_vals):
                n = float(fc[c, -1])
                for k in range(b):
                    cnt = float(fc[c, off + k])
                    if cnt > 0 and n > 0:
                        out.append(f"{f.ordinal}{delim}{cv}{delim}{f.bin_label(k)}{delim}{cnt / n!r}")
            off += b
        return out

    def mim(self) -> list[tuple[int, float]]:
        return sorted(self.result.feature_class.items(), key=lambda kv: -kv[1])

    def _pair(self, d: dict, a: int, b: int) -> float:
        return d.get((a, b), d.get((b, a), 0.0))

    def _greedy(self, score_fn, bootstrap: bool = False) -> list[tuple[int, float]]:
        feats = list(self.result.feature_class)
        sel: list[int] = []
        out: list[tuple[int, float]] = []
        if bootstrap:
            f0, v0 = self.mim()[0]
            sel.append(f0)
            out.append((f0, v0))
        while len(sel) < len(feats):
            best, arg = -math.inf, None
            for f in feats:
                if f in sel:
                    continue
                s = score_fn(f, sel)
                if s > best:
                    best, arg = s, f
            sel.append(arg)
            out.append((arg, best))
        return out

    def mifs(self, beta: float | None = None) -> list[tuple[int, float]]:
        b = self.redundancy_factor if beta is None else beta
        r = self.result
        return self._greedy(lambda f, sel: r.feature_class[f] - b * sum(self._pair(r.feature_pair, f, s) for s in sel))

    def jmi(self) -> list[tuple[int, float]]:
        r = self.result
        return self._greedy(lambda f, sel: sum(self._pair(r.pair_class, f, s) for s in sel), bootstrap=True)

    def disr(self) -> list[tuple[int, float]]:
        r = self.result
        return self._greedy(lambda f, sel: sum(self._pair(r.pair_class, f, s) /
                                               max(self._pair(r.pair_class_entropy, f, s), 1e-300) for s in sel),
                            bootstrap=True)

    def mrmr(self) -> list[tuple[int, float]]:
        r = self.result
        return self._greedy(lambda f, sel: r.feature_class[f] - (
            sum(self._pair(r.feature_pair, f, s) for s in sel) / len(sel) if sel else 0.0))


# ================================================================================================
# contingency statistics
# ================================================================================================
class ContingencyStats:
    """Statistics of an r x c count table (ContingencyMatrix semantics)."""

    def __init__(self, table: torch.Tensor):
        self.t = table.double().cpu()

    def cramer_index(self) -> float:
        t = self.t
        rs = t.sum(1).clamp_min(1)
        cs = t.sum(0).clamp_min(1)
        pearson = float((t * t / (rs.view(-1, 1) * cs.view(1, -1))).sum()) - 1.0
        return pearson / (min(t.shape) - 1)

    def cramers_v(self) -> float:
        return math.sqrt(max(self.cramer_index(), 0.0))

    def concentration_coeff(self) -> float:
        t = self.t
        tot = t.sum()
        rs, cs = t.sum(1) / tot, t.sum(0) / tot
        e = t / tot
        s1 = float(((e * e).sum(1) / rs.clamp_min(1e-300)).sum())
        s2 = float((cs * cs).sum())
        return (s1 - s2) / (1.0 - s2)

    def uncertainty_coeff(self) -> float:
        t = self.t
        tot = t.sum()
        rs, cs = t.sum(1) / tot, t.sum(0) / tot
        e = t / tot
        m = e > 0
        arg = (e * cs.view(1, -1) / rs.view(-1, 1).clamp_min(1e-300))
        s1 = float((e[m] * torch.log10(arg[m])).sum())
        mc = cs > 0
        s2 = float((cs[mc] * torch.log10(cs[mc])).sum())
        return s1 / s2

    def chi_square(self) -> tuple[float, int]:
        t = self.t
        tot = t.sum()
        exp = t.sum(1, keepdim=True) * t.sum(0, keepdim=True) / tot
        m = exp > 0
        return float(((t - exp) ** 2 / exp.clamp_min(1e-300))[m].sum()), (t.shape[0] - 1) * (t.shape[1] - 1)


def categorical_correlation(t: Table, pairs: Sequence[tuple[int, int]] | None = None,
                            stat: str = "cramer", comm: Comm | None = None) -> dict[tuple[int, int], float]:
    """CramerCorrelation / HeterogeneityReductionCorrelation over attribute pairs (ordinals)."""
    ords = [f.ordinal for f in t.binned_fields]
    if pairs is None:
        pairs = [(ords[a], ords[b]) for a in range(len(ords)) for b in range(a + 1, len(ords))]
    ip = [(ords.index(a), ords.index(b)) for a, b in pairs]
    tabs = H.pair_histogram(t.codes, t.n, t.bins, ip, None, 1)
    out = {}
    for (a, b), tab in zip(pairs, tabs):
        tab = tab[0].clone()
        _reduce(comm, tab)
        cs = ContingencyStats(tab)
        out[(a, b)] = {"cramer": cs.cramer_index, "concentration": cs.concentration_coeff,
                       "uncertainty": cs.uncertainty_coeff, "gini": cs.concentration_coeff}[stat]()
    return out


def numerical_correlation(X: torch.Tensor, comm: Comm | None = None) -> torch.Tensor:
    """Pearson correlation matrix of the columns of X [n, D] (one GEMM + one all-reduce)."""
    X = X.double()
    n = torch.tensor([X.shape[0]], dtype=torch.float64, device=X.device)
    s = X.sum(0)
    G = X.T @ X
    _reduce(comm, n, s, G)
    mean = s / n
    cov = G / n - mean.view(-1, 1) * mean.view(1, -1)
    sd = cov.diag().clamp_min(1e-300).sqrt()
    return cov / (sd.view(-1, 1) * sd.view(1, -1))


# ================================================================================================
# class affinity & encodings
# ================================================================================================
def class_affinity(t: Table, strategy: str = "oddsRatio", pos_class: int = 0,
                   comm: Comm | None = None) -> dict[int, list[tuple[str, float]]]:
    """Per categorical attribute, (value, affinity score) sorted descending
    (CategoricalClassAffinity: class-conditional value distributions P(v|pos), P(v|neg))."""
    cnt = H.class_histogram(t.codes, t.n, t.bins, t.labels, t.n_classes).double()
    _reduce(comm, cnt)
    out, o = {}, 0
    neg_class = 1 - pos_class if t.n_classes == 2 else None
    for j, f in enumerate(t.binned_fields):
        b = f.num_bins
        blk = cnt[:, o:o + b]
        pd = blk[pos_class] / blk[pos_class].sum().clamp_min(1)
        nd = (blk[neg_class] if neg_class is not None else blk.sum(0) - blk[pos_class])
        nd = nd / nd.sum().clamp_min(1)
        if strategy == "oddsRatio":
            s = (pd / (1 - pd)) / (nd / (1 - nd))
        elif strategy == "distrDiff":
            s = pd - nd
        elif strategy == "minRisk":
            s = pd * (1 - nd)
        elif strategy == "klDiff":
            s = pd * torch.log(pd / nd)
        else:
            raise ValueError(strategy)
        vals = [(f.bin_label(k), float(s[k])) for k in range(b)]
        out[f.ordinal] = sorted(vals, key=lambda kv: -kv[1] if not math.isnan(kv[1]) else math.inf)
        o += b
    return out


def supervised_encoding(t: Table, strategy: str = "supervisedRatio", scale: int = 1000, pos_class: int = 1,
                        comm: Comm | None = None, integer: bool = True) -> dict[int, dict[str, float]]:
    """Categorical value -> continuous value: positive rate x scale, or weight of evidence
    ln((pos/allPos)/(neg/allNeg)) x scale (zero negative counts use 1, like the MR reducer; the Spark
    variant's "negCount = posCount" bug is NOT reproduced)."""
    cnt = H.class_histogram(t.codes, t.n, t.bins, t.labels, t.n_classes, count_labels=True).double()
    _reduce(comm, cnt)
    neg_class = 1 - pos_class
    all_pos, all_neg = float(cnt[pos_class, -1]), float(cnt[neg_class, -1])
    out, o = {}, 0
    for f in t.binned_fields:
        b = f.num_bins
        pos = cnt[pos_class, o:o + b]
        neg = cnt[neg_class, o:o + b]
        if strategy == "weightOfEvidence":
            v = torch.log((pos / max(all_pos, 1)) / (torch.where(neg == 0, torch.ones_like(neg), neg) / max(all_neg, 1))) * scale
        else:
            v = pos * scale / (pos + neg).clamp_min(1)
        if integer:
            v = torch.trunc(v)
        out[f.ordinal] = {f.bin_label(k): float(v[k]) for k in range(b) if float(pos[k] + neg[k]) > 0}
        o += b
    return out


def apply_encoding(t: Table, enc: dict[int, dict[str, float]], default: float = 0.0) -> torch.Tensor:
    """Encoded [n, F] float matrix (gather through a per-attribute lookup table on device)."""
    cols = []
    for j, f in enumerate(t.binned_fields):
        if f.ordinal not in enc:
            continue
        # one slot per code incl. the missing code (255 / 65535; int32 codes clamp into the last slot)
        m = min(t.missing + 1, f.num_bins + 1)
        lut = torch.full((max(m, t.missing + 1) if t.codes.dtype != torch.int32 else m,), default,
                         dtype=torch.float64)
        e = enc[f.ordinal]
        ks = [k for k in range(f.num_bins) if f.bin_label(k) in e]
        if ks:
            lut[torch.tensor(ks)] = torch.tensor([e[f.bin_label(k)] for k in ks], dtype=torch.float64)
        cols.append(lut.float().to(t.device)[t.codes[j, : t.n].long().clamp(max=lut.numel() - 1)])
    return torch.stack(cols, 1) if cols else torch.zeros((t.n, 0), device=t.device)


def leave_one_out_encoding(t: Table, target: torch.Tensor, noise: float = 0.0, reg: float = 0.0,
                           seed: int = 0, comm: Comm | None = None, formula: str = "reference") -> torch.Tensor:
    """Leave-one-out target encoding per categorical value, on the K23 kernels.

    ``formula="reference"`` (default) is S/explore/CategoricalLeaveOneOutEncoding.scala:110-125:
    ``(sum_v - y_i) / (count_v - 1 + reg) * (1 + z)`` with ``z ~ N(0, noise)`` truncated at 3 sd
    (the ``categoricalLeaveOneOutEncoding`` job uses the same function).
    ``formula="smoothed"`` is a deliberate variant that is NOT in the reference: the prior
    ``reg * global_mean`` is added to the numerator (shrinkage towards the global mean) and the
    noise is uniform ``1 + noise * (2u - 1)``.

    The kernel computes ``(s - y + reg * g) / (k - 1 + reg) * (1 + amp * (2u - 1))``; the
    reference formula is the case ``g = 0``, ``amp = 1``, ``u = (z + 1) / 2``."""
    from ..ops import encode_ops as E
    if formula not in ("reference", "smoothed"):
        raise ValueError(f"formula must be 'reference' or 'smoothed', got {formula!r}")
    n = t.n
    y = target[:n].double().to(t.codes.device)
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    gsum = y.sum().view(1)
    gcnt = torch.tensor([float(n)], dtype=torch.float64, device=y.device)
    nf = len(t.binned_fields)
    codes = t.codes[:nf]
    from ..data.table import code_slots
    s, k = E.loo_stats(codes, n, y, code_slots(codes, t.bins[:nf]))  # K23: per (column, value) sums, counts
    _reduce(comm, gsum, gcnt, s, k)
    u = None
    if noise > 0:
        # one stream per column, drawn in column order from the seeded host generator
        if formula == "reference":
            z = torch.stack([(torch.randn(n, generator=g, dtype=torch.float64) * noise).clamp(-3 * noise, 3 * noise)
                             for _ in range(nf)])
            u, amp = (z + 1.0) / 2.0, 1.0
        else:
            u, amp = torch.stack([torch.rand(n, generator=g) for _ in range(nf)]).double(), float(noise)
    else:
        amp = 0.0
    gmean = torch.zeros(1, dtype=torch.float64, device=y.device) if formula == "reference" else gsum / gcnt
    return E.loo_apply(codes, n, y, s, k, gmean, reg=reg, noise=u, amp=amp)


def _hash_slot(j: int, v: str, size: int, signed: bool) -> tuple[int, float]:
    h = int.from_bytes(hashlib.md5(f"{j}:{v}".encode()).digest()[:8], "little")
    return h % size, (-1.0 if (signed and (h >> 63) & 1) else 1.0)


def feature_hashing(values: Sequence[Sequence[str]], size: int, signed: bool = True) -> torch.Tensor:
    """Hashing trick over categorical strings (index hash + sign hash), [n, size]
    (S/explore/CategoricalFeatureHashingEncoding.scala:107-119).  Each distinct (column, value) is
    hashed once; the rows are then one vectorised scatter-add."""
    cache: dict[tuple[int, str], int] = {}
    slots, signs, keys = [], [], []
    for row in values:
        for j, v in enumerate(row):
            key = (j, v)
            u = cache.get(key)
            if u is None:
                u = cache[key] = len(slots)
                idx, sg = _hash_slot(j, v, size, signed)
                slots.append(idx)
                signs.append(sg)
            keys.append(u)
    out = torch.zeros((len(values), size), dtype=torch.float32)
    if not keys:
        return out
    lens = torch.tensor([len(r) for r in values])
    rows = torch.repeat_interleave(torch.arange(len(values)), lens)
    k = torch.tensor(keys)
    return out.index_put_((rows, torch.tensor(slots)[k]), torch.tensor(signs, dtype=torch.float32)[k],
                          accumulate=True)


def feature_hashing_table(t: Table, size: int, signed: bool = True) -> torch.Tensor:
    """``feature_hashing`` of a Table's categorical columns on its device: every dictionary value
    is hashed once on the host into a per-column (slot, sign) lookup table, the [n, size] matrix is
    built by one gather + scatter-add over the resident codes (no per-record host work)."""
    cats = [(j, f) for j, f in enumerate(t.binned_fields) if f.is_categorical]
    out = torch.zeros((t.n, size), dtype=torch.float32, device=t.device)
    rows = torch.arange(t.n, device=t.device)
    for pos, (j, f) in enumerate(cats):
        lut_i = torch.zeros(t.missing + 1, dtype=torch.long)
        lut_s = torch.zeros(t.missing + 1, dtype=torch.float32)  # missing code contributes 0
        for k, v in enumerate(f.cardinality):
            lut_i[k], lut_s[k] = _hash_slot(pos, v, size, signed)
        c = t.codes[j, : t.n].long()
        out.index_put_((rows, lut_i.to(t.device)[c]), lut_s.to(t.device)[c], accumulate=True)
    return out


def binary_dummy(t: Table, true_val: str = "1", false_val: str = "0") -> tuple[torch.Tensor, list[str]]:
    """One-hot (binary dummy) variables for every categorical attribute: (uint8 [n, sum B], names)."""
    cols, names = [], []
    for j, f in enumerate(t.binned_fields):
        if not f.is_categorical:
            continue
        c = t.codes[j, : t.n].long()
        for k, v in enumerate(f.cardinality):
            cols.append((c == k).to(torch.uint8))
            names.append(f"{f.name}_{v}")
    return (torch.stack(cols, 1) if cols else torch.zeros((t.n, 0), dtype=torch.uint8)), names


def linear_map(X: torch.Tensor, M: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """y = M x (+ b) for selected numeric fields (S/util/LinearMapper.scala:61-89)."""
    y = X.float() @ M.float().T.to(X.device)
    return y + bias.to(X.device) if bias is not None else y


# ================================================================================================
# rules, drift, event time
# ================================================================================================
class RuleEvaluator:
    """Named rules over records -> per-rule class counts -> support and confidence
    (J/explore/RuleEvaluator.java:122-268).  A rule is a callable(table) -> bool mask [n]
    (antecedent) plus a consequent class index."""

    def __init__(self, rules: dict[str, tuple], conf_strategy: str = "confAccuracy", comm: Comm | None = None):
        self.rules = rules
        self.conf_strategy = conf_strategy
        self.comm = comm

    def evaluate(self, t: Table) -> dict[str, dict[str, float]]:
        out = {}
        lab = t.labels[: t.n].long()
        C = t.n_classes
        for name, (cond, consequent) in self.rules.items():
            m = cond(t)
            cnt = torch.bincount(lab[m], minlength=C)[:C].double()
            tot = torch.tensor([float(t.n)], dtype=torch.float64, device=cnt.device)
            _reduce(self.comm, cnt, tot)
            covered = float(cnt.sum())
            if self.conf_strategy == "confEntropy":
                p = cnt / max(covered, 1)
                conf = 1.0 - float(_plogp_sum(p)) / math.log(C)
            else:
                conf = float(cnt[consequent]) / max(covered, 1)
            out[name] = {"support": covered / float(tot), "confidence": conf, "count": covered}
        return out


def kolmogorov_smirnov_drift(ref_hist: torch.Tensor, cur_hist: torch.Tensor, c: float = 1.36) -> tuple[float, float, bool]:
    """KS statistic between two histograms over identical bins and the critical value
    c * sqrt((n1+n2)/(n1 n2)) (S/explore/KolmogorovSmirnovModelDrift.scala:57-76)."""
    r, q = ref_hist.double(), cur_hist.double()
    n1, n2 = float(r.sum()), float(q.sum())
    ks = float((torch.cumsum(r, -1) / n1 - torch.cumsum(q, -1) / n2).abs().max())
    crit = c * math.sqrt((n1 + n2) / (n1 * n2))
    return ks, crit, ks > crit


def event_time_distribution(epoch_s: torch.Tensor, unit: str = "hourOfDay", tz_offset_s: int = 0) -> torch.Tensor:
    """Histogram of event hour-of-day (24) or day-of-week (7) (S/sequence/EventTimeDistribution)."""
    t = epoch_s.long() + tz_offset_s
    if unit == "hourOfDay":
        return torch.bincount((t // 3600) % 24, minlength=24)
    if unit == "dayOfWeek":
        return torch.bincount(((t // 86400) + 3) % 7, minlength=7)  # 1970-01-01 was a Thursday
    raise ValueError(unit)


def numeric_histogram(x: torch.Tensor, bin_width: float, lo: float | None = None, n_bins: int | None = None):
    """Fixed-width histogram (P/lib/stats.py Histogram): (counts, lo)."""
    x = x[~torch.isnan(x)].double()
    lo = float(x.min()) if lo is None else lo
    b = torch.floor((x - lo) / bin_width).long()
    nb = int(b.max()) + 1 if n_bins is None else n_bins
    return torch.bincount(b.clamp(0, nb - 1), minlength=nb), lo
