"""Naive Bayes: distributed training + batched inference (the first end-to-end slice).

Reference components (behaviour, not code):

* ``BayesianDistribution`` (MR) — per record x feature emits ``(class, featOrd, bin) -> 1`` and
  ``(class, featOrd) -> (1, v, v^2)`` for continuous features; the reducer writes feature
  posterior, class prior and feature prior lines (``J/bayesian/BayesianDistribution.java:137-178,
  :263-327``).  Here: ONE fused K2 histogram launch per rank over the device-resident columns,
  one deterministic moments launch, then ONE all-reduce of the ``[C, TB]`` counts and the
  ``[C, Fc, 3]`` moments over RCCL.
* ``BayesianModel`` / ``FeaturePosterior`` — probability tables (``J/bayesian/BayesianModel.java:
  50-74, :217-233``).  Here: log-probability tensors staged in LDS by the inference kernel.
* ``BayesianPredictor`` (map-only) — ``P(f|c) P(c) / P(f)`` in integer percent, default (max) or
  cost-based arbitration, optional "classified/ambiguous" margin, Validation counters
  (``J/bayesian/BayesianPredictor.java:227-421``).  Here: one inference kernel launch that also
  accumulates the confusion matrix; counters are all-reduced once.

The reference's text model layout is kept for interchange: ``class,featOrd,bin,count`` (feature
posterior), ``class,,,count`` (class prior), ``,featOrd,bin,count`` (feature prior),
``class,featOrd,,mean,stdDev`` / ``,featOrd,,mean,stdDev`` (continuous).
"""
from __future__ import annotations

import itertools
import math
import os
from dataclasses import dataclass
from pathlib import Path

import torch

from .. import _native
from ..data.table import Table
from ..ops import histogram as H
from ..parallel.comm import Comm, get_comm
from ..utils.metrics import ConfusionMatrix, Counters
from ..utils.schema import FeatureSchema
from ..utils.tracing import traced

_LOG_FLOOR = math.log(1e-12)
# AVMI_NB_OVERLAP=0 keeps the multi-GPU all-reduce on the caller's stream
_OVERLAP_REDUCE = os.environ.get("AVMI_NB_OVERLAP", "1") != "0"
_SIDE_STREAMS: dict = {}


def _side_stream(device: torch.device):
    """One side stream per device for the model-reduce work of multi-GPU fits."""
    key = torch.device(device).index
    st = _SIDE_STREAMS.get(key)
    if st is None:
        st = _SIDE_STREAMS[key] = torch.cuda.Stream(device=device)
    return st


@dataclass
class NBPrediction:
    pred: torch.Tensor           # int32 [n] predicted class code
    prob: torch.Tensor | None    # float32 [n, C] posterior (normalised) or reference ratio
    confusion: torch.Tensor | None  # int64 [C, C] (actual, predicted)


class NaiveBayes:
    def __init__(self, schema: FeatureSchema | None = None, laplace: float = 0.0,
                 comm: Comm | None = None):
        self.schema = schema
        self.laplace = float(laplace)
        self.comm = comm
        self.counts: torch.Tensor | None = None      # int64 [C, TB]
        self.class_n: torch.Tensor | None = None     # int64 [C]
        self.moments: torch.Tensor | None = None     # f64 [C, Fc, 3]
        self.bins: list[int] = []
        self.binned_ordinals: list[int] = []
        self.numeric_ordinals: list[int] = []
        self.class_values: list[str] = []
        self.counters = Counters()
        self._tables: dict | None = None
        self._ready = None            # event after the side-stream all-reduce / finalize (GPU, >1 rank)
        self._side = None
        self._comm = None             # the communicator of a side-stream (unchecked) reduce

    # The model tensors are read through properties: when the all-reduce of a multi-GPU fit runs on
    # the side stream, the first read on another stream waits for it (see _reduce_on_side_stream).
    @property
    def counts(self):
        self._wait()
        return self._counts

    @counts.setter
    def counts(self, v):
        self._counts = v

    @property
    def class_n(self):
        self._wait()
        return self._class_n

    @class_n.setter
    def class_n(self, v):
        self._class_n = v

    @property
    def moments(self):
        self._wait()
        return self._moments

    @moments.setter
    def moments(self, v):
        self._moments = v

    def _wait(self) -> None:
        """Make the current stream wait for a pending side-stream reduce / finalize, and mark the
        model tensors as used on it (the caching allocator must not recycle them early)."""
        ev = self.__dict__.get("_ready")
        if ev is None:
            return
        self._ready = None
        comm = self.__dict__.get("_comm")
        if comm is not None:
            comm.check(block=False)       # raise now if a finished p2p sum of this fit failed
        cur = torch.cuda.current_stream(self._both.device)
        cur.wait_event(ev)
        ts = [self._both, self._moments] + (list(self._tables.values()) if self._tables else [])
        for t in ts:
            if t is not None and t.is_cuda and t.numel():
                t.record_stream(cur)

    def _reduce_on_side_stream(self, comm: Comm, both: torch.Tensor, moments: torch.Tensor) -> None:
        """Multi-GPU fit on the GPU: the RCCL all-reduce (and later the finalize of tables()) is
        issued on a per-device side stream that waits for this step's histogram, so the caller's
        stream is free to start the NEXT histogram while the collective runs — the collective
        overlaps compute instead of sitting between steps.  Any read of the model (properties,
        tables consumers, predict) waits on the recorded event first."""
        main = torch.cuda.current_stream(both.device)
        side = _side_stream(both.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            # unchecked (asynchronous) on the peer-mapped path: a failed wait surfaces at the
            # communicator's next collective, at the first host read of the model, or at the output
            # gate of a job (Comm.check)
            comm.all_reduce(both, checked=False)
            if moments.numel():
                comm.all_reduce(moments, checked=False)
        self._comm = comm
        both.record_stream(side)
        if moments.numel():
            moments.record_stream(side)
        self._side = side
        ev = torch.cuda.Event()
        ev.record(side)
        self._ready = ev

    # ----------------------------------------------------------------------------------------
    # training
    # ----------------------------------------------------------------------------------------
    @traced("nb.fit", nbytes=lambda self, t, *a, **k: t.n * (t.codes.shape[0] + 1), device=lambda self, t, *a, **k: t.device)
    def fit(self, t: Table, reduce: bool = True) -> "NaiveBayes":
        """Count on this rank's shard, then all-reduce across ranks."""
        comm = self.comm or get_comm()
        self.bins = t.bins
        self.binned_ordinals = [f.ordinal for f in t.binned_fields]
        self.numeric_ordinals = [f.ordinal for f in t.numeric_fields]
        self.class_values = list(t.class_field.cardinality) if t.class_field else ["_"]
        C = t.n_classes
        # one fused launch: [C, TB] feature counts + a class-count column (no host sync)
        rp = self._packed(t)
        if rp is not None:
            both = H.class_histogram_packed(rp, count_labels=True)
        else:
            both = H.class_histogram(t.codes, t.n, self.bins, t.labels, C, count_labels=True)
        moments = H.class_moments(t.numeric, t.n, t.labels, C)
        self._ready, self._side = None, None
        if reduce and comm.is_distributed:
            if both.is_cuda and _OVERLAP_REDUCE and comm.backend != "gloo":
                self._reduce_on_side_stream(comm, both, moments)
            else:
                comm.all_reduce(both)
                if moments.numel():
                    comm.all_reduce(moments)
        self._both = both
        self.counts, self.class_n = both[:, :-1], both[:, -1]
        self.moments = moments
        self._tables = None
        if both.is_cuda and self.bins:
            # the model IS the tables: one fused finalize launch, queued behind the counts (on the
            # side stream when the all-reduce runs there, so it never blocks the caller's stream)
            if self._ready is not None:
                ev = self._ready
                with torch.cuda.stream(self._side):
                    self._side.wait_event(ev)
                    self._tables_impl(None)
                ev2 = torch.cuda.Event()
                ev2.record(self._side)
                self._ready = ev2
            else:
                self._tables_impl(None)
        return self

    def _packed(self, t: Table):
        """The table's row-packed records when they describe exactly these rows and bins."""
        rp = getattr(t, "rowpack", None)
        if rp is not None and rp.n == t.n and rp.n_classes == t.n_classes and rp.bins == self.bins:
            return rp
        return None

    def partial_fit(self, t: Table) -> "NaiveBayes":
        """Accumulate more data (streaming / out-of-core).  Call ``reduce()`` once at the end."""
        if self.counts is None:
            return self.fit(t, reduce=False)
        rp = self._packed(t)
        if rp is not None:
            H.class_histogram_packed(rp, out=self._both, count_labels=True)
        else:
            H.class_histogram(t.codes, t.n, self.bins, t.labels, t.n_classes, out=self._both,
                              count_labels=True)
        self.moments += H.class_moments(t.numeric, t.n, t.labels, t.n_classes)
        self._tables = None
        return self

    def reduce(self) -> "NaiveBayes":
        comm = self.comm or get_comm()
        if comm.is_distributed:
            comm.all_reduce(self._both)
            if self.moments.numel():
                comm.all_reduce(self.moments)
        self._tables = None
        return self

    # ----------------------------------------------------------------------------------------
    # probability tables
    # ----------------------------------------------------------------------------------------
    @property
    def n_classes(self) -> int:
        return int(self.counts.shape[0])

    def class_counts(self) -> torch.Tensor:
        """Records per class (the class prior counts)."""
        return self.class_n

    def tables(self, device=None) -> dict:
        """Log-probability tables (cached; a GPU fit computes them eagerly — see fit)."""
        if self._tables is not None and (device is None or self._tables["logp"].device == torch.device(device)):
            self._wait()
            return self._tables
        self._wait()
        return self._tables_impl(device)

    def _tables_impl(self, device=None) -> dict:
        dev = torch.device(device) if device is not None else self.counts.device
        a = self.laplace
        if dev.type == "cuda" and self._both is not None and self._both.device == dev and self.bins:
            # one fused launch (bayes.hip nb_finalize) instead of ~40 small ops
            offs = H._dev_i32(list(itertools.accumulate([0] + list(self.bins[:-1]))), dev)
            bins = H._dev_i32(list(self.bins), dev)
            logp, logfp, logprior = _native.C().nb_finalize(self._both.contiguous(), offs, bins, int(sum(self.bins)),
                                                             float(a), float(_LOG_FLOOR))
        else:
            cnt = self.counts.double().to(dev)
            C, TB = cnt.shape
            logp = torch.empty((C, TB), dtype=torch.float64, device=dev)
            logfp = torch.empty((TB,), dtype=torch.float64, device=dev)
            o = 0
            for b in self.bins:
                blk = cnt[:, o:o + b] + a
                logp[:, o:o + b] = torch.log(blk / blk.sum(1, keepdim=True).clamp_min(1e-300))
                pri = cnt[:, o:o + b].sum(0) + a
                logfp[o:o + b] = torch.log(pri / pri.sum().clamp_min(1e-300))
                o += b
            logp = torch.nan_to_num(logp, nan=_LOG_FLOOR).clamp_min(_LOG_FLOOR)
            logfp = torch.nan_to_num(logfp, nan=_LOG_FLOOR).clamp_min(_LOG_FLOOR)
            cc = self.class_counts().double().to(dev)
            logprior = torch.log((cc / cc.sum().clamp_min(1)).clamp_min(1e-300)).clamp_min(_LOG_FLOOR)
        if self.moments.numel() == 0:
            e = torch.zeros((self.n_classes, 0), device=dev)
            ep = torch.zeros((0,), device=dev)
            self._tables = {"logp": logp.float().contiguous(), "logfp": logfp.float().contiguous(),
                            "logprior": logprior.float().contiguous(), "gmean": e, "ginvstd": e, "glognorm": e,
                            "pmean": ep, "pinvstd": ep, "plognorm": ep}
            return self._tables
        # Gaussian parameters of continuous features (sample std, like the reference reducer)
        m = self.moments.to(dev)
        n_, s_, q_ = m[..., 0], m[..., 1], m[..., 2]
        mean = s_ / n_.clamp_min(1)
        var = ((q_ - n_ * mean * mean) / (n_ - 1).clamp_min(1)).clamp_min(1e-12)
        std = var.sqrt()
        pn, ps, pq = n_.sum(0), s_.sum(0), q_.sum(0)
        pmean = ps / pn.clamp_min(1)
        pstd = ((pq - pn * pmean * pmean) / (pn - 1).clamp_min(1)).clamp_min(1e-12).sqrt()
        half_log_2pi = 0.5 * math.log(2 * math.pi)
        self._tables = {
            "logp": logp.float().contiguous(), "logfp": logfp.float().contiguous(),
            "logprior": logprior.float().contiguous(),
            "gmean": mean.float().contiguous(), "ginvstd": (1.0 / std).float().contiguous(),
            "glognorm": (-torch.log(std) - half_log_2pi).float().contiguous(),
            "pmean": pmean.float().contiguous(), "pinvstd": (1.0 / pstd).float().contiguous(),
            "plognorm": (-torch.log(pstd) - half_log_2pi).float().contiguous(),
        }
        return self._tables

    # ----------------------------------------------------------------------------------------
    # inference
    # ----------------------------------------------------------------------------------------
    @traced("nb.predict", nbytes=lambda self, t, *a, **k: t.n * (t.codes.shape[0] + 1), device=lambda self, t, *a, **k: t.device)
    def predict(self, t: Table, ref_scale: bool = False, with_prob: bool = True,
                validate: bool = True) -> NBPrediction:
        tb = self.tables(t.device)
        C = self.n_classes
        n = t.n
        offs = H._dev_i32(t.offsets, t.device)
        pred = torch.empty((max(n, 1),), dtype=torch.int32, device=t.device)
        post = torch.empty((max(n, 1), C), dtype=torch.float32, device=t.device) if with_prob else None
        conf = (torch.zeros((C, C), dtype=torch.int64, device=t.device)
                if validate and t.labels is not None else None)
        has_x = t.numeric.shape[0] > 0
        if t.device.type == "cuda" and not t.wide:
            _native.C().nb_predict(t.codes, n, offs, tb["logp"], tb["logfp"],
                                   t.numeric if has_x else None,
                                   tb["gmean"] if has_x else None, tb["ginvstd"] if has_x else None,
                                   tb["glognorm"] if has_x else None, tb["pmean"] if has_x else None,
                                   tb["pinvstd"] if has_x else None, tb["plognorm"] if has_x else None,
                                   tb["logprior"], bool(ref_scale), post, pred, t.labels, conf)
        elif t.device.type == "cuda" and C <= 32:
            # wide (uint16 / int32 code) tables: transposed model read through L2 (bayes.hip)
            if "logpT" not in tb:
                tb["logpT"] = tb["logp"].T.contiguous()
            _native.C().nb_predict_wide(t.codes.contiguous(), n, offs, H._dev_i32(t.bins, t.device), tb["logpT"],
                                        tb["logfp"], t.numeric if has_x else None,
                                        tb["gmean"] if has_x else None, tb["ginvstd"] if has_x else None,
                                        tb["glognorm"] if has_x else None, tb["pmean"] if has_x else None,
                                        tb["pinvstd"] if has_x else None, tb["plognorm"] if has_x else None,
                                        tb["logprior"], bool(ref_scale), post, pred, t.labels, conf)
        else:   # CPU oracle (and > 32 classes on the GPU, as batched torch gathers)
            self._predict_ref(t, tb, ref_scale, post, pred, conf)
        return NBPrediction(pred[:n], None if post is None else post[:n], conf)

    def _predict_ref(self, t: Table, tb: dict, ref_scale: bool, post, pred, conf) -> None:
        n, C = t.n, self.n_classes
        s = tb["logprior"].view(1, C).expand(n, C).clone()
        lfp = torch.zeros(n, device=s.device)
        zero = torch.zeros(1, device=s.device)
        o = 0
        for f, b in enumerate(self.bins):
            v = t.codes[f, :n].long()
            ok = v < b
            vv = torch.where(ok, v, torch.zeros_like(v)) + o
            s += torch.where(ok.unsqueeze(1), tb["logp"][:, vv].T, zero)
            lfp += torch.where(ok, tb["logfp"][vv], zero)
            o += b
        if t.numeric.shape[0]:
            x = t.numeric[:, :n].T  # [n, Fc]
            z = (x.unsqueeze(1) - tb["gmean"].unsqueeze(0)) * tb["ginvstd"].unsqueeze(0)
            s += (tb["glognorm"].unsqueeze(0) - 0.5 * z * z).sum(2)
            zp = (x - tb["pmean"]) * tb["pinvstd"]
            lfp += (tb["plognorm"] - 0.5 * zp * zp).sum(1)
        pred[:n] = torch.argmax(s, 1).int()
        if post is not None:
            post[:n] = torch.exp(s - lfp.unsqueeze(1)) if ref_scale else torch.softmax(s, 1)
        if conf is not None:
            a = t.labels[:n].long()
            ok = a < C
            conf += torch.bincount(a[ok] * C + pred[:n].long()[ok], minlength=C * C).view(C, C)

    def feature_loglik(self, t: Table) -> tuple[torch.Tensor, torch.Tensor]:
        """Per-row, per-feature, per-class log-likelihood terms ``[n, Fcat + Fnum, C]`` and class
        log-priors — the decomposition the feature-subset optimiser scores subsets with (a subset's
        posterior score is the masked sum over the feature axis)."""
        tb = self.tables(t.device)
        n, C = t.n, self.n_classes
        cols = []
        o = 0
        for f, b in enumerate(self.bins):
            v = t.codes[f, :n].long()
            ok = v < b
            vv = torch.where(ok, v, torch.zeros_like(v)) + o
            cols.append(torch.where(ok.unsqueeze(1), tb["logp"][:, vv].T, torch.zeros((), device=t.device)))
            o += b
        if t.numeric.shape[0]:
            x = t.numeric[:, :n].T
            z = (x.unsqueeze(1) - tb["gmean"].unsqueeze(0)) * tb["ginvstd"].unsqueeze(0)   # [n, C, Fc]
            g = tb["glognorm"].unsqueeze(0) - 0.5 * z * z
            cols.extend(g[:, :, j] for j in range(g.shape[2]))
        return torch.stack(cols, 1), tb["logprior"]

    def feature_probs(self, t: Table) -> tuple[torch.Tensor, torch.Tensor]:
        """(feature prior probability P(f) [n], feature posterior P(f|c) [n, C]) per record — the
        ``bap.output.feature.prob.only`` output (BayesianPredictor.java:271-285, BayesianModel
        ``getFeaturePriorProb`` / ``getFeaturePostProb``: products over the features)."""
        terms, _ = self.feature_loglik(t)                       # [n, F, C]
        tb = self.tables(t.device)
        n = t.n
        lfp = torch.zeros(n, device=t.device)
        o = 0
        for f, b in enumerate(self.bins):
            v = t.codes[f, :n].long()
            ok = v < b
            lfp += torch.where(ok, tb["logfp"][torch.where(ok, v, torch.zeros_like(v)) + o], torch.zeros((), device=t.device))
            o += b
        if t.numeric.shape[0]:
            zp = (t.numeric[:, :n].T - tb["pmean"]) * tb["pinvstd"]
            lfp += (tb["plognorm"] - 0.5 * zp * zp).sum(1)
        return torch.exp(lfp.double()), torch.exp(terms.double().sum(1))

    def validation_counters(self, conf: torch.Tensor, comm: Comm | None = None,
                            pos_class: int = 1) -> Counters:
        """Reference "Validation" counter group from an (all-reduced) confusion matrix."""
        comm = comm or self.comm or get_comm()
        conf = conf.clone()
        if comm.is_distributed:
            comm.all_reduce(conf)
        c = conf.cpu()
        cm = ConfusionMatrix(self.class_values[0], self.class_values[min(pos_class, len(self.class_values) - 1)])
        if c.shape[0] >= 2:
            cm.add_counts(tp=int(c[pos_class, pos_class]), fp=int(c[:, pos_class].sum() - c[pos_class, pos_class]),
                          tn=int(c.sum() - c[pos_class, :].sum() - c[:, pos_class].sum() + c[pos_class, pos_class]),
                          fn=int(c[pos_class, :].sum() - c[pos_class, pos_class]))
        cm.to_counters(self.counters)
        self.counters.set("Validation", "Correct", int(torch.diag(c).sum()))
        self.counters.set("Validation", "Incorrect", int(c.sum() - torch.diag(c).sum()))
        return self.counters

    @staticmethod
    def arbitrate_cost(prob_pct: torch.Tensor, fp_cost: float, fn_cost: float, pos: int = 1) -> torch.Tensor:
        """Cost-based arbitration (``J/util/CostBasedArbitrator.java:50-64``): predict positive when
        the expected cost of a false negative exceeds that of a false positive."""
        pos_p = prob_pct[:, pos].float()
        neg_p = prob_pct[:, 1 - pos].float()
        return (pos_p * fn_cost > neg_p * fp_cost).int() * pos + (pos_p * fn_cost <= neg_p * fp_cost).int() * (1 - pos)

    # ----------------------------------------------------------------------------------------
    # reference text model I/O
    # ----------------------------------------------------------------------------------------
    def model_lines(self, delim: str = ",") -> list[str]:
        schema = self.schema
        cnt = self.counts.cpu()
        lines: list[str] = []
        o = 0
        for f, (ordn, b) in enumerate(zip(self.binned_ordinals, self.bins)):
            field = schema.find_field_by_ordinal(ordn) if schema else None
            for c, cv in enumerate(self.class_values):
                for k in range(b):
                    v = int(cnt[c, o + k])
                    if v:
                        lab = field.bin_label(k) if field else str(k)
                        lines.append(delim.join([cv, str(ordn), lab, str(v)]))
            for k in range(b):
                v = int(cnt[:, o + k].sum())
                if v:
                    lab = field.bin_label(k) if field else str(k)
                    lines.append(delim.join(["", str(ordn), lab, str(v)]))
            o += b
        cc = self.class_counts().cpu()
        for c, cv in enumerate(self.class_values):
            lines.append(delim.join([cv, "", "", str(int(cc[c]))]))
        if self.numeric_ordinals:
            m = self.moments.cpu()
            for j, ordn in enumerate(self.numeric_ordinals):
                for c, cv in enumerate(self.class_values):
                    n_, s_, q_ = (float(x) for x in m[c, j])
                    mean = s_ / max(n_, 1)
                    std = math.sqrt(max(q_ - n_ * mean * mean, 0) / max(n_ - 1, 1))
                    lines.append(delim.join([cv, str(ordn), "", f"{mean:.6g}", f"{std:.6g}"]))
                n_, s_, q_ = (float(x) for x in m[:, j].sum(0))
                mean = s_ / max(n_, 1)
                std = math.sqrt(max(q_ - n_ * mean * mean, 0) / max(n_ - 1, 1))
                lines.append(delim.join(["", str(ordn), "", f"{mean:.6g}", f"{std:.6g}"]))
        return lines

    def save_model(self, path: str | Path, delim: str = ",") -> None:
        Path(path).write_text("\n".join(self.model_lines(delim)) + "\n")

    @classmethod
    def load_model(cls, path: str | Path, schema: FeatureSchema, delim: str = ",",
                   comm: Comm | None = None, device="cpu") -> "NaiveBayes":
        """Load a reference-format model (ours or the Java job's ``part-r-00000``)."""
        nb = cls(schema, comm=comm)
        cls_f = schema.find_class_attr_field()
        nb.class_values = list(cls_f.cardinality)
        feats = schema.feature_fields
        binned = [f for f in feats if f.is_binned]
        numeric = [f for f in feats if not f.is_binned and f.is_numeric]
        nb.bins = [f.num_bins for f in binned]
        nb.binned_ordinals = [f.ordinal for f in binned]
        nb.numeric_ordinals = [f.ordinal for f in numeric]
        offs = {}
        o = 0
        for f in binned:
            offs[f.ordinal] = (o, f)
            o += f.num_bins
        C = len(nb.class_values)
        counts = torch.zeros((C, o), dtype=torch.int64)
        moments = torch.zeros((C, len(numeric), 3), dtype=torch.float64)
        cprior = torch.zeros(C, dtype=torch.int64)
        num_idx = {f.ordinal: j for j, f in enumerate(numeric)}
        for line in Path(path).read_text().splitlines():
            if not line.strip():
                continue
            it = line.split(delim)
            while len(it) < 5:
                it.append("")
            if it[0] == "":
                continue  # feature prior lines are derivable from the posteriors
            c = nb.class_values.index(it[0])
            if it[1] == "" and it[2] == "":
                cprior[c] += int(it[3])
                continue
            ordn = int(it[1])
            if it[2] != "":
                base, f = offs[ordn]
                if f.is_categorical:
                    k = f.cardinality.index(it[2])
                else:
                    k = int(it[2]) - f.bucket_offset
                counts[c, base + k] += int(it[3])
            else:
                j = num_idx[ordn]
                mean, std = float(it[3]), float(it[4])
                nc = float(cprior[c]) or 1.0
                moments[c, j] = torch.tensor([nc, mean * nc, (std * std) * (nc - 1) + nc * mean * mean],
                                             dtype=torch.float64)
        # fix up moment counts now that all class priors are known
        for c in range(C):
            nc = float(cprior[c])
            if nc > 0 and moments.shape[1]:
                mean = moments[c, :, 1] / moments[c, :, 0].clamp_min(1)
                var = (moments[c, :, 2] - moments[c, :, 0] * mean * mean) / (moments[c, :, 0] - 1).clamp_min(1)
                moments[c, :, 0] = nc
                moments[c, :, 1] = mean * nc
                moments[c, :, 2] = var * (nc - 1) + nc * mean * mean
        nb._both = torch.cat([counts, cprior.view(C, 1)], 1).to(device)
        nb.counts, nb.class_n = nb._both[:, :-1], nb._both[:, -1]
        nb.moments = moments.to(device)
        return nb


def _label_counts(t: Table, C: int) -> torch.Tensor:
    if t.labels is None:
        return torch.tensor([t.n], dtype=torch.int64, device=t.device)
    lab = t.labels[: t.n]
    lab = lab[lab < C].long()
    return torch.bincount(lab, minlength=C)[:C].to(torch.int64)


# ================================================================================================
# text mode (BayesianDistribution.mapText, J/bayesian/BayesianDistribution.java:186-195)
# ================================================================================================
# Lucene StandardAnalyzer's English stop set (the tokenizer the reference uses)
_STOP = frozenset("a an and are as at be but by for if in into is it no not of on or such that the their then "
                  "there these they this to was will with".split())


def tokenize(text: str) -> list[str]:
    """Lower-case alphanumeric tokens minus the analyzer's stop words."""
    import re
    return [w for w in re.findall(r"[a-z0-9]+", text.lower()) if w not in _STOP]


class TextNaiveBayesModel:
    """Multinomial NB over word tokens: the text is one feature (ordinal 1 in the model lines) whose
    bins are the tokens.  Training counts are one ``[C, V]`` bincount over a vocabulary shared by all
    ranks, all-reduced once; lines keep the tabular model layout (``class,1,token,count``,
    ``class,,,docCount``, ``,1,token,count``)."""

    FEATURE_ORDINAL = 1

    def __init__(self, classes: list[str], vocab: list[str], counts: torch.Tensor, docs: torch.Tensor):
        self.classes, self.vocab = classes, vocab
        self.counts, self.docs = counts, docs          # int64 [C, V], int64 [C]

    @classmethod
    def fit_native(cls, ctx, class_ord: int = 1, text_ord: int = 0) -> "TextNaiveBayesModel | None":
        """``fit_lines`` over native token tables (None when the layout needs the row path): one
        ``[C, V]`` bincount of (class, word) over the shard's words, all-reduced; the vocabulary is
        the global set of text words (the merged dictionary's lowered entries that occur)."""
        got = cls.word_tokens(ctx, class_ord, text_ord)
        if got is None:
            return None
        line, wid, uniq, ccode, fields = got
        classes = ctx.union(fields.strings(torch.unique(ccode[ccode >= 0])))
        cl = fields.map_codes(ccode, classes).long().cpu()
        C, Vu = len(classes), len(uniq)
        dev = ctx.device
        counts = torch.bincount((cl[line] * Vu + wid).to(dev), minlength=C * Vu)[: C * Vu].view(C, Vu)
        docs = torch.bincount(cl.to(dev), minlength=C)[:C]
        ctx.all_reduce(counts, docs)
        used = torch.nonzero(counts.sum(0) > 0).view(-1)
        vocab = [uniq[i] for i in used.tolist()]
        return cls(classes, vocab, counts[:, used], docs)

    @classmethod
    def fit_lines(cls, lines: list[str], split, ctx, class_ord: int = 1, text_ord: int = 0) -> "TextNaiveBayesModel":
        rows = [split(l) for l in lines]
        toks = [tokenize(r[text_ord]) for r in rows]
        classes = ctx.union(r[class_ord] for r in rows)
        vocab = ctx.union(w for ts in toks for w in ts)
        ci = {c: i for i, c in enumerate(classes)}
        vi = {w: i for i, w in enumerate(vocab)}
        C, V = len(classes), len(vocab)
        cl = torch.tensor([ci[r[class_ord]] for r in rows], dtype=torch.long)
        flat_c = torch.repeat_interleave(cl, torch.tensor([len(t) for t in toks], dtype=torch.long))
        flat_w = torch.tensor([vi[w] for t in toks for w in t], dtype=torch.long)
        dev = ctx.device
        counts = torch.bincount((flat_c * V + flat_w).to(dev), minlength=C * V)[: C * V].view(C, V)
        docs = torch.bincount(cl.to(dev), minlength=C)[:C]
        ctx.all_reduce(counts, docs)
        return cls(classes, vocab, counts, docs)

    def model_lines(self, delim: str = ",") -> list[str]:
        f = self.FEATURE_ORDINAL
        cnt = self.counts.cpu()
        out = []
        for c, cv in enumerate(self.classes):
            for w in torch.nonzero(cnt[c]).view(-1).tolist():
                out.append(f"{cv}{delim}{f}{delim}{self.vocab[w]}{delim}{int(cnt[c, w])}")
        for c, cv in enumerate(self.classes):
            out.append(f"{cv}{delim}{delim}{delim}{int(self.docs[c])}")
        tot = cnt.sum(0)
        for w in torch.nonzero(tot).view(-1).tolist():
            out.append(f"{delim}{f}{delim}{self.vocab[w]}{delim}{int(tot[w])}")
        return out

    @classmethod
    def load(cls, path, split) -> "TextNaiveBayesModel":
        from ..jobs.common import read_lines
        post: dict[tuple[str, str], int] = {}
        docs: dict[str, int] = {}
        for l in read_lines(path):
            p = split(l)
            if p[0] and p[1] and p[2]:
                post[(p[0], p[2])] = int(float(p[3]))
            elif p[0] and not p[1]:
                docs[p[0]] = int(float(p[3]))
        classes = sorted(docs)
        vocab = sorted({w for _, w in post})
        ci = {c: i for i, c in enumerate(classes)}
        vi = {w: i for i, w in enumerate(vocab)}
        counts = torch.zeros((len(classes), len(vocab)), dtype=torch.long)
        for (c, w), n in post.items():
            counts[ci[c], vi[w]] = n
        return cls(classes, vocab, counts, torch.tensor([docs[c] for c in classes], dtype=torch.long))

    def predict(self, texts: list[str], alpha: float = 1.0) -> tuple[list[int], list[float]]:
        """Multinomial NB with Laplace smoothing: argmax_c log P(c) + sum_w n_w log P(w|c); the
        bag-of-words matrix times the log-probability table is one GEMM."""
        vi = {w: i for i, w in enumerate(self.vocab)}
        rows, cols = [], []
        for i, t in enumerate(texts):
            for w in tokenize(t):
                if w in vi:
                    rows.append(i)
                    cols.append(vi[w])
        pred, prob = self.predict_bow(torch.tensor(rows, dtype=torch.long), torch.tensor(cols, dtype=torch.long),
                                      len(texts), alpha)
        return pred.tolist(), prob.tolist()

    def predict_bow(self, rows: torch.Tensor, cols: torch.Tensor, n: int, alpha: float = 1.0):
        """Class index and probability tensors of ``n`` documents given as (document, word id)
        occurrence pairs (word ids into ``vocab``)."""
        C, V = self.counts.shape
        dev = self.counts.device
        bow = torch.zeros((n, V), dtype=torch.float64, device=dev)
        if rows.numel():
            bow.index_put_((rows.to(dev), cols.to(dev)), torch.ones(rows.numel(), dtype=torch.float64, device=dev),
                           accumulate=True)
        cnt = self.counts.double()
        logp = torch.log((cnt + alpha) / (cnt.sum(1, keepdim=True) + alpha * V))
        prior = torch.log(self.docs.double() / self.docs.sum().clamp_min(1)).to(dev)
        s = bow @ logp.T + prior
        p = torch.softmax(s, 1)
        best = p.max(1)
        return best.indices, best.values

    # -- native text tokens ---------------------------------------------------------------------
    @staticmethod
    def word_tokens(ctx, class_ord: int = 1, text_ord: int = 0):
        """The ``tokenize`` words of every line's text field from native token tables, or None when
        the layout is not ``text<delim>class`` with a one-character delimiter.  Returns (line of
        every word token int64, lowered word id int64, lowered word strings, class codes per line,
        class Records).  Two native passes over the shard: the fields (class codes), and the bytes
        split at every non-alphanumeric byte (the text field's words are the tokens before the
        class field's); case folding and stop words are dictionary-level."""
        dl = ctx.native_delim()
        if dl is None or text_ord != 0 or class_ord != 1 or dl.isalnum():
            return None
        fields = ctx.records(modes="xd", tail_mode="x")
        ok = torch.tensor([float(fields.width() in (0, 2))])
        if ctx.comm.is_distributed:
            ctx.comm.all_reduce(ok, "min")          # every rank takes the same path
        if not bool(ok[0] > 0):
            return None
        seps = "".join(chr(c) for c in range(1, 256) if not (chr(c).isascii() and chr(c).isalnum()))
        words = ctx.records(delims=seps, tail_mode="d")
        if words.n_lines != fields.n_lines:
            return None
        low = [w.lower() for w in words.vocab]
        uniq = sorted(set(low))
        ui = {w: i for i, w in enumerate(uniq)}
        lut = torch.tensor([ui[w] if (w and w not in _STOP) else -1 for w in low] or [-1], dtype=torch.long)
        # tokens of the class string (same split), per class code: they end every line
        import re
        cls = fields.field(1).long().cpu()
        off = words.off.cpu()
        lens = off[1:] - off[:-1]
        # the class field's pieces: every separator inside it adds a (possibly empty) token, so
        # count its separator-delimited pieces instead of its words
        pieces = torch.tensor([len(re.split("[" + re.escape(seps) + "]", v)) for v in fields.vocab] or [1],
                              dtype=torch.long)
        text_len = lens - torch.where(cls >= 0, pieces[cls.clamp_min(0)], torch.zeros_like(cls))
        codes = words.codes.long().cpu()
        line = torch.repeat_interleave(torch.arange(words.n_lines), lens)
        pos = torch.arange(codes.numel()) - off[:-1][line]
        keep = pos < text_len[line]
        wid = torch.where(codes >= 0, lut[codes.clamp_min(0)], torch.full_like(codes, -1))
        keep &= wid >= 0
        return line[keep], wid[keep], uniq, cls, fields
