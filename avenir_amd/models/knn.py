"""k-nearest-neighbour classification / regression (``J/knn``).

Reference pipeline (``resource/knn.sh``): an external all-pairs distance job -> Bayesian
feature-posterior job -> reduce-side join -> ``NearestNeighbor`` reducer that takes the top
``nen.top.match.count`` neighbours per test record and scores classes with a kernel
(``none`` / ``linearMultiplicative`` / ``linearAdditive`` / ``gaussian``), optional class-conditional
weighting by the neighbour's Naive Bayes feature posterior, optional inverse-distance weighting,
a positive-class decision threshold, cost-based arbitration, or regression by
average / median / simple linear regression (``J/knn/NearestNeighbor.java:317-406``,
``J/knn/Neighborhood.java:150-337``).

Here the whole pipeline runs in one process: mixed-type records are embedded so the MFMA distance
kernel applies (``ops.distance.encode_mixed``), the fused distance + top-k kernel returns the k
neighbours without materialising distances, and the kernel-weighted vote is a handful of batched
tensor ops.  Multi-GPU: training shards travel the ring (``distributed_knn``).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .. import _native
from ..ops import distance as dist
from ..parallel.comm import Comm, get_comm
from ..utils.metrics import ConfusionMatrix, Counters

KERNEL_SCALE = 1000.0
_VOTE_KERNELS = {"none": 0, "linearMultiplicative": 1, "linearAdditive": 2, "gaussian": 3}


@dataclass
class KnnResult:
    pred: torch.Tensor             # class index [n] (classification) or value [n] (regression)
    class_scores: torch.Tensor | None   # [n, C] kernel-weighted class scores
    class_prob: torch.Tensor | None     # [n, C] integer-percent-style probabilities (0..100)
    neighbors: torch.Tensor        # [n, k] neighbour indices (global)
    distances: torch.Tensor        # [n, k]


class NearestNeighbor:
    def __init__(self, k: int = 5, kernel: str = "none", kernel_param: float = 30.0,
                 metric: str = "euclidean", distance_scale: float = KERNEL_SCALE,
                 class_cond_weighted: bool = False, inverse_distance_weighted: bool = False,
                 decision_threshold: float = -1.0, positive_class: int = 1,
                 regression: str | None = None, comm: Comm | None = None):
        self.k = k
        self.kernel = kernel
        self.kernel_param = kernel_param
        self.metric = metric
        self.scale = distance_scale
        self.class_cond_weighted = class_cond_weighted
        self.inverse_distance_weighted = inverse_distance_weighted
        self.decision_threshold = decision_threshold
        self.positive_class = positive_class
        self.regression = regression
        self.comm = comm
        self.counters = Counters()

    @classmethod
    def from_config(cls, cfg) -> "NearestNeighbor":
        """``nen.``-prefixed keys (resource/knn.properties)."""
        return cls(k=cfg.get_int("top.match.count", 5), kernel=cfg.get_str("kernel.function", "none"),
                   kernel_param=cfg.get_float("kernel.param", 30.0),
                   class_cond_weighted=cfg.get_bool("class.condtion.weighted", False),
                   inverse_distance_weighted=cfg.get_bool("inverse.distance.weighted", False),
                   decision_threshold=cfg.get_float("decision.threshold", -1.0),
                   regression=cfg.get_str("regression.method", None)
                   if cfg.get_str("prediction.mode", "classification") == "regression" else None)

    def fit(self, X: torch.Tensor, y: torch.Tensor, n_classes: int | None = None,
            feature_post_prob: torch.Tensor | None = None, index_base: int = 0) -> "NearestNeighbor":
        """Training vectors (this rank's shard), labels (class index or regression target), optional
        per-training-record feature posterior (class-conditional weighting, from NaiveBayes)."""
        self.X = X.float().contiguous()
        self.y = y
        self.n_classes = n_classes or (int(y.max()) + 1 if y.numel() else 1)
        self.post = feature_post_prob
        self.index_base = index_base
        self.Xc = self.wc = None
        return self

    def fit_mixed(self, Xn: torch.Tensor, Xc: torch.Tensor, wc: torch.Tensor, y: torch.Tensor,
                  n_classes: int | None = None, index_base: int = 0) -> "NearestNeighbor":
        """Mixed-type training records: numeric block ``Xn`` [n, Dn] (already scaled), categorical
        codes ``Xc`` int [n, Dc] (-1 missing) with per-column mismatch weights ``wc``.  Queries
        then pass their own ``Qc``; distances run in ``mixed_knn_kernel`` (no one-hot matrix)."""
        self.fit(Xn, y, n_classes, index_base=index_base)
        self.Xc, self.wc = Xc.int().contiguous(), wc.float().contiguous()
        return self

    def _kernel_scores(self, d: torch.Tensor) -> torch.Tensor:
        ds = d * self.scale
        kf = self.kernel
        if kf == "none":
            s = torch.ones_like(ds)
        elif kf == "linearMultiplicative":
            s = torch.where(ds == 0, torch.full_like(ds, 2 * KERNEL_SCALE), KERNEL_SCALE / ds.clamp_min(1e-9))
        elif kf == "linearAdditive":
            s = KERNEL_SCALE - ds
        elif kf == "gaussian":
            tmp = ds / self.kernel_param
            s = KERNEL_SCALE * torch.exp(-0.5 * tmp * tmp)
        else:
            raise ValueError(f"unknown kernel function {kf}")
        if self.inverse_distance_weighted:
            s = s / ds.clamp_min(1.0)
        return torch.where(torch.isinf(d), torch.zeros_like(s), s)

    def kneighbors(self, Q: torch.Tensor, exclude_self: bool = False, q_base: int = 0, Qc: torch.Tensor | None = None):
        comm = self.comm or get_comm()
        if getattr(self, "Xc", None) is not None:
            if Qc is None or exclude_self:
                raise ValueError("mixed-type kNN needs the queries' categorical codes (and no exclude_self)")
            return dist.distributed_knn_mixed(Q.float(), Qc, self.X, self.Xc, self.wc, self.k, comm,
                                              r_base=self.index_base)
        if comm.is_distributed:
            # y / posterior of remote shards are gathered once (labels are tiny next to vectors)
            return dist.distributed_knn(Q.float(), self.X, self.k, comm, self.metric, r_base=self.index_base,
                                        q_base=q_base, exclude_self=exclude_self)
        return dist.knn(Q.float(), self.X, self.k, self.metric, exclude_self=exclude_self, q_base=q_base,
                        r_base=self.index_base)

    def _global_labels(self):
        comm = self.comm or get_comm()
        if not comm.is_distributed:
            return self.y, self.post
        ys = comm.all_gather_v(self.y)
        ps = comm.all_gather_v(self.post) if self.post is not None else None
        return ys, ps

    def predict(self, Q: torch.Tensor, exclude_self: bool = False, q_base: int = 0,
                Qc: torch.Tensor | None = None) -> KnnResult:
        d, idx = self.kneighbors(Q, exclude_self, q_base, Qc)
        ys, ps = self._global_labels()
        valid = idx >= 0
        gi = idx.clamp_min(0)
        ny = ys[gi]
        if self.regression:
            v = ny.float()
            if self.regression == "average":
                pred = (v * valid).sum(1) / valid.sum(1).clamp_min(1)
            elif self.regression == "median":
                vv = torch.where(valid, v, torch.full_like(v, float("nan")))
                pred = torch.nanquantile(vv, 0.5, dim=1)
            elif self.regression == "linearRegression":
                # simple regression of target on distance (Neighborhood.doRegression)
                x = d.float()
                m = valid.float()
                nx = m.sum(1).clamp_min(1)
                mx = (x * m).sum(1) / nx
                my = (v * m).sum(1) / nx
                sxy = ((x - mx.unsqueeze(1)) * (v - my.unsqueeze(1)) * m).sum(1)
                sxx = (((x - mx.unsqueeze(1)) ** 2) * m).sum(1).clamp_min(1e-12)
                pred = my - (sxy / sxx) * mx  # predict at distance 0
            else:
                raise ValueError(f"unknown regression method {self.regression}")
            return KnnResult(pred, None, None, idx, d)
        C = self.n_classes
        kern = _VOTE_KERNELS.get(self.kernel)
        if Q.is_cuda and C <= 64 and kern is not None and (
                not self.class_cond_weighted or (ps is not None and (ps.dim() == 1 or ps.shape[1] == C))):
            # K10: one launch for kernel weights, class-conditional weights, class sums, percent
            # probabilities and the decision (knn_vote_kernel in distance.hip)
            post = ps.float().contiguous() if self.class_cond_weighted else None
            scores, prob, pred = _native.C().knn_vote(
                d.float().contiguous(), idx.contiguous(), ys.long().contiguous(), post, int(C), kern,
                float(self.kernel_param), float(self.scale), float(KERNEL_SCALE),
                bool(self.inverse_distance_weighted),
                float(self.decision_threshold) if C == 2 else -1.0, int(self.positive_class))
            return KnnResult(pred, scores, prob, idx, d)
        s = self._kernel_scores(d) * valid
        if self.class_cond_weighted:
            if ps is None:
                raise ValueError("class conditional weighting needs feature posterior probabilities")
            s = s * ps[gi].float().gather(2, ny.long().clamp(0, C - 1).unsqueeze(2)).squeeze(2) if ps.dim() == 2 and ps.shape[1] == C \
                else s * ps[gi].float()
        scores = torch.zeros((Q.shape[0], C), dtype=torch.float32, device=Q.device)
        scores.scatter_add_(1, ny.long().clamp(0, C - 1), s.float())
        total = scores.sum(1, keepdim=True)
        prob = torch.where(total > 0, scores * 100.0 / torch.where(total > 0, total, torch.ones_like(total)),
                           torch.zeros_like(scores))
        if self.decision_threshold > 0 and C == 2:
            pos = self.positive_class
            ratio = scores[:, pos] / scores[:, 1 - pos].clamp_min(1e-12)
            pred = torch.where(ratio > self.decision_threshold, torch.full_like(ratio, pos),
                               torch.full_like(ratio, 1 - pos)).long()
        else:
            pred = scores.argmax(1)
        return KnnResult(pred, scores, prob, idx, d)

    def validate(self, Q: torch.Tensor, y_true: torch.Tensor, neg: str = "0", pos: str = "1") -> Counters:
        r = self.predict(Q)
        cm = ConfusionMatrix(neg, pos)
        p, a = r.pred.long().cpu(), y_true.long().cpu()
        P = self.positive_class
        cm.add_counts(int(((p == P) & (a == P)).sum()), int(((p == P) & (a != P)).sum()),
                      int(((p != P) & (a != P)).sum()), int(((p != P) & (a == P)).sum()))
        cm.to_counters(self.counters)
        return self.counters
