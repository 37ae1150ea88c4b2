"""Distance ops (K9/K11): fused MFMA distance + top-k, ring-pass distributed kNN, cluster sums,
and the mixed-type record encoding that turns schema records into a euclidean space."""
from __future__ import annotations

import math

import torch

from .. import _native
from ..data.table import MISSING, Table
from ..utils.tracing import traced

_MFMA_METRICS = ("euclidean", "sqeuclidean", "cosine")
_KMAX = 64          # largest k of the fused kernel (register-resident sorted lists)


def _cpu_topk(Q, R, k, metric, p, exclude_self, q_base, r_base, chunk=4096):
    ds, ix = [], []
    for s in range(0, Q.shape[0], chunk):
        q = Q[s:s + chunk]
        if metric in ("sqeuclidean", "euclidean"):
            d = torch.cdist(q.double(), R.double()) ** 2
        elif metric == "cosine":
            qn = torch.nn.functional.normalize(q.double(), dim=1)
            rn = torch.nn.functional.normalize(R.double(), dim=1)
            d = (1 - qn @ rn.T).clamp_min(0)
        elif metric == "manhattan":
            d = torch.cdist(q.double(), R.double(), p=1)
        elif metric == "minkowski":
            d = torch.cdist(q.double(), R.double(), p=p)
        else:
            raise ValueError(f"unknown metric {metric}")
        if exclude_self:
            qi = torch.arange(s, s + q.shape[0], device=d.device).view(-1, 1) + q_base
            ri = torch.arange(R.shape[0], device=d.device).view(1, -1) + r_base
            d = torch.where(qi == ri, torch.full_like(d, math.inf), d)
        kk = min(k, R.shape[0])
        v, i = torch.topk(d, kk, dim=1, largest=False)
        if kk < k:
            v = torch.cat([v, torch.full((v.shape[0], k - kk), math.inf, dtype=v.dtype, device=v.device)], 1)
            i = torch.cat([i, torch.full((i.shape[0], k - kk), -1, dtype=i.dtype, device=i.device)], 1)
        i = torch.where(torch.isinf(v), torch.full_like(i, -1), i + r_base)
        ds.append(v.float())
        ix.append(i)
    return torch.cat(ds), torch.cat(ix)


@traced("knn", flops=lambda Q, R, *a, **k: 2.0 * Q.shape[0] * R.shape[0] * Q.shape[1], device=lambda Q, *a, **k: Q.device)
def knn(Q: torch.Tensor, R: torch.Tensor, k: int, metric: str = "euclidean", p: float = 2.0,
        exclude_self: bool = False, q_base: int = 0, r_base: int = 0, prec: int = -1) -> tuple[torch.Tensor, torch.Tensor]:
    """k nearest references of every query: (dist float32 [M, k] ascending, idx int64 [M, k]);
    idx = -1 / dist = inf when fewer than k candidates.  ``sqeuclidean`` returns squared distances,
    ``cosine`` returns 1 - cos.  On the GPU every metric with k <= 64 runs the fused distance +
    top-k kernel (K9); larger k use chunked device distance blocks + ``torch.topk``.  ``prec``
    (euclidean family on the GPU): -1 the process default (``AVMI_KNN_MFMA``, bf16x6), 0 fp32 MFMA,
    3 / 6 split-bf16 x3 / x6 dot products."""
    Q = Q.float().contiguous()
    R = R.float().contiguous()
    if metric == "minkowski" and p == 2.0:
        metric = "euclidean"
    elif metric == "minkowski" and p == 1.0:
        metric = "manhattan"
    kmet = {"euclidean": 0, "sqeuclidean": 0, "cosine": 0, "manhattan": 1, "minkowski": 2}.get(metric)
    if Q.is_cuda and kmet is not None and k <= _KMAX:
        # fused tile distance + top-k: MFMA dot products (euclidean family) or VALU |q - r|^p
        if metric == "cosine":
            Q = torch.nn.functional.normalize(Q, dim=1)
            R = torch.nn.functional.normalize(R, dim=1)
        d, i, splits = _native.C().knn_topk(Q, R, int(k), int(q_base), int(r_base), bool(exclude_self), 0,
                                            kmet, float(p), int(prec))
        if splits > 1:  # merge the per-split top-k slabs [S, M, k] -> [M, k]
            d = d.permute(1, 0, 2).reshape(Q.shape[0], -1)
            i = i.permute(1, 0, 2).reshape(Q.shape[0], -1)
            d, j = torch.topk(d, int(k), dim=1, largest=False)
            i = torch.gather(i, 1, j)
        else:
            d, i = d[0], i[0]
        if metric == "cosine":
            return d * 0.5, i
        if metric == "minkowski":
            return d.pow(1.0 / p), i
        return (d.sqrt() if metric == "euclidean" else d), i
    d, i = _cpu_topk(Q, R, k, "sqeuclidean" if metric == "euclidean" else metric, p, exclude_self,
                     q_base, r_base)
    return (d.sqrt() if metric == "euclidean" else d), i


def merge_topk(d1, i1, d2, i2, k):
    d = torch.cat([d1, d2], 1)
    i = torch.cat([i1, i2], 1)
    v, j = torch.topk(d, k, dim=1, largest=False)
    return v, torch.gather(i, 1, j)


def _merge_topk_by_id(d1, i1, d2, i2, k):
    """merge_topk with ties broken by the smaller global id (order-independent)."""
    d = torch.cat([d1, d2], 1)
    i = torch.cat([i1, i2], 1)
    o = torch.argsort(torch.where(i >= 0, i, torch.full_like(i, 1 << 62)), dim=1, stable=True)
    d, i = torch.gather(d, 1, o), torch.gather(i, 1, o)
    o = torch.argsort(d, dim=1, stable=True)[:, :k]
    return torch.gather(d, 1, o), torch.gather(i, 1, o)


def distributed_knn(Q: torch.Tensor, R: torch.Tensor, k: int, comm, metric: str = "euclidean",
                    r_base: int = 0, q_base: int = 0, exclude_self: bool = False, r_ids: torch.Tensor | None = None):
    """Systolic all-pairs kNN: every rank keeps its query shard and passes its reference shard
    around the ring — no bucket-pair replication.  The shard sizes are exchanged
    ONCE up front (one all-gather), so every hop's receive buffer and global index base are known on
    the host; the send/receive of the NEXT shard is posted (``Comm.ring_pass_start``) before the
    fused distance + top-k of the current one, so the transfer over xGMI overlaps the compute.
    ``r_base`` is this rank's global index offset of R (kept for the single-rank path).
    ``r_ids``: explicit global ids of R's rows (e.g. a class subset of a shard); they travel around
    the ring with the rows and are what the result indexes (``exclude_self`` not supported then)."""
    if r_ids is not None:
        return _distributed_knn_ids(Q, R, r_ids.long(), k, comm, metric)
    if not comm.is_distributed:
        return knn(Q, R, k, metric, exclude_self=exclude_self, q_base=q_base, r_base=r_base)
    best_d = torch.full((Q.shape[0], k), math.inf, device=Q.device)
    best_i = torch.full((Q.shape[0], k), -1, dtype=torch.long, device=Q.device)
    n = torch.tensor([R.shape[0]], dtype=torch.long, device=Q.device)
    sizes = comm.all_gather(n).view(-1).tolist()
    bases = [0]
    for c in sizes[:-1]:
        bases.append(bases[-1] + c)
    cur = R.contiguous()
    W, me = comm.world, comm.rank
    for step in range(W):
        owner = (me - step) % W                 # whose shard ``cur`` is
        pending = None
        if step + 1 < W:
            src = (me - step - 1) % W
            pending = comm.ring_pass_start(cur, sizes[src])
        d, i = knn(Q, cur, k, metric, exclude_self=exclude_self, q_base=q_base, r_base=bases[owner])
        best_d, best_i = merge_topk(best_d, best_i, d, i, k)
        if pending is not None:
            cur = comm.ring_pass_finish(pending)
    return best_d, best_i


def mixed_knn_max_dims() -> int:
    """Largest numeric / categorical column count of the ``mixed_knn_kernel`` (and k <= 32)."""
    try:
        return int(_native.C().mixed_knn_max_dims())
    except (AttributeError, RuntimeError, ImportError):
        return 32


def distributed_knn_mixed(Qn, Qc, Rn, Rc, wc, k: int, comm, r_base: int = 0):
    """``knn_mixed`` with the reference shards travelling the ring (as ``distributed_knn``): the
    numeric block and the categorical codes (bit-cast to float32) travel as ONE [nr, Dn + Dc]
    buffer, the next shard's transfer is posted before the current shard's kernel."""
    if not comm.is_distributed:
        return knn_mixed(Qn, Qc, Rn, Rc, wc, k, r_base)
    Dn = Rn.shape[1]
    best_d = torch.full((Qn.shape[0], k), math.inf, device=Qn.device)
    best_i = torch.full((Qn.shape[0], k), -1, dtype=torch.long, device=Qn.device)
    sizes = comm.all_gather(torch.tensor([Rn.shape[0]], dtype=torch.long, device=Qn.device)).view(-1).tolist()
    bases = [0]
    for c in sizes[:-1]:
        bases.append(bases[-1] + c)
    cur = torch.cat([Rn.float(), Rc.int().contiguous().view(torch.float32)], 1).contiguous()
    W, me = comm.world, comm.rank
    for step in range(W):
        owner = (me - step) % W
        pending = None
        if step + 1 < W:
            pending = comm.ring_pass_start(cur, sizes[(me - step - 1) % W])
        d, i = knn_mixed(Qn, Qc, cur[:, :Dn].contiguous(), cur[:, Dn:].contiguous().view(torch.int32), wc, k,
                         bases[owner])
        best_d, best_i = merge_topk(best_d, best_i, d, i.long(), k)
        if pending is not None:
            cur = comm.ring_pass_finish(pending)
    return best_d, best_i


def _distributed_knn_ids(Q, R, ids, k, comm, metric):
    """distributed_knn over reference rows carrying explicit global ids (ring of (rows, ids))."""
    best_d = torch.full((Q.shape[0], k), math.inf, device=Q.device)
    best_i = torch.full((Q.shape[0], k), -1, dtype=torch.long, device=Q.device)
    W, me = comm.world, comm.rank
    sizes = [R.shape[0]]
    if comm.is_distributed:
        sizes = comm.all_gather(torch.tensor([R.shape[0]], dtype=torch.long, device=Q.device)).view(-1).tolist()
    cur, cur_ids = R.contiguous(), ids.contiguous()
    for step in range(W):
        pending = None
        if step + 1 < W:
            src = (me - step - 1) % W
            pending = (comm.ring_pass_start(cur, sizes[src]), comm.ring_pass_start(cur_ids, sizes[src]))
        if cur.shape[0] and Q.shape[0]:
            d, i = knn(Q, cur, min(k, cur.shape[0]), metric)
            gi = torch.where(i >= 0, cur_ids[i.clamp_min(0)], i)
            if d.shape[1] < k:
                pad = k - d.shape[1]
                d = torch.cat([d, torch.full((d.shape[0], pad), math.inf, device=d.device)], 1)
                gi = torch.cat([gi, torch.full((gi.shape[0], pad), -1, dtype=gi.dtype, device=gi.device)], 1)
            best_d, best_i = _merge_topk_by_id(best_d, best_i, d, gi, k)
        if pending is not None:
            cur = comm.ring_pass_finish(pending[0])
            cur_ids = comm.ring_pass_finish(pending[1])
    return best_d, best_i


def pairwise(Q: torch.Tensor, R: torch.Tensor, metric: str = "euclidean", p: float = 2.0) -> torch.Tensor:
    """Full distance matrix (for small problems / outputs that need every pair)."""
    if metric in ("euclidean", "sqeuclidean"):
        d = torch.cdist(Q.float(), R.float())
        return d * d if metric == "sqeuclidean" else d
    if metric == "cosine":
        return 1 - torch.nn.functional.normalize(Q.float(), dim=1) @ torch.nn.functional.normalize(R.float(), dim=1).T
    if metric == "manhattan":
        return torch.cdist(Q.float(), R.float(), p=1)
    if metric == "minkowski":
        return torch.cdist(Q.float(), R.float(), p=p)
    if metric == "jaccard":
        a, b = (Q > 0).float(), (R > 0).float()
        inter = a @ b.T
        union = a.sum(1, keepdim=True) + b.sum(1).unsqueeze(0) - inter
        return 1 - inter / union.clamp_min(1e-12)
    raise ValueError(metric)


def cluster_accumulate(X: torch.Tensor, assign: torch.Tensor, K: int) -> tuple[torch.Tensor, torch.Tensor]:
    """Per-cluster feature sums (f64 [K, D]) and counts (int64 [K]) of the assigned rows."""
    if X.is_cuda:
        return _native.C().cluster_accumulate(X.float().contiguous(), assign.int().contiguous(), int(K))
    a = assign.long()
    ok = (a >= 0) & (a < K)
    sums = torch.zeros((K, X.shape[1]), dtype=torch.float64)
    sums.index_add_(0, a[ok], X[ok].double())
    counts = torch.bincount(a[ok], minlength=K)[:K].long()
    return sums, counts


def split_mixed(t: Table, weights: dict[int, float] | None = None, ranges: dict[int, tuple] | None = None):
    """The mixed-type distance's columns without one-hot expansion: (numeric f32 [n, Dn] scaled by
    sqrt(w) / range — bucketed attributes as ordinals, as in ``encode_mixed`` —, categorical codes
    int32 [n, Dc] with -1 for missing, categorical weights f32 [Dc])."""
    enc_num, cats, wcat = [], [], []
    n = t.n
    num_only = Table(t.schema, t.n, t.codes[:0], [], t.numeric, t.numeric_fields, t.labels, t.class_field)
    if t.numeric_fields:
        enc_num.append(encode_mixed(num_only, weights, ranges))
    for j, f in enumerate(t.binned_fields):
        w = (weights or {}).get(f.ordinal, f.weight)
        c = t.codes[j, :n].long()
        if f.is_categorical:
            cats.append(torch.where(c < f.num_bins, c, torch.full_like(c, -1)).int())
            wcat.append(float(w))
        else:
            b = max(f.num_bins - 1, 1)
            enc_num.append((torch.where(c >= t.missing, torch.zeros_like(c), c).float() / b * math.sqrt(w)).unsqueeze(1))
    num = torch.cat(enc_num, 1).contiguous() if enc_num else torch.zeros((n, 0), device=t.device)
    cat = torch.stack(cats, 1).contiguous() if cats else torch.zeros((n, 0), dtype=torch.int32, device=t.device)
    return num, cat, torch.tensor(wcat, dtype=torch.float32, device=t.device)


def knn_mixed(Qn, Qc, Rn, Rc, wc, k: int, r_base: int = 0):
    """k nearest references under the mixed-type distance (``split_mixed`` columns): euclidean
    distances f32 [nq, k] (+inf / -1 for missing slots) and global indices.  GPU: one
    ``mixed_knn_kernel`` launch; CPU: the same arithmetic on the one-hot embedding's terms."""
    k = int(k)
    if Qn.is_cuda:
        return tuple(_native.C().mixed_knn(Qn.float().contiguous(), Qc.int().contiguous(), Rn.float().contiguous(),
                                           Rc.int().contiguous(), wc.float().contiguous(), k, int(r_base)))
    nq, nr = Qn.shape[0], Rn.shape[0]
    out_d = torch.full((nq, k), math.inf)
    out_i = torch.full((nq, k), -1, dtype=torch.long)
    for s in range(0, nq, 1024):
        q, qc = Qn[s:s + 1024].float(), Qc[s:s + 1024].long()
        d2 = torch.cdist(q, Rn.float()) ** 2 if Qn.shape[1] else torch.zeros((q.shape[0], nr))
        for f in range(Qc.shape[1]):
            a, b = qc[:, f].view(-1, 1), Rc[:, f].long().view(1, -1)
            w = float(wc[f])
            d2 = d2 + torch.where((a < 0) & (b < 0), 0.0, torch.where((a < 0) | (b < 0), 0.5 * w,
                                                                      torch.where(a != b, w, 0.0)))
        kk = min(k, nr)
        v, i = torch.topk(d2, kk, dim=1, largest=False, sorted=True)
        out_d[s:s + 1024, :kk] = v.clamp_min(0).sqrt()
        out_i[s:s + 1024, :kk] = i + r_base
    return out_d, out_i


def encode_mixed(t: Table, weights: dict[int, float] | None = None, ranges: dict[int, tuple] | None = None) -> torch.Tensor:
    """Dense [n, D] float32 embedding whose squared euclidean distance equals the mixed-type record
    distance: numeric attributes contribute w * ((x - y) / range)^2, categorical attributes
    w * [x != y] (one-hot scaled by sqrt(w / 2)).  Bucketed attributes are treated as ordinal."""
    cols = []
    n = t.n
    for j, f in enumerate(t.numeric_fields):
        w = (weights or {}).get(f.ordinal, f.weight)
        x = t.numeric[j, :n]
        if ranges and f.ordinal in ranges:
            lo, hi = ranges[f.ordinal]
        elif f.min is not None and f.max is not None:
            lo, hi = f.min, f.max
        else:
            lo, hi = float(torch.nan_to_num(x).min()), float(torch.nan_to_num(x).max())
        rng = max(hi - lo, 1e-12)
        cols.append(((torch.nan_to_num(x) - lo) / rng * math.sqrt(w)).unsqueeze(1))
    for j, f in enumerate(t.binned_fields):
        w = (weights or {}).get(f.ordinal, f.weight)
        c = t.codes[j, :n].long()
        if f.is_categorical:
            b = f.num_bins
            oh = torch.zeros((n, b), dtype=torch.float32, device=t.device)
            ok = c < b
            oh[torch.nonzero(ok).squeeze(1), c[ok]] = math.sqrt(w / 2.0)
            cols.append(oh)
        else:
            b = max(f.num_bins - 1, 1)
            cols.append((torch.where(c >= t.missing, torch.zeros_like(c), c).float() / b * math.sqrt(w)).unsqueeze(1))
    if not cols:
        return torch.zeros((n, 0), device=t.device)
    return torch.cat(cols, 1).contiguous()
