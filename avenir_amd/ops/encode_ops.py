"""Column statistics (K26) and leave-one-out target encoding (K23) ops (encode.hip).

GPU tensors go to the HIP kernels (fail loudly if the extension is missing); CPU tensors run the
PyTorch fp64 oracle of the same op, which the GPU tests compare against.

* ``column_moments`` backs ``DataExplorer.getStats`` (P/mlextra/daexp.py getStats: mean, std,
  skew, kurtosis, min, max) with two streaming passes instead of a chain of torch reductions.
* ``loo_stats`` / ``loo_apply`` back ``models.explore.leave_one_out_encoding``
  (S/explore/CategoricalLeaveOneOutEncoding.scala:80-118); the cross-rank all-reduce of the
  per-(column, value) sums and counts sits between the two.
"""
from __future__ import annotations

import torch

from .. import _native

MOMENT_FIELDS = ("count", "sum", "min", "max", "m2", "m3", "m4", "mean")


def column_moments(X: torch.Tensor, n: int | None = None) -> torch.Tensor:
    """double [F, 8] = (count, sum, min, max, m2, m3, m4, mean) of each row of a column-major
    [F, ld] (or 1-D) matrix over its first ``n`` entries; NaNs are skipped, m_k are central power
    sums divided by the count.  A column without values (n == 0 or all NaN) has count 0, sum 0
    and NaN for every other statistic, on both devices."""
    X2 = X.view(1, -1) if X.dim() == 1 else X
    n = X2.shape[1] if n is None else int(n)
    if n == 0:
        out = torch.full((X2.shape[0], 8), float("nan"), dtype=torch.float64, device=X2.device)
        out[:, :2] = 0.0
        return out
    if X2.is_cuda:
        if X2.dtype not in (torch.float32, torch.float64):
            X2 = X2.double()
        if X2.dtype == torch.float32 and (X2.shape[1] % 4 or X2.data_ptr() % 16 or not X2.is_contiguous()):
            X2 = X2.double()
        return _empty_as_nan(_native.C().col_moments(X2.contiguous(), n))
    x = X2[:, :n].double()
    ok = ~torch.isnan(x)
    cnt = ok.sum(1).double()
    xs = torch.where(ok, x, torch.zeros_like(x))
    sm = xs.sum(1)
    lo = torch.where(ok, x, torch.full_like(x, float("inf"))).min(1).values
    hi = torch.where(ok, x, torch.full_like(x, float("-inf"))).max(1).values
    c1 = cnt.clamp_min(1.0)
    mean = sm / c1
    d = torch.where(ok, x - mean[:, None], torch.zeros_like(x))
    d2 = d * d
    return _empty_as_nan(torch.stack([cnt, sm, lo, hi, d2.sum(1) / c1, (d2 * d).sum(1) / c1, (d2 * d2).sum(1) / c1,
                                      mean], 1))


def _empty_as_nan(m: torch.Tensor) -> torch.Tensor:
    empty = m[:, 0] == 0
    if bool(empty.any()):
        m = m.clone()
        m[empty, 2:] = float("nan")
        m[empty, 1] = 0.0
    return m


def moments_dict(row: torch.Tensor) -> dict[str, float]:
    """(count, sum, min, max, m2, m3, m4, mean) -> the getStats scalars (population std, skew and
    excess kurtosis, as daexp.py computes them with scipy's defaults)."""
    v = [float(a) for a in row.cpu()]
    cnt, sm, lo, hi, m2, m3, m4, mean = v
    sd = m2 ** 0.5
    return {"count": cnt, "sum": sm, "min": lo, "max": hi, "mean": mean, "std": sd,
            "skew": m3 / sd ** 3 if sd > 0 else float("nan"),
            "kurtosis": m4 / sd ** 4 - 3 if sd > 0 else float("nan")}


def _slots(codes: torch.Tensor, slots: int | None = None) -> int:
    if codes.dtype == torch.int32:
        if slots is None:
            raise ValueError("int32 codes need slots = max code + 2 (data.table.code_slots)")
        return int(slots)
    if codes.dtype == torch.uint16:
        return int(slots) if slots is not None else 65536
    return 256


def _clamped(codes: torch.Tensor, n: int, m: int) -> torch.Tensor:
    """Codes as int64 with every value >= m - 1 (missing, out of range) in the last slot."""
    return codes[:, :n].long().clamp(max=m - 1)


def loo_stats(codes: torch.Tensor, n: int, y: torch.Tensor, slots: int | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    """Per (column, code) target sum (double [F, m]) and count (int32 [F, m]) over ``n`` rows of
    ``codes`` [F, ld] (uint8: m = 256, uint16: m = ``slots`` or 65536, int32: m = ``slots``; codes
    >= m - 1 are counted in slot m - 1)."""
    y = y[:n].double().contiguous()
    m = _slots(codes, slots)
    if codes.is_cuda:
        return tuple(_native.C().loo_stats(codes.contiguous(), int(n), y, m if codes.dtype != torch.uint8 else -1))
    F = codes.shape[0]
    c = _clamped(codes, n, m) + torch.arange(F).view(-1, 1) * m
    s = torch.zeros(F * m, dtype=torch.float64).index_add_(0, c.reshape(-1), y.repeat(F))
    k = torch.zeros(F * m, dtype=torch.int64).index_add_(0, c.reshape(-1), torch.ones(F * n, dtype=torch.int64))
    return s.view(F, m), k.view(F, m).int()


def loo_apply(codes: torch.Tensor, n: int, y: torch.Tensor, s: torch.Tensor, k: torch.Tensor, gmean: torch.Tensor,
              reg: float = 0.0, noise: torch.Tensor | None = None, amp: float = 0.0) -> torch.Tensor:
    """float32 [n, F]: (s[c] - y + reg * gmean) / max(k[c] - 1 + reg, 1e-12), times
    (1 + amp * (2u - 1)) when uniforms ``noise`` [F, n] are given (one stream per column)."""
    y = y[:n].double().contiguous()
    gm = gmean.double().reshape(-1)[:1].contiguous()
    if codes.is_cuda:
        nz = noise[:, :n].double().contiguous().to(codes.device) if noise is not None else None
        return _native.C().loo_apply(codes.contiguous(), int(n), y, s.double().contiguous(), k.int().contiguous(),
                                     gm.to(codes.device), float(reg), nz, float(amp),
                                     int(s.shape[1]) if codes.dtype != torch.uint8 else -1)
    F = codes.shape[0]
    cols = []
    cl = _clamped(codes, n, int(s.shape[1]))
    for j in range(F):
        c = cl[j]
        v = (s[j, c] - y + reg * gm) / (k[j, c].double() - 1 + reg).clamp_min(1e-12)
        if noise is not None:
            v = v * (1 + amp * (2 * noise[j, :n].double() - 1))
        cols.append(v.float())
    return torch.stack(cols, 1) if cols else torch.zeros((n, 0))


def unique_rows(X: torch.Tensor, return_inverse: bool = False):
    """``torch.unique(X, dim=0)`` (rows in lexicographic order, optionally the inverse) for integer
    rows.  When the per-column value ranges multiply to less than 2^62 the rows are packed into one
    int64 key first, so the work is a 1-D sort instead of the row-wise unique (140 ms for
    16.7 M x 2 rows on an MI355X against a few ms); otherwise the row-wise unique."""
    if X.dim() != 2 or X.shape[0] == 0 or X.shape[1] == 0 or X.is_floating_point():
        return torch.unique(X, dim=0, return_inverse=return_inverse)
    Xl = X.long()
    lo = Xl.min(0).values
    span = (Xl.max(0).values - lo + 1).tolist()
    total = 1
    for s in span:
        total *= int(s)
    if total >= 1 << 62:
        return torch.unique(X, dim=0, return_inverse=return_inverse)
    key = torch.zeros(X.shape[0], dtype=torch.long, device=X.device)
    for j, s in enumerate(span):                # first column most significant: lexicographic order
        key = key * int(s) + (Xl[:, j] - lo[j])
    if return_inverse:
        uk, inv = torch.unique(key, return_inverse=True)
    else:
        uk, inv = torch.unique(key), None
    cols = []
    for j in range(len(span) - 1, -1, -1):
        cols.append(uk % span[j] + lo[j])
        uk = uk // span[j]
    U = torch.stack(cols[::-1], 1).to(X.dtype)
    return (U, inv) if return_inverse else U
