"""K25 re-sampling ops (csrc/kernels/resample.hip): GPU tensors go to the HIP kernels, CPU tensors
to a bit-identical host twin on the same counter-based Philox4x32-10 streams (ops/random.py).

Every draw is keyed by (seed, stream, GLOBAL record index), so a rank computes exactly what one
process would compute for the records it owns (world-size invariant re-sampling)."""
from __future__ import annotations

import numpy as np
import torch

from .. import _native
from .random import philox4x32, u32_to_unit

STREAM_UNDERSAMPLE = 0x0025_0001
STREAM_BAGGING = 0x0025_0002
_SMOTE_STREAM = 0x5EED0025


def uniform(seed: int, stream: int, base: int, n: int, device="cpu") -> torch.Tensor:
    """float32 [n]: u(seed, stream, base + i) in (0, 1]."""
    dev = torch.device(device)
    seed &= 0x7FFFFFFFFFFFFFFF
    if dev.type == "cuda":
        return _native.C().resample_uniform(int(seed), int(stream), int(base), int(n), torch.empty(0, device=dev))
    x, _, _, _ = philox4x32(seed, stream, np.arange(base, base + n, dtype=np.uint64))
    return torch.from_numpy(u32_to_unit(x))


def smote_rows(X: torch.Tensor, Xn: torch.Tensor, nn: torch.Tensor, Cs: torch.Tensor | None, Cn: torch.Tensor | None,
               mult: int, gbase: int, seed: int, exponential: bool = False, exp_mean: float = 1.0):
    """``mult`` synthetic rows per source row r (output row r * mult + j, draw counter
    (gbase + r) * mult + j): numeric = X[r] + gap * (Xn[r, pick] - X[r]), categorical from the
    source or the picked neighbour.  Returns (newX [m*mult, D], newC [m*mult, Dc], pick [m*mult])."""
    seed &= 0x7FFFFFFFFFFFFFFF
    m, D = X.shape
    k = Xn.shape[1]
    if X.is_cuda:
        return tuple(_native.C().smote(X.float().contiguous(), Xn.float().contiguous(), nn.int().contiguous(),
                                       None if Cs is None else Cs.int().contiguous(),
                                       None if Cn is None else Cn.int().contiguous(), int(mult), int(gbase),
                                       int(seed), bool(exponential), float(exp_mean)))
    o = np.arange(m * mult, dtype=np.int64)
    r = o // max(mult, 1)
    j = o - r * mult
    ctr = ((gbase + r) * mult + j).astype(np.uint64)
    dx, dy, dz, _ = philox4x32(seed, _SMOTE_STREAM, ctr)
    cnt = nn.numpy().astype(np.int64)[r]
    ux = u32_to_unit(dx)
    if exponential:
        e = -float(np.float32(exp_mean)) * np.log(ux.astype(np.float64))
        pick = np.rint(e).astype(np.int64) - 1
        pick = np.clip(pick, 0, np.maximum(cnt - 1, 0))
    else:
        pick = (ux * cnt.astype(np.float32)).astype(np.int64)
        pick = np.minimum(pick, np.maximum(cnt - 1, 0))
    pick = np.where(cnt > 0, pick, 0)
    gap = (u32_to_unit(dy) - np.float32(1.0 / 16777216.0)).astype(np.float32)
    Xs = X.float().numpy()[r]
    Xnb = np.where((cnt > 0)[:, None], Xn.float().numpy()[r, pick], Xs)
    newX = (Xs + gap[:, None] * (Xnb - Xs)).astype(np.float32)
    newC = np.zeros((m * mult, 0 if Cs is None else Cs.shape[1]), dtype=np.int32)
    if Cs is not None:
        cs = Cs.int().numpy()[r]
        cn = np.where((cnt > 0)[:, None], Cn.int().numpy()[r, pick], cs)
        newC = np.where((dz >> np.uint32(31)).astype(bool)[:, None], cs, cn).astype(np.int32)
    return (torch.from_numpy(newX), torch.from_numpy(newC),
            torch.from_numpy(np.where(cnt > 0, pick, -1).astype(np.int32)))
