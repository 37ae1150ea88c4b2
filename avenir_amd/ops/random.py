"""Counter-based Philox4x32-10 (the same generator as ``avenir_common.h``) for host-side reference
paths, so CPU and GPU code draw bit-identical random streams for a given (seed, offset, index)."""
from __future__ import annotations

import numpy as np
import torch

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
_MASK = np.uint64(0xFFFFFFFF)


def philox4x32(seed: int, offset: int, idx: np.ndarray) -> tuple[np.ndarray, ...]:
    """Vectorised philox4x32-10 of counters (idx_lo, idx_hi, offset_lo, offset_hi) with key = seed."""
    idx = np.asarray(idx, dtype=np.uint64)
    c0 = (idx & _MASK).astype(np.uint32)
    c1 = (idx >> np.uint64(32)).astype(np.uint32)
    c2 = np.full_like(c0, np.uint32(offset & 0xFFFFFFFF))
    c3 = np.full_like(c0, np.uint32((offset >> 32) & 0xFFFFFFFF))
    k0 = np.uint32(seed & 0xFFFFFFFF)
    k1 = np.uint32((seed >> 32) & 0xFFFFFFFF)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = _M0 * c0.astype(np.uint64)
            p1 = _M1 * c2.astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & _MASK).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & _MASK).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = np.uint32((int(k0) + int(_W0)) & 0xFFFFFFFF)
            k1 = np.uint32((int(k1) + int(_W1)) & 0xFFFFFFFF)
    return c0, c1, c2, c3


def u32_to_unit(x: np.ndarray) -> np.ndarray:
    """Uniform in (0, 1] exactly as the device helper (24 high bits, +1, / 2^24), float32."""
    return ((x >> np.uint32(8)).astype(np.float32) + np.float32(1.0)) * np.float32(1.0 / 16777216.0)


def uniform(seed: int, offset: int, n: int, device="cpu") -> torch.Tensor:
    x, _, _, _ = philox4x32(seed, offset, np.arange(n, dtype=np.uint64))
    return torch.from_numpy(u32_to_unit(x)).to(device)
