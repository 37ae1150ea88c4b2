"""The device output formatter (format.hip) against the host formatter (csrc/host/format.cpp):
identical bytes for every column kind, including doubles at rounding ties (exact binary values,
round half to even), negative zero, NaN / inf, and the fallback (-1) for values outside the exact
fixed-point fast path."""
from __future__ import annotations

import os

import pytest
import torch

from avenir_amd import _native
from avenir_amd.data import records as R
from avenir_amd.data.lines import LineSpans


def _host(cols, n, delim, tmp):
    p = os.path.join(tmp, "host.txt")
    _native.C().format_columns_file(cols, n, delim, 4, p, False)
    return open(p, "rb").read()


def _dev(cols, n, delim, tmp, like):
    p = os.path.join(tmp, "dev.txt")
    w = _native.C().format_device(cols, n, delim, p, False, 4, like)
    return w, (open(p, "rb").read() if w >= 0 else None)


@pytest.mark.gpu
@pytest.mark.parametrize("delim", [",", "::"])
def test_device_formatter_equals_host(cuda, tmp_path, delim):
    g = torch.Generator().manual_seed(0)
    n = 5000
    tab = ["", "a", "bb", "ccc", "état"]
    idx = torch.randint(-1, 6, (n,), generator=g).int()
    cnt = torch.randint(0, 5, (n,), generator=g)
    off = torch.cat([torch.zeros(1, dtype=torch.long), torch.cumsum(cnt, 0)])
    lidx = torch.randint(0, 5, (int(off[-1]),), generator=g).int()
    ints = torch.randint(-(1 << 62), 1 << 62, (n,), generator=g)
    ints[:4] = torch.tensor([0, -1, 9223372036854775807, -9223372036854775807 - 1])
    x = (torch.randn(n, generator=g) * 10 ** torch.randint(-6, 8, (n,), generator=g).double()).double()
    ties = torch.tensor([0.125, 0.375, 2.675, 1.005, -0.0, 0.5, 1.5, 2.5, -2.5, 1e-30, 123456.789,
                         float("nan"), float("inf"), float("-inf")], dtype=torch.float64)
    x[: ties.numel()] = ties
    lines = [f"f{i},{i * 7 % 13},x y,{'z' * (i % 4)}" for i in range(n)]
    spans = LineSpans.from_strings(lines)
    buf, poff = spans.pack()
    dbuf = buf.to(cuda)
    st = poff[:-1].to(cuda)
    ln = (poff[1:] - poff[:-1]).to(cuda)
    _, a, l = spans.spans()
    for prec in (0, 1, 3, 9):
        host_cols = [("s", tab, idx), ("l", tab, lidx, off), ("i", ints), ("f", x, prec), ("c", "lit"), ("g", "]"),
                     ("r", spans, a, l, ","), ("rf", spans, a, l, 1, ","), ("rf", spans, a, l, -1, ","),
                     ("rt", spans, a, l, 2, ",")]
        dev_cols = [("s", tab, idx.to(cuda)), ("l", tab, lidx.to(cuda), off.to(cuda)), ("i", ints.to(cuda)),
                    ("f", x.to(cuda), prec), ("c", "lit"), ("g", "]"), ("dr", dbuf, st, ln, ","),
                    ("drf", dbuf, st, ln, 1, ","), ("drf", dbuf, st, ln, -1, ","), ("drt", dbuf, st, ln, 2, ",")]
        h = _host(host_cols, n, delim, tmp_path)
        w, d = _dev(dev_cols, n, delim, tmp_path, x.to(cuda))
        assert w == len(h) and d == h, prec


@pytest.mark.gpu
def test_device_formatter_falls_back_outside_fast_path(cuda, tmp_path):
    x = torch.tensor([1.0, 1e300], dtype=torch.float64, device=cuda)
    w, _ = _dev([("f", x, 3)], 2, ",", tmp_path, x)
    assert w == -1
    w, _ = _dev([("f", x[:1], 12)], 1, ",", tmp_path, x)
    assert w == -1


@pytest.mark.gpu
def test_format_lines_uses_device_twin(cuda, tmp_path, monkeypatch):
    """format_lines with device tensors and a device line twin takes the GPU path and writes the
    same file as the host path."""
    monkeypatch.setattr(R, "DEVICE_FORMAT_MIN_ROWS", 0)
    lines = [f"id{i},{i % 3}" for i in range(1000)]
    spans = LineSpans.from_strings(lines)
    buf, poff = spans.pack()
    spans.dev = (buf.to(cuda), poff[:-1].to(cuda), (poff[1:] - poff[:-1]).to(cuda))
    sel = spans.select(torch.arange(999, -1, -3))
    vals = torch.linspace(-2, 2, len(sel), dtype=torch.float64, device=cuda)
    cols = [sel.column("rf", 0, ","), ("f", vals, 4), ("s", ["p", "q"], (vals > 0).int())]
    assert R._device_columns(cols, len(sel)) is not None
    R.format_lines(cols, len(sel), ",", path=str(tmp_path / "d.txt"))
    monkeypatch.setenv("AVMI_DEVICE_FORMAT", "0")
    R.format_lines(cols, len(sel), ",", path=str(tmp_path / "h.txt"))
    assert (tmp_path / "d.txt").read_bytes() == (tmp_path / "h.txt").read_bytes()


@pytest.mark.gpu
def test_device_repr_equals_python(cuda, tmp_path):
    """prec -2 (Python repr, the shortest round-trip digits) on the device: the same bytes as
    ``repr`` for random magnitudes 1e-10 .. 1e16, powers of two and their neighbours, decimal
    fractions, signed zero and the non-finite values; values outside the exact 128-bit path
    (here 1e300) send the whole column to the host formatter (-1)."""
    import math
    g = torch.Generator().manual_seed(3)
    n = 200000
    # |x| in [1e-10, 1e16): at most 31 fraction digits, the device path's whole range
    sign = torch.where(torch.rand(n, generator=g) < 0.5, -1.0, 1.0).double()
    x = sign * (0.1 + 9.9 * torch.rand(n, generator=g, dtype=torch.float64)) * 10.0 ** torch.randint(-9, 15, (n,), generator=g).double()
    extra = [0.1, 0.2, 0.3, 1 / 3, 2 / 3, 1e-4, 1e-5, 9.999999999999999e-05, 1e15, 123456789.0, 0.5, 2.675, 1.005,
             -0.0, 0.0, 4503599627370496.0, 12.0, 100.0, float("nan"), float("inf"), float("-inf")]
    extra += [s * math.ldexp(1.0, k) for k in range(-40, 52) for s in (1, -1)]
    extra += [math.nextafter(math.ldexp(1.0, k), d) for k in range(-40, 52) for d in (0.0, 1e308)]
    extra += [i / 1000 for i in range(1, 5000)] + [-i / 7 for i in range(1, 5000)]
    x = torch.cat([x, torch.tensor(extra, dtype=torch.float64)])
    m = x.numel()
    w, d = _dev([("f", x.to(cuda), -2)], m, ",", tmp_path, x.to(cuda))
    assert w >= 0
    want = "".join(repr(v) + "\n" for v in x.tolist()).encode()
    assert d == want
    big = torch.tensor([1.5, 1e300], dtype=torch.float64, device=cuda)
    assert _dev([("f", big, -2)], 2, ",", tmp_path, big)[0] == -1
