"""CPU tests of two round-4 host helpers: ``ops.encode_ops.unique_rows`` (packed-key row unique,
= ``torch.unique(dim=0)``) and the deferred host spans of ``data.lines.LineSpans`` (a selection /
raw-line column of spans with a device twin builds its host form only when the host formatter
needs it; a CPU twin stands in for the GPU one here)."""
from __future__ import annotations

import torch

from avenir_amd.data.lines import LineSpans, _Col, host_column
from avenir_amd.data.records import format_lines
from avenir_amd.ops.encode_ops import unique_rows


def test_unique_rows_matches_torch_unique():
    g = torch.Generator().manual_seed(0)
    cases = [torch.randint(-3, 7, (2000, 3), generator=g), torch.randint(0, 1000, (500, 1), generator=g),
             torch.randint(-1, 2, (100, 6), generator=g).int(), torch.zeros((5, 2), dtype=torch.long)]
    for X in cases:
        u, inv = unique_rows(X, True)
        eu, einv = torch.unique(X, dim=0, return_inverse=True)
        assert torch.equal(u, eu) and torch.equal(inv, einv) and u.dtype == X.dtype
        assert torch.equal(unique_rows(X), eu)


def test_unique_rows_falls_back_for_wide_keys_and_floats():
    X = torch.tensor([[0, 1 << 40], [1 << 40, 0], [0, 1 << 40]], dtype=torch.long)   # span product >= 2^62
    assert torch.equal(unique_rows(X), torch.unique(X, dim=0))
    F = torch.tensor([[0.5, 1.0], [0.5, 1.0], [0.25, 2.0]])
    assert torch.equal(unique_rows(F), torch.unique(F, dim=0))
    E = torch.zeros((0, 3), dtype=torch.long)
    assert unique_rows(E).shape == (0, 3)


def _spans_with_twin(lines):
    sp = LineSpans.from_strings(lines)
    sp._strings = None                           # behave like file / shard spans (no Python strings)
    buf, off = sp.pack()
    sp.dev = (buf, off[:-1].clone(), off[1:] - off[:-1])
    return sp


def test_deferred_selection_and_columns_equal_eager(tmp_path):
    lines = [f"id{i},{i % 5},v{i * 3}" for i in range(300)]
    sp = _spans_with_twin(lines)
    keep = torch.arange(300) % 3 != 1
    sel = sp.select(keep)
    assert sel._pending is not None and len(sel) == int(keep.sum())
    col = sel.column("rf", 0, ",")
    assert isinstance(col, _Col) and col.src is not None and col.dev is not None and len(col) == 1
    host = host_column(col)
    assert host[0] == "rf" and len(host) == 6
    eager = LineSpans.from_strings([l for l, k in zip(lines, keep.tolist()) if k])
    want = format_lines([eager.column("rf", 0, ","), eager.column("r", delims=",")], len(eager), ";")
    got = format_lines([sel.column("rf", 0, ","), sel.column("r", delims=",")], len(sel), ";")
    assert got == want
    # nested selections resolve through their parents; indexing builds the host spans
    sub = sel.select(torch.tensor([2, 0]))
    assert sub[0] == [l for l, k in zip(lines, keep.tolist()) if k][2]
    p = tmp_path / "o.txt"
    format_lines([sub.column("r")], len(sub), ",", path=str(p))
    kept = [l for l, k in zip(lines, keep.tolist()) if k]
    assert p.read_text() == kept[2] + "\n" + kept[0] + "\n"
