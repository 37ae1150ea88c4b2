"""Record tables for the reference's non-schema text layouts.

The reference's sequence, transaction, tagged-token, pair-distance and event jobs split every line
with ``String.split`` and look the tokens up in HashMaps inside their mappers (state sequences
J/markov/MarkovStateTransitionModel.java:116-133, transactions
J/association/FrequentItemsApriori.java:133-196, ``obs:state`` tokens
J/markov/HiddenMarkovModelBuilder.java:136-260, pair-distance rows
J/explore/TopMatchesByClass.java:133-211 and J/knn/NearestNeighbor.java:130-183, time-stamped
events S/markov/StateTransitionRate.scala:91-167).

Here :func:`read_records` turns a rank's byte range of the input (a file, a Hadoop-style directory
of part files, or a comma list of those) into a :class:`Records` CSR table in ONE native pass:

* every rank reads only its own byte range (a line belongs to the rank whose range holds its first
  byte, as Hadoop's input splits); blank lines are dropped, a trailing CR is removed;
* every field is a token: a dictionary code (first-occurrence order), a parsed double, or nothing,
  by a per-field mode string (``'d'`` / ``'n'`` / ``'x'``, ``tail_mode`` beyond it); a
  sub-delimiter splits each dictionary token once more (``obs:state`` -> code, sub code);
* on a GPU the bytes are uploaded once and tokenized by the K1 device kernels
  (``csrc/kernels/records.hip``); on the host by the multi-threaded ``TextShard``
  (``csrc/host/records.cpp``).  Both give identical tables;
* with several ranks the dictionaries are merged once (all-gather of the vocabularies, rank order:
  the merged order is the global first-occurrence order, so codes do not depend on the world
  size) and the local codes remapped on the device.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import Sequence

import torch

from .. import _native
from .lines import host_column

#: bytes of a shard below which a GPU job tokenizes on the host and copies the table over
DEVICE_MIN_BYTES = int(os.environ.get("AVMI_GPU_RECORDS_MIN_BYTES", str(4 << 20)))


def input_paths(path: str | Path | Sequence) -> list[str]:
    """The files behind an input: a file, a directory of part files (sorted, hidden and ``_``
    files skipped) or a comma-separated list of those (``FileInputFormat.addInputPaths``)."""
    items = [path] if isinstance(path, (str, Path)) else list(path)
    out: list[str] = []
    for it in items:
        parts = [str(it)] if Path(str(it)).exists() else str(it).split(",")
        for one in parts:
            p = Path(one)
            if p.is_dir():
                out += [str(f) for f in sorted(p.iterdir()) if f.is_file() and not f.name.startswith((".", "_"))]
            else:
                out.append(str(p))
    return out


def _threads() -> int:
    return max(1, min(16, os.cpu_count() or 8))


@dataclass
class Records:
    """CSR token table of one rank's lines.

    ``off`` int64 [L+1] token offsets per line; ``codes`` int32 [T] dictionary codes (-1 for
    non-dictionary fields); ``sub`` int32 [T] sub-delimiter codes (-1 when absent) or None;
    ``nums`` float64 [T] (NaN for non-numeric fields) or None; ``vocab`` the dictionary strings;
    ``line_base`` the global index of this rank's first line."""
    off: torch.Tensor
    codes: torch.Tensor
    sub: torch.Tensor | None
    nums: torch.Tensor | None
    vocab: list[str]
    line_base: int = 0
    stats: dict = field(default_factory=dict)
    _shard: object = None
    #: the dictionary's bytes on the device (device tokenizer, single shard): vbytes uint8, voff /
    #: vlen int64 per entry — string-order sorts of keys then run on the device
    vbytes: tuple | None = None
    #: (paths, rank, world, skip_header) of the shard, to re-index its raw lines on demand
    _src: tuple | None = None
    _spans: object = None
    _file_lines: tuple | None = None    # (path, start, end byte offsets) of a device-tokenized shard
    _dev_lines: tuple | None = None     # (uploaded bytes, line starts, lengths) on the device

    @property
    def n_lines(self) -> int:
        return self.off.numel() - 1

    @property
    def n_tokens(self) -> int:
        return self.codes.numel()

    @property
    def device(self) -> torch.device:
        return self.codes.device

    def lens(self) -> torch.Tensor:
        return self.off[1:] - self.off[:-1]

    def width(self) -> int | None:
        """The common number of fields of every line, or None when lines differ."""
        if self.n_lines == 0:
            return 0
        ln = self.lens()
        w = int(ln[0])
        return w if bool((ln == w).all()) else None

    def line_of_token(self) -> torch.Tensor:
        """int64 [T]: the line index of every token."""
        return torch.repeat_interleave(torch.arange(self.n_lines, device=self.device), self.lens())

    def index(self, values: Sequence[str]) -> torch.Tensor:
        """int32 [V]: dictionary code -> position in ``values`` (-1 when absent)."""
        pos = {v: i for i, v in enumerate(values)}
        return torch.tensor([pos.get(w, -1) for w in self.vocab] or [0], dtype=torch.int32, device=self.device)[
            : len(self.vocab)]

    def map_codes(self, codes: torch.Tensor, values: Sequence[str]) -> torch.Tensor:
        """``codes`` (dictionary codes, -1 = none) translated to positions in ``values`` (-1)."""
        lut = self.index(values)
        if lut.numel() == 0:
            return torch.full_like(codes, -1)
        return torch.where(codes >= 0, lut[codes.clamp_min(0).long()], torch.full_like(codes, -1))

    def field(self, j: int, numeric: bool = False) -> torch.Tensor:
        """Codes (or values) of field ``j`` of every line; -1 (NaN) for lines with fewer fields.
        Negative ``j`` counts from the end of each line."""
        src = self.nums if numeric else self.codes
        if src is None:
            raise ValueError("no numeric tokens were parsed (read_records(numeric=...))")
        lens = self.lens()
        idx = (self.off[1:] + j) if j < 0 else (self.off[:-1] + j)
        ok = (idx >= self.off[:-1]) & (idx < self.off[1:]) & (lens > 0)
        fill = float("nan") if numeric else -1
        if src.numel() == 0:
            return torch.full((self.n_lines,), fill, dtype=src.dtype, device=self.device)
        vals = src[idx.clamp(0, max(0, src.numel() - 1))]
        return torch.where(ok, vals, torch.full_like(vals, fill))

    def dense(self, width: int, numeric: bool = False) -> torch.Tensor:
        """[L, width] view of the tokens of fixed-width lines."""
        src = self.nums if numeric else self.codes
        return src.view(self.n_lines, width)

    def padded(self, codes: torch.Tensor | None = None, start: int = 0, drop: Sequence[int] = (), fill: int = -1,
               min_len: int = 0, dtype=torch.int16) -> tuple[torch.Tensor, torch.Tensor]:
        """Per-line token rows as a padded ``[L, W]`` matrix: the tokens at field positions
        ``>= start`` except ``drop`` (e.g. a class field inside a sequence), left-aligned, ``fill``
        beyond each line's end.  ``codes`` defaults to the dictionary codes (any per-token int
        tensor, e.g. mapped states).  Returns (matrix, kept-token count per line).  Fixed-width
        tables are a strided column selection; ragged ones one scatter."""
        src = self.codes if codes is None else codes
        L = self.n_lines
        w = self.width()
        dropset = {d for d in drop if d >= start}
        if w is not None:
            cols = [j for j in range(start, w) if j not in dropset]
            cnt = torch.full((L,), len(cols), dtype=torch.int64, device=self.device)
            if not cols or L == 0:
                return torch.full((L, max(min_len, len(cols))), fill, dtype=dtype, device=self.device), cnt
            M = src.view(L, w)[:, torch.tensor(cols, device=self.device)]
            if len(cols) < min_len:
                M = torch.cat([M, torch.full((L, min_len - len(cols)), fill, dtype=M.dtype, device=self.device)], 1)
            return M.to(dtype), cnt
        tl = self.line_of_token()
        pos = torch.arange(self.n_tokens, device=self.device) - self.off[:-1][tl]
        keep = pos >= start
        for d in dropset:
            keep &= pos != d
        cs = torch.cumsum(keep.long(), 0)
        before = torch.cat([torch.zeros(1, dtype=torch.long, device=self.device), cs])[self.off[:-1]]
        cnt = torch.cat([torch.zeros(1, dtype=torch.long, device=self.device), cs])[self.off[1:]] - before
        W = max(min_len, int(cnt.max()) if L else 0)
        M = torch.full((L, W), fill, dtype=dtype, device=self.device)
        if W and bool(keep.any()):
            newpos = cs - 1 - before[tl]
            M[tl[keep], newpos[keep]] = src[keep].to(dtype)
        return M, cnt

    def strings(self, codes: torch.Tensor | Sequence[int]) -> list[str]:
        v = self.vocab
        cs = codes.tolist() if isinstance(codes, torch.Tensor) else list(codes)
        return [v[c] if c >= 0 else "" for c in cs]

    def lines(self) -> list[str]:
        """The raw text of this rank's lines as Python strings (prefer :meth:`line_spans`)."""
        return self.line_spans().tolist()

    def line_spans(self):
        """This rank's raw lines as byte spans (data/lines.LineSpans) for the native formatter:
        the host tokenizer's shard, or — for a device-tokenized table — a host line index of the
        same byte range built on first use (one multi-threaded newline scan, no tokenizing)."""
        from .lines import LineSpans
        if self._spans is None and self._file_lines is not None:
            path, starts, ends = self._file_lines
            self._spans = LineSpans.from_file(path, starts, ends)
        if self._spans is None:
            if self._shard is None and self._src is not None:
                paths, rank, world, skip = self._src
                C = _native.host()
                if C is not None:
                    self._shard = C.TextShard(paths, rank, world, _threads(), skip)
                else:
                    self._spans = LineSpans.from_strings(_py_lines(paths, rank, world, skip))
            if self._spans is None:
                if self._shard is None:
                    raise RuntimeError("raw lines are not available for this table")
                self._spans = LineSpans.from_shard(self._shard)
            if len(self._spans) != self.n_lines:
                raise RuntimeError("line index does not match the token table")
        if self._dev_lines is not None and self._spans.dev is None:
            self._spans.dev = self._dev_lines
        return self._spans

    def to(self, device) -> "Records":
        mv = lambda t: None if t is None else t.to(device)
        return Records(mv(self.off), mv(self.codes), mv(self.sub), mv(self.nums), self.vocab, self.line_base,
                       self.stats, self._shard, _src=self._src, _spans=self._spans, _file_lines=self._file_lines,
                       _dev_lines=self._dev_lines)


# ------------------------------------------------------------------------------------------------
def read_records(path, *, comm=None, delims: str = ",", sub_delim: str = "", modes: str = "", tail_mode: str = "d",
                 trim: bool = False, numeric: bool = False, device="cpu", skip_header: bool = False,
                 shard: bool = True, last_mode: str = "") -> Records:
    """This rank's :class:`Records` of ``path`` (see the module docstring).  ``comm``: the job's
    communicator (byte-range shard + dictionary merge when distributed); ``shard=False`` reads the
    whole input on every rank (side files); ``last_mode``: the mode of every line's last field
    (e.g. ``'n'`` for a trailing rank / distance of any line width)."""
    paths = input_paths(path)
    dist = comm is not None and comm.is_distributed and shard
    rank, world = (comm.rank, comm.world) if dist else (0, 1)
    dev = torch.device(device)
    C = _native.host()
    rec = None
    if C is not None:
        if dev.type == "cuda" and hasattr(C, "text_tokenize_device") and not skip_header:
            total = sum(os.path.getsize(p) for p in paths)
            if total // world >= DEVICE_MIN_BYTES:
                r = C.text_tokenize_device(paths, rank, world, delims, sub_delim, modes, tail_mode, trim, numeric,
                                           torch.empty(0, device=dev), 1 << 24, last_mode)
                if r is not None:
                    off, codes, sub, nums, vocab, stats = r
                    vb = (stats.pop("vbytes"), stats.pop("voff"), stats.pop("vlen"))
                    fl = None
                    if "line_file" in stats:     # the shard lies in one file: lines as file offsets
                        fl = (paths[int(stats.pop("line_file"))], stats.pop("line_starts"), stats.pop("line_ends"))
                    dl = (stats.pop("line_buf"), stats.pop("line_rel_starts"), stats.pop("line_rel_ends"))
                    rec = Records(off, codes, sub, nums, list(vocab), stats=dict(stats, path="device"), vbytes=vb)
                    rec._file_lines = fl
                    rec._dev_lines = (dl[0], dl[1], dl[2] - dl[1])
        if rec is None:
            sh = C.TextShard(paths, rank, world, _threads(), skip_header)
            off, codes, sub, nums, vocab = sh.tokenize(delims, sub_delim, modes, tail_mode, trim, numeric, last_mode)
            rec = Records(off, codes, sub, nums, list(vocab), stats={"path": "host", "bytes": sh.bytes_read()},
                          _shard=sh)
            if dev.type != "cpu":
                rec = rec.to(dev)
    else:
        rec = _read_records_py(paths, rank, world, delims, sub_delim, modes, tail_mode, trim, numeric, skip_header,
                               last_mode)
        rec = rec.to(dev) if dev.type != "cpu" else rec
    rec._src = (paths, rank, world, skip_header)
    if dist:
        _merge_vocab(rec, comm)
    return rec


def _merge_vocab(rec: Records, comm) -> None:
    """Global dictionary = the rank-ordered union of the shard dictionaries (= global first
    occurrence); local codes are remapped on their device; ``line_base`` from the line counts."""
    parts = comm.all_gather_object((rec.vocab, rec.n_lines))
    glob: dict[str, int] = {}
    for voc, _ in parts:
        for w in voc:
            if w not in glob:
                glob[w] = len(glob)
    rec.line_base = sum(n for _, n in parts[: comm.rank])
    rec.vbytes = None     # the merged dictionary's entries no longer match the shard's bytes
    if rec.vocab:
        lut = torch.tensor([glob[w] for w in rec.vocab], dtype=torch.int32, device=rec.device)
        remap = lambda c: torch.where(c >= 0, lut[c.clamp_min(0).long()], c)
        rec.codes = remap(rec.codes)
        if rec.sub is not None:
            rec.sub = remap(rec.sub)
    rec.vocab = list(glob)


def _py_lines(paths, rank: int, world: int, skip_header: bool) -> list[str]:
    """Pure-Python twin of the native byte-range shard: non-blank lines whose first byte lies in
    this rank's range of the concatenated files."""
    total = sum(os.path.getsize(p) for p in paths)
    lo, hi = total * rank // world, total * (rank + 1) // world
    out: list[str] = []
    base = 0
    for p in paths:
        raw = Path(p).read_bytes()
        start = 0
        while start < len(raw):
            nl = raw.find(b"\n", start)
            end = len(raw) if nl < 0 else nl
            if lo <= base + start < hi:
                ln = raw[start:end].decode()
                ln = ln[:-1] if ln.endswith("\r") else ln
                if ln.strip(" \t\r\v\f"):
                    out.append(ln)
            start = end + 1
        base += len(raw)
    if skip_header and rank == 0 and out:
        out = out[1:]
    return out


def _read_records_py(paths, rank, world, delims, sub_delim, modes, tail_mode, trim, numeric, skip_header,
                     last_mode: str = "") -> Records:
    """Pure-Python twin of the native tokenizers (used when the extension is not built)."""
    import math
    import re
    lines = _py_lines(paths, rank, world, skip_header)
    sep = "[" + re.escape(delims or ",") + "]"
    vocab: dict[str, int] = {}
    off, codes, sub, nums = [0], [], [], []
    for ln in lines:
        fields = re.split(sep, ln)
        for f, tok in enumerate(fields):
            m = last_mode if (last_mode and f == len(fields) - 1) else (modes[f] if f < len(modes) else tail_mode)
            if trim:
                tok = tok.strip(" \t\r\v\f")
            c, s, v = -1, -1, math.nan
            if m == "d":
                a, b = (tok.split(sub_delim, 1) + [None])[:2] if sub_delim else (tok, None)
                c = vocab.setdefault(a, len(vocab))
                if b is not None:
                    s = vocab.setdefault(b, len(vocab))
            elif m == "n":
                try:
                    v = float(tok.strip(" \t\r\v\f"))
                except ValueError:
                    v = math.nan
            codes.append(c)
            sub.append(s)
            nums.append(v)
        off.append(len(codes))
    return Records(torch.tensor(off, dtype=torch.int64), torch.tensor(codes, dtype=torch.int32),
                   torch.tensor(sub, dtype=torch.int32) if sub_delim else None,
                   torch.tensor(nums, dtype=torch.float64) if numeric else None, list(vocab), stats={"path": "python"})


def shard_lines(path, comm=None, shard: bool = True, skip_header: bool = False) -> list[str]:
    """This rank's non-blank lines of ``path`` (byte-range shard; all lines with ``shard=False``)."""
    paths = input_paths(path)
    dist = comm is not None and comm.is_distributed and shard
    rank, world = (comm.rank, comm.world) if dist else (0, 1)
    C = _native.host()
    if C is not None:
        sh = C.TextShard(paths, rank, world, _threads(), skip_header)
        return sh.lines(0, sh.num_lines())
    return _py_lines(paths, rank, world, skip_header)


def format_lines(cols: list[tuple], n: int, delim: str = ",", path: str | None = None, append: bool = False):
    """Output text of ``n`` rows assembled column by column (native, multi-threaded):
    ``("s", table, idx)`` string-table lookups, ``("f", values, prec)`` numbers (prec < 0: ``%g``),
    ``("i", ints)``, ``("c", literal)``, ``("g", literal)`` glued on without a delimiter,
    ``("l", table, idx, off)`` a variable-length list of table strings per row (CSR),
    ``("lp", table, idx, ints, off)`` the same with an integer after every string, and the raw
    input line kinds of ``data/lines.LineSpans.column``: ``("r", ...)`` the line, ``("rf", ...)``
    one of its fields, ``("rt", ...)`` its fields from one on.  ``prec`` -2 writes Python's
    ``repr`` of the value.  Every row ends with a newline.  With ``path`` the text goes straight
    into that file (threads pwrite their blocks; ``append`` adds to it) and the byte count is
    returned instead of the bytes."""
    C = _native.host()
    if C is not None:
        if path is not None:
            dcols = _device_columns(cols, n)
            if dcols is not None:     # rows formatted on the GPU (format.hip), written by host threads
                w = C.format_device(dcols[0], int(n), delim, str(path), bool(append), _threads(), dcols[1])
                if w >= 0:
                    return w
            return C.format_columns_file([host_column(c) for c in cols], int(n), delim, _threads(), str(path),
                                         bool(append))
        return C.format_columns([host_column(c) for c in cols], int(n), delim, _threads())
    cols = [host_column(c) for c in cols]
    if path is not None:
        data = format_lines(cols, n, delim)
        with open(path, "ab" if append else "wb") as fh:
            fh.write(data)
        return len(data)
    rows = [[] for _ in range(n)]
    glue_pre = [""] * n
    for c in cols:
        k = c[0]
        if k == "g":
            for r in range(n):
                if rows[r]:
                    rows[r][-1] += c[1]
                else:
                    glue_pre[r] += c[1]
            continue
        if k == "s":
            tab, idx = c[1], c[2].tolist()
            for r in range(n):
                rows[r].append(tab[idx[r]] if 0 <= idx[r] < len(tab) else "")
        elif k == "f":
            vals, prec = c[1].tolist(), (c[2] if len(c) > 2 else 6)
            for r in range(n):
                v = vals[r]
                rows[r].append(repr(v) if prec == -2 else
                               ("NaN" if v != v else (f"{v:.{prec}f}" if prec >= 0 else f"{v:g}")))
        elif k == "i":
            vals = c[1].tolist()
            for r in range(n):
                rows[r].append(str(int(vals[r])))
        elif k == "c":
            for r in range(n):
                rows[r].append(c[1])
        elif k == "l":
            tab, idx, off = c[1], c[2].tolist(), c[3].tolist()
            for r in range(n):
                rows[r] += [tab[i] if 0 <= i < len(tab) else "" for i in idx[off[r]:off[r + 1]]]
        elif k == "lp":
            tab, idx, iv, off = c[1], c[2].tolist(), c[3].tolist(), c[4].tolist()
            for r in range(n):
                for j in range(off[r], off[r + 1]):
                    rows[r] += [tab[idx[j]] if 0 <= idx[j] < len(tab) else "", str(int(iv[j]))]
        elif k in ("r", "rf", "rt"):
            import ctypes
            import re
            a, ln = c[2].tolist(), c[3].tolist()
            fld = c[4] if k != "r" else 0
            dl = c[5] if k != "r" else (c[4] if len(c) > 4 else "")
            sp = re.compile("[" + re.escape(dl) + "]") if dl else None
            for r in range(n):
                txt = ctypes.string_at(a[r], ln[r]).decode()
                if k == "r":
                    rows[r].append(sp.sub(delim, txt) if sp else txt)
                    continue
                parts = sp.split(txt) if sp else [txt]
                if k == "rf":
                    ok = -len(parts) <= fld < len(parts)
                    rows[r].append(parts[fld] if ok else "")
                else:
                    rows[r].append(delim.join(parts[fld:]) if fld < len(parts) else "")
        else:
            raise ValueError(f"unknown column kind {k!r}")
    out = []
    for r in range(n):
        if rows[r]:
            rows[r][0] = glue_pre[r] + rows[r][0]
            out.append(delim.join(rows[r]) + "\n")
        else:
            out.append(glue_pre[r] + "\n")
    return "".join(out).encode()


#: rows from which ``format_lines`` formats on the GPU when every column is device-resident
DEVICE_FORMAT_MIN_ROWS = int(os.environ.get("AVMI_DEVICE_FORMAT_MIN_ROWS", str(1 << 18)))


def _device_columns(cols: list, n: int):
    """(device column tuples, a device tensor) when every column can be formatted on the GPU
    (tensors already on a GPU, raw-line columns with a device twin, literals, string tables), at
    least one column is device data and ``n`` is large enough; else None."""
    if n < DEVICE_FORMAT_MIN_ROWS or os.environ.get("AVMI_DEVICE_FORMAT", "1") == "0":
        return None
    out, like = [], None
    for c in cols:
        k = c[0]
        if k in ("c", "g"):
            out.append(c)
            continue
        if k in ("r", "rf", "rt"):
            d = getattr(c, "dev", None)
            if d is None:
                return None
            out.append(d)
            like = torch.empty(0, device=d[1].device)
            continue
        if k == "f" and not (len(c) > 2 and (0 <= int(c[2]) <= 9 or int(c[2]) == -2)):
            return None
        tens = {"s": [2], "l": [2, 3], "lp": [2, 3, 4], "f": [1], "i": [1]}.get(k)
        if tens is None:
            return None
        for j in tens:
            t = c[j]
            if not (isinstance(t, torch.Tensor) and t.is_cuda):
                return None
            like = torch.empty(0, device=t.device)
        out.append(c)
    return (out, like) if like is not None else None


# ------------------------------------------------------------------------------------------------
# keyed (reduce-side) helpers: the MapReduce shuffle as one all-to-all
_KEY_BYTES = 7          # bytes per non-negative int64 sort word
_KEY_WORDS = 3         # strings up to 21 bytes sort on the device


def _pack_words(b: torch.Tensor, lens: torch.Tensor) -> list[torch.Tensor]:
    """[n, 21] uint8 (zero padded) -> 3 int64 words, most significant first (big-endian 7-byte
    groups: non-negative, so signed order = byte order = code-point order of UTF-8 text)."""
    out = []
    for w in range(_KEY_WORDS):
        v = torch.zeros(b.shape[0], dtype=torch.int64, device=b.device)
        for j in range(_KEY_BYTES):
            v = v * 256 + b[:, w * _KEY_BYTES + j].long()
        out.append(v)
    return out


def _string_order(rec: Records, idx: torch.Tensor) -> torch.Tensor | None:
    """Permutation sorting dictionary entries ``idx`` by their strings, on ``idx``'s device, or
    None when an entry is longer than 21 bytes (the caller then sorts on the host)."""
    dev = idx.device
    W = _KEY_BYTES * _KEY_WORDS
    if rec.vbytes is not None and rec.vbytes[0].device == dev:
        vb, vo, vl = rec.vbytes
        lens = vl[idx]
        if lens.numel() and int(lens.max()) > W:
            return None
        j = torch.arange(W, device=dev)
        pos = (vo[idx].view(-1, 1) + j).clamp_max(max(0, vb.numel() - 1))
        b = torch.where(j < lens.view(-1, 1), vb[pos] if vb.numel() else torch.zeros_like(pos, dtype=torch.uint8),
                        torch.zeros((), dtype=torch.uint8, device=dev))
    else:
        import numpy as np
        voc = rec.vocab
        enc = [voc[i].encode() for i in idx.tolist()]
        ln = np.fromiter(map(len, enc), dtype=np.int64, count=len(enc))
        if ln.size and int(ln.max()) > W:
            return None
        # one joined buffer scattered into the [n, W] byte matrix (no per-entry numpy call)
        flat = np.frombuffer(b"".join(enc), dtype=np.uint8)
        arr = np.zeros((len(enc), W), dtype=np.uint8)
        if flat.size:
            starts = np.cumsum(ln) - ln
            row = np.repeat(np.arange(len(enc)), ln)
            arr[row, np.arange(flat.size) - np.repeat(starts, ln)] = flat
        b = torch.from_numpy(arr).to(dev)
        lens = None
    words = _pack_words(b, lens)
    order = torch.arange(idx.numel(), device=dev)
    for w in reversed(words):       # LSD: stable sorts from the least significant word
        order = order[torch.argsort(w[order], stable=True)]
    return order


def sorted_keys(rec: Records, codes: torch.Tensor, comm=None) -> tuple[torch.Tensor, torch.Tensor]:
    """The distinct dictionary codes of ``codes`` over all ranks, ordered by their strings (the
    reducer key order of the reference), and a [V] lookup code -> position in that order (-1).
    Presence is one all-reduce of a [V] byte mask; the string order comes from packed byte keys
    sorted on the device (a host string sort only for entries longer than 21 bytes)."""
    V = len(rec.vocab)
    dev = codes.device
    present = torch.zeros(max(1, V), dtype=torch.uint8, device=dev)
    c = codes[codes >= 0].long()
    if c.numel():
        present[c] = 1
    if comm is not None and comm.is_distributed:
        comm.all_reduce(present, "max")
    idx = torch.nonzero(present[:V]).view(-1)
    order = _string_order(rec, idx) if idx.numel() else idx
    if order is None:
        import numpy as np
        o = np.argsort(np.array([rec.vocab[i] for i in idx.tolist()]), kind="stable")
        order = torch.from_numpy(o.astype(np.int64)).to(dev)
    keys = idx[order]
    pos = torch.full((max(1, V),), -1, dtype=torch.int64, device=dev)
    pos[keys] = torch.arange(keys.numel(), device=dev)
    return keys, pos[:V]


def sorted_key_tuples(rec: Records, cols: list[torch.Tensor], comm=None):
    """Composite keys of several dictionary-coded fields (``cols``: per field the codes of every
    row, all rows valid) in the reference's reducer order — tuples of strings compared field by
    field — over all ranks.  Returns (kpos int64 [n]: the global position of every row's key,
    G: the number of distinct keys, key codes int64 [G, m] (host) in that order).  The field codes'
    string ranks come from ONE device packed-key sort (``sorted_keys``); a key is the mixed-radix
    number of its ranks, and the distinct keys of all ranks are one all-gather."""
    dev = cols[0].device if cols else rec.device
    m = len(cols)
    n = cols[0].numel() if cols else 0
    if m == 0:
        return torch.zeros(n, dtype=torch.long, device=dev), 1, torch.zeros((1, 0), dtype=torch.long)
    keys, pos = sorted_keys(rec, torch.cat([c.reshape(-1) for c in cols]), comm)
    R = keys.numel() + 1
    if R ** m >= (1 << 62):
        raise ValueError("composite key space exceeds 2^62")
    comp = torch.zeros(n, dtype=torch.long, device=dev)
    for c in cols:
        comp = comp * R + pos[c.long()]
    loc = torch.unique(comp)
    if comm is not None and comm.is_distributed:
        cdev = comm.device if comm.pg_backend == "nccl" else torch.device("cpu")
        allc = torch.unique(comm.all_gather_v(loc.to(cdev))).to(dev)
    else:
        allc = loc
    kpos = torch.searchsorted(allc, comp)
    digits, rem = [], allc.clone()
    for _ in range(m):
        digits.append(rem % R)
        rem = rem // R
    table = torch.stack([keys[d] for d in reversed(digits)], 1).cpu() if allc.numel() else \
        torch.zeros((0, m), dtype=torch.long)
    return kpos, int(allc.numel()), table


def segment_rank(first: torch.Tensor) -> torch.Tensor:
    """Position of every element inside its segment (``first`` marks segment starts, element 0
    included): segment id by one inclusive scan, the segment's first index gathered from the head
    list.  Replaces a ``cummax`` of start indices, which ROCm runs as a slow single-pass scan (54 ms
    of a 33 M-element topMatchesByClass against a few ms for cumsum + gather)."""
    n = first.numel()
    if n == 0:
        return torch.zeros(0, dtype=torch.long, device=first.device)
    seg = torch.cumsum(first.long(), 0) - 1
    heads = torch.nonzero(first).view(-1)
    return torch.arange(n, device=first.device) - heads[seg]


def owner_of(pos: torch.Tensor, n_keys: int, world: int) -> torch.Tensor:
    """Rank owning sorted key position ``pos`` when the keys are cut into contiguous balanced
    blocks (data/table.shard_range): the rank-ordered concatenation of the owners' outputs is the
    global key order, so outputs do not depend on the world size."""
    base, rem = divmod(n_keys, world)
    starts = torch.tensor([r * base + min(r, rem) for r in range(world)], dtype=torch.int64, device=pos.device)
    return (torch.searchsorted(starts, pos.long(), right=True) - 1).clamp_min(0)


def shuffle(comm, owner: torch.Tensor, cols: list[torch.Tensor]) -> list[torch.Tensor]:
    """Send every row (``cols`` share dim 0) to rank ``owner[row]`` with one all-to-all; the
    received rows come in source-rank order, each source's rows in their original order, so a
    stable sort downstream sees the global input order.  float64 columns travel bit-exact."""
    if comm is None or not comm.is_distributed:
        return cols
    kinds = [c.dtype for c in cols]
    packed = torch.stack([c.view(torch.int64) if c.dtype == torch.float64 else c.long() for c in cols], 1) \
        if cols else torch.zeros((owner.numel(), 0), dtype=torch.int64, device=owner.device)
    order = torch.argsort(owner, stable=True)
    counts = torch.bincount(owner, minlength=comm.world).tolist()
    chunks = list(torch.split(packed[order], counts))
    recv = torch.cat(comm.all_to_all_v(chunks), 0)
    out = []
    for j, dt in enumerate(kinds):
        col = recv[:, j].contiguous()
        out.append(col.view(torch.float64) if dt == torch.float64 else col.to(dt))
    return out


def shuffle_spans(comm, owner: torch.Tensor, spans):
    """The line bytes behind ``spans`` sent along with :func:`shuffle` (same ``owner``): every
    destination receives its lines in source-rank order, each source's lines in their original
    order — aligned with the rows :func:`shuffle` delivers.  Returns a LineSpans over the
    received bytes (one packed byte all-to-all plus one of the lengths)."""
    from .lines import LineSpans
    owner = owner.cpu()
    order = torch.argsort(owner, stable=True)
    counts = torch.bincount(owner, minlength=comm.world).tolist()
    buf, off = spans.select(order).pack()
    lens = off[1:] - off[:-1]
    bounds = [0]
    for c in counts:
        bounds.append(bounds[-1] + c)
    byte_chunks = [buf[int(off[bounds[r]]):int(off[bounds[r + 1]])] for r in range(comm.world)]
    len_chunks = [lens[bounds[r]:bounds[r + 1]] for r in range(comm.world)]
    rb = torch.cat(comm.all_to_all_v(byte_chunks), 0) if comm.world else buf
    rl = torch.cat(comm.all_to_all_v(len_chunks), 0)
    return LineSpans.from_packed(rb, torch.cat([torch.zeros(1, dtype=torch.long), torch.cumsum(rl, 0)]))


def numeric_lut(vocab: list[str], device) -> torch.Tensor:
    """float64 [V]: the number each dictionary string parses to (NaN otherwise) — numeric fields
    tokenized as dictionary entries (ranks, small integer fields)."""
    import numpy as np
    out = np.full(max(1, len(vocab)), np.nan)
    for i, v in enumerate(vocab):
        try:
            out[i] = float(v)
        except ValueError:
            pass
    return torch.from_numpy(out[: len(vocab)]).to(device)
