"""Columnar, schema-encoded tables (layer N3 of SURVEY.md §7.1).

A ``Table`` is the device-resident form of a CSV file described by a ``FeatureSchema``:

* ``codes``   uint8 ``[Fb, ld]`` — binned features (categorical dictionary codes, or int/double
  bucketized by ``bucketWidth``), feature-major (SoA) with ``ld`` a multiple of 16 so the HIP
  kernels stream 16 rows per 128-bit load.  Unknown / missing values are coded 255.  When any
  binned field has more than 255 values (the reference keys categoricals by raw string, so
  high-cardinality fields such as supplier / product ids are legal) the table is *wide*: codes are
  uint16 with 65535 = missing, counted by the K2w kernel (``wide.hip``); beyond 65,534 values the
  codes are int32 with INT32_MAX = missing (same kernel, int32 instantiation).
* ``numeric`` float32 ``[Fn, ld]`` — continuous (un-bucketized) numeric features.
* ``labels``  uint8 ``[ld]`` — class attribute codes (255 = unknown).
* ``ids``     list of record id strings (when the schema has an id field).

Rows can be loaded as one contiguous shard per rank (``rank``/``world``) — the replacement for
Hadoop input splits: every rank reads only its own byte range of the file.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import Sequence

import numpy as np
import torch

from .. import _native
from ..utils.schema import FeatureField, FeatureSchema
from ..utils.tracing import traced

CAT, BUCKET, FLOAT, INT = 0, 1, 2, 3
MISSING = 255
MISSING16 = 65535
MISSING32 = 2**31 - 1
_MISSING_OF = {torch.uint8: MISSING, torch.uint16: MISSING16, torch.int32: MISSING32}


def missing_code(codes: torch.Tensor) -> int:
    """The 'missing / unknown' code of a code tensor (255 uint8, 65535 uint16, INT32_MAX int32)."""
    return _MISSING_OF.get(codes.dtype, MISSING)


def needs_wide(fields) -> bool:
    return any(f.num_bins > 255 for f in fields)


def code_width(fields) -> int:
    """0: uint8 codes, 1: uint16 (> 255 values), 2: int32 (> 65,534 values in some field)."""
    top = max((f.num_bins for f in fields), default=0)
    return 2 if top > 65534 else (1 if top > 255 else 0)


_CODE_DTYPE = (torch.uint8, torch.uint16, torch.int32)


def code_slots(codes: torch.Tensor, bins) -> int:
    """Per-column table size for code-indexed lookups: every valid code plus one missing slot."""
    if codes.dtype in (torch.int32, torch.uint16):
        return max([int(b) for b in bins] + [1]) + 1
    return 256


_ESCAPED_LITERALS = {r"\t": "\t", r"\|": "|", r"\.": ".", r"\\": "\\", r"\$": "$", r"\^": "^"}


def _literal(delim: str) -> str | None:
    """The literal separator a ``field.delim.regex`` value denotes, or None for a real regex."""
    import re
    if delim in _ESCAPED_LITERALS:
        return _ESCAPED_LITERALS[delim]
    return delim if delim and re.escape(delim) == delim else None


def split_regex(delim: str):
    """A splitter for the reference's ``field.delim.regex`` (Java ``String.split(regex)``): plain
    ``str.split`` for a literal separator (one or several characters, e.g. the ``,,`` of the REST
    record lists), a compiled regex otherwise."""
    import re
    lit = _literal(delim)
    if lit is not None:
        return lambda s: s.split(lit)
    return re.compile(delim).split


def _is_regex(delim: str) -> bool:
    return _literal(delim or ",") is None


def pad16(n: int) -> int:
    return max(16, ((n + 15) // 16) * 16)


@dataclass
class Table:
    schema: FeatureSchema | None
    n: int
    codes: torch.Tensor                      # uint8 [Fb, ld]
    binned_fields: list[FeatureField]
    numeric: torch.Tensor                    # float32 [Fn, ld]
    numeric_fields: list[FeatureField]
    labels: torch.Tensor | None = None       # uint8 [ld]
    class_field: FeatureField | None = None
    ids: list[str] | None = None
    lines: list[str] | None = None
    row_offset: int = 0                      # global index of row 0 (sharded loads)
    meta: dict = field(default_factory=dict)
    rowpack: object | None = None            # ops.histogram.RowPacked (see pack_rows)

    # -- geometry ---------------------------------------------------------------------------------
    @property
    def ld(self) -> int:
        return int(self.codes.shape[1]) if self.codes.numel() else pad16(self.n)

    @property
    def bins(self) -> list[int]:
        return [f.num_bins for f in self.binned_fields]

    @property
    def offsets(self) -> list[int]:
        out, o = [], 0
        for b in self.bins:
            out.append(o)
            o += b
        return out

    @property
    def missing(self) -> int:
        return missing_code(self.codes)

    @property
    def wide(self) -> bool:
        """Codes wider than a byte (uint16, or int32 beyond 65,534 values)."""
        return self.codes.dtype != torch.uint8

    @property
    def total_bins(self) -> int:
        return int(sum(self.bins))

    @property
    def n_classes(self) -> int:
        return len(self.class_field.cardinality) if self.class_field is not None else 1

    @property
    def device(self) -> torch.device:
        return self.codes.device

    def pack_rows(self) -> "Table":
        """Attach the 16-bit row-packed form of the binned codes + class
        (``ops.histogram.pack_rows``) when the schema fits; Naive Bayes training then streams
        2 bytes per record instead of one byte per code column.  No-op when it does not fit."""
        from ..ops.histogram import pack_rows
        self.rowpack = pack_rows(self.codes, self.n, self.bins, self.labels, self.n_classes)
        return self

    def to(self, device) -> "Table":
        dev = torch.device(device)
        return Table(self.schema, self.n, self.codes.to(dev), self.binned_fields,
                     self.numeric.to(dev), self.numeric_fields,
                     None if self.labels is None else self.labels.to(dev), self.class_field,
                     self.ids, self.lines, self.row_offset, dict(self.meta))

    def slice_rows(self, start: int, end: int) -> "Table":
        """Row range [start, end) as a new table (copies into a fresh 16-aligned layout)."""
        end = min(end, self.n)
        m = max(0, end - start)
        ld = pad16(m)
        codes = torch.full((self.codes.shape[0], ld), self.missing, dtype=self.codes.dtype, device=self.device)
        codes[:, :m] = self.codes[:, start:end]
        num = torch.zeros((self.numeric.shape[0], ld), dtype=torch.float32, device=self.device)
        num[:, :m] = self.numeric[:, start:end]
        lab = None
        if self.labels is not None:
            lab = torch.full((ld,), MISSING, dtype=torch.uint8, device=self.device)
            lab[:m] = self.labels[start:end]
        return Table(self.schema, m, codes, self.binned_fields, num, self.numeric_fields, lab,
                     self.class_field, self.ids[start:end] if self.ids else None,
                     self.lines[start:end] if self.lines else None, self.row_offset + start,
                     dict(self.meta))

    def select_rows(self, idx: torch.Tensor) -> "Table":
        idx = idx.to(self.device).long()
        m = int(idx.numel())
        ld = pad16(m)
        codes = torch.full((self.codes.shape[0], ld), self.missing, dtype=self.codes.dtype, device=self.device)
        codes[:, :m] = self.codes[:, idx]
        num = torch.zeros((self.numeric.shape[0], ld), dtype=torch.float32, device=self.device)
        num[:, :m] = self.numeric[:, idx]
        lab = None
        if self.labels is not None:
            lab = torch.full((ld,), MISSING, dtype=torch.uint8, device=self.device)
            lab[:m] = self.labels[idx]
        il = idx.cpu().tolist()
        return Table(self.schema, m, codes, self.binned_fields, num, self.numeric_fields, lab,
                     self.class_field, [self.ids[i] for i in il] if self.ids else None,
                     _select_lines(self.lines, idx, il), 0, dict(self.meta))

    def label_values(self) -> list[str]:
        if self.class_field is None or self.labels is None:
            return []
        card = self.class_field.cardinality
        return [card[c] if c < len(card) else "" for c in self.labels[: self.n].cpu().tolist()]

    def dense_features(self, one_hot: bool = False) -> torch.Tensor:
        """[n, D] float32 feature matrix (numeric as-is, binned as code or one-hot) in schema order."""
        cols = []
        fields = sorted([(f.ordinal, "b", i) for i, f in enumerate(self.binned_fields)] +
                        [(f.ordinal, "n", i) for i, f in enumerate(self.numeric_fields)])
        for _, kind, i in fields:
            if kind == "n":
                cols.append(self.numeric[i, : self.n].unsqueeze(1))
            else:
                c = self.codes[i, : self.n].long()
                if one_hot:
                    b = self.binned_fields[i].num_bins
                    oh = torch.zeros((self.n, b), dtype=torch.float32, device=self.device)
                    ok = c < b
                    oh[ok.nonzero().squeeze(1), c[ok]] = 1.0
                    cols.append(oh)
                else:
                    cols.append(c.float().unsqueeze(1))
        if not cols:
            return torch.zeros((self.n, 0), device=self.device)
        return torch.cat(cols, dim=1)


def _select_lines(lines, idx: torch.Tensor, il: list[int]):
    if not lines:
        return None
    from .lines import LineSpans
    if isinstance(lines, LineSpans):
        return lines.select(idx)
    return [lines[i] for i in il]


# ------------------------------------------------------------------------------------------------
def _spec_for(f: FeatureField, width: int = 0) -> tuple:
    """Native parse spec; ``width`` 0 uint8, 1 uint16, 2 int32 codes (categoricals only; buckets
    stay <= uint16)."""
    width = int(width)
    top = (MISSING32 - 1) if width == 2 else (65534 if width else 254)
    if f.is_categorical:
        return (f.ordinal, CAT, list(f.cardinality or []), 1.0, 0, top, width)
    if f.is_bucketed:
        w = min(width, 1)
        return (f.ordinal, BUCKET, [], float(f.bucket_width), f.bucket_offset,
                min(65534 if w else 254, f.num_bins - 1), w)
    return (f.ordinal, FLOAT, [], 1.0, 0, top, 0)


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced row range of ``rank`` (first ``n % world`` ranks get one extra row)."""
    base, rem = divmod(n, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


class LazyColumn(Sequence):
    """A string column of the native CSV file (e.g. the record ids), materialised as Python
    strings on first access: training jobs over 10^8 records never touch the ids, and building
    them eagerly cost more than parsing the file."""

    def __init__(self, csv, ordinal: int, r0: int, r1: int):
        """``csv``: a native CsvFile, or a zero-argument factory of one (the device parser keeps
        no host index, so the host one is only built if the strings are ever asked for)."""
        self._csv, self._ord, self._r0, self._r1 = csv, ordinal, r0, r1
        self._vals: list[str] | None = None

    def _get(self) -> list[str]:
        if self._vals is None:
            csv = self._csv() if callable(self._csv) else self._csv
            self._vals = csv.column_strings(self._ord)[self._r0:self._r1]
            self._csv = None
        return self._vals

    def __len__(self) -> int:
        return self._r1 - self._r0

    def __bool__(self) -> bool:
        return self._r1 > self._r0

    def __getitem__(self, i):
        return self._get()[i]

    def __iter__(self):
        return iter(self._get())

    def __eq__(self, other):
        return list(self._get()) == list(other)


def _nbytes(path) -> int:
    return sum(os.path.getsize(p) for p in path) if isinstance(path, (list, tuple)) else os.path.getsize(path)


@traced("data.load_csv", nbytes=lambda path, *a, **k: _nbytes(path))
def load_csv(path: str | Path | list, schema: FeatureSchema, delim: str = ",", *, rank: int = 0,
             world: int = 1, device: str | torch.device = "cpu", keep_lines: bool = False,
             skip_header: bool = False, nthreads: int | None = None, feature_ordinals: Sequence[int] | None = None,
             class_ordinal: int | None = None, raw_numeric: bool = False) -> Table:
    """Parse ``path`` into a ``Table`` (this rank's shard) with the native K1 parser.

    ``path`` may be a list of files (a Hadoop part-file directory): they are read as one byte
    stream by the native parser, without a temporary concatenated copy.

    ``raw_numeric``: keep int/double features as raw float columns even when the schema gives a
    ``bucketWidth`` (the tree builders bin them by their own split points)."""
    if raw_numeric:
        import copy
        schema = copy.deepcopy(schema)
        for f in schema.fields:
            if f.is_numeric:
                f.bucket_width = None
    feats = [f for f in schema.feature_fields
             if feature_ordinals is None or f.ordinal in set(feature_ordinals)]
    if feature_ordinals is not None:
        # allow selecting non-"feature" fields explicitly
        have = {f.ordinal for f in feats}
        feats += [schema.find_field_by_ordinal(o) for o in feature_ordinals if o not in have]
        feats.sort(key=lambda f: f.ordinal)
    cls_f = (schema.find_field_by_ordinal(class_ordinal) if class_ordinal is not None
             else schema.find_class_attr_field())
    multi = isinstance(path, (list, tuple))
    if multi and len(path) == 1:
        path, multi = path[0], False
    C = _native.host()
    use_native = C is not None and not _is_regex(delim)
    if nthreads is None:    # parse threads: the machine's cores, capped at a GPU box's CPU share
        nthreads = max(1, min(16, os.cpu_count() or 8))
    dev = torch.device(device)
    if (use_native and not multi and dev.type == "cuda" and len(_literal(delim or ",")) == 1
            and hasattr(C, "csv_parse_device") and os.path.getsize(path) >= _GPU_CSV_MIN_BYTES
            and all(f.cardinality or not f.is_categorical for f in feats)
            and (cls_f is None or cls_f.cardinality)):
        t = _load_csv_device(C, path, schema, delim, skip_header, rank, world, dev, feats, cls_f, nthreads,
                             keep_lines)
        if t is not None:
            return t
    if use_native:
        csv = (C.CsvFile([str(p) for p in path], 0, 1, _literal(delim or ","), skip_header, nthreads) if multi
               else C.CsvFile(str(path), _literal(delim or ","), skip_header, nthreads))
    else:
        csv = None
    # categorical fields without a schema cardinality: dictionary in first-seen order over the
    # WHOLE file (identical on every rank), any size (uint16 codes above 255 values)
    for f in feats:
        if f.is_categorical and not f.cardinality:
            if csv is not None:
                f.cardinality = csv.distinct(f.ordinal, MISSING32 - 1)
            else:
                f.cardinality = _distinct_py(_py_lines_of(path, skip_header), f.ordinal, delim)
    binned = [f for f in feats if f.is_binned]
    numeric = [f for f in feats if not f.is_binned and f.is_numeric]
    width = code_width(binned)
    cdt = _CODE_DTYPE[width]
    miss = _MISSING_OF[cdt]
    if csv is not None:
        total = csv.num_rows()
        r0, r1 = shard_range(total, rank, world)
        specs = [_spec_for(f, width) for f in binned] + [_spec_for(f) for f in numeric]
        if cls_f is not None:
            if not cls_f.cardinality:
                cls_f.cardinality = csv.distinct(cls_f.ordinal, 255)
            specs.append(_spec_for(cls_f))
        cols, _bad = csv.parse(specs, r0, r1)
        n = r1 - r0
        ld = pad16(n)
        codes = (torch.stack([c[:ld].to(cdt) if c.dtype != cdt else c[:ld] for c in cols[: len(binned)]])
                 if binned else torch.zeros((0, ld), dtype=cdt))
        if binned and cdt == torch.int32:     # uint16 bucket columns: their missing code -> INT32_MAX
            for j, c in enumerate(cols[: len(binned)]):
                if c.dtype == torch.uint16:
                    codes[j][codes[j] == MISSING16] = MISSING32
        numc = cols[len(binned): len(binned) + len(numeric)]
        num = torch.zeros((len(numeric), ld), dtype=torch.float32)
        for i, c in enumerate(numc):
            num[i, :n] = c
        labels = cols[-1][:ld].clone() if cls_f is not None else None
        ids = None
        idf = schema.id_field
        lines = None
        if idf is not None:
            ids = LazyColumn(csv, idf.ordinal, r0, r1)
        if keep_lines:   # byte spans into the mapped file, strings only on demand (data/lines.py)
            from .lines import LineSpans
            lines = LineSpans.from_csv(csv, r0, r1)
    else:  # pure-Python path: regex delimiters, or no native module
        all_lines = _py_lines_of(path, skip_header)
        r0, r1 = shard_range(len(all_lines), rank, world)
        splitter = split_regex(delim or ",")
        rows = [splitter(ln) for ln in all_lines[r0:r1]]
        n = len(rows)
        ld = pad16(n)
        codes = torch.full((len(binned), ld), miss, dtype=cdt)
        for j, f in enumerate(binned):
            if f.is_categorical:     # dictionary lookup (first occurrence wins, as the native parser)
                lut: dict[str, int] = {}
                for i, v in enumerate(f.cardinality):
                    lut.setdefault(v, i)
                vals = [lut.get(r[f.ordinal].strip(), miss) if f.ordinal < len(r) else miss for r in rows]
            else:
                vals = [_encode_py(f, r[f.ordinal] if f.ordinal < len(r) else "", miss) for r in rows]
            codes[j, :n] = torch.tensor(vals, dtype=torch.int64).to(cdt)
        num = torch.zeros((len(numeric), ld), dtype=torch.float32)
        for j, f in enumerate(numeric):
            num[j, :n] = torch.tensor([_float(r[f.ordinal]) if f.ordinal < len(r) else math.nan
                                       for r in rows])
        labels = None
        if cls_f is not None:
            if not cls_f.cardinality:
                seen: dict[str, None] = {}
                for r in rows:
                    seen.setdefault(r[cls_f.ordinal].strip(), None)
                cls_f.cardinality = list(seen)
            labels = torch.full((ld,), MISSING, dtype=torch.uint8)
            labels[:n] = torch.tensor([_encode_py(cls_f, r[cls_f.ordinal]) for r in rows],
                                      dtype=torch.uint8)
        idf = schema.id_field
        ids = [r[idf.ordinal] for r in rows] if idf is not None else None
        lines = None
        if keep_lines:
            from .lines import LineSpans
            lines = LineSpans.from_strings(all_lines[r0:r1])
    t = Table(schema, n, codes, binned, num, numeric, labels, cls_f, ids, lines, r0,
              meta={"parser": "host" if csv is not None else "python"})
    return t.to(device) if str(device) != "cpu" else t


_GPU_CSV_MIN_BYTES = int(os.environ.get("AVMI_GPU_CSV_MIN_BYTES", str(32 << 20)))


def _load_csv_device(C, path, schema, delim, skip_header, rank, world, dev, feats, cls_f, nthreads,
                     keep_lines: bool = False):
    """K1 on the GPU (csrc/kernels/csv.hip): upload the file, index lines and parse the schema's
    columns on the device (in passes of up to 64 columns); same codes as the host parser.  None when
    a column kind needs the host path (int32 codes).  ``keep_lines``: the rows' byte spans in the
    file (from the device line index) as a lazy data/lines.LineSpans."""
    binned = [f for f in feats if f.is_binned]
    numeric = [f for f in feats if not f.is_binned and f.is_numeric]
    width = code_width(binned)
    if width > 1:
        return None                          # int32 codes: the host parser
    wide = width == 1
    specs = [_spec_for(f, width) for f in binned] + [_spec_for(f) for f in numeric]
    if cls_f is not None:
        specs.append(_spec_for(cls_f))
    if any(sp[1] not in (CAT, BUCKET, FLOAT) for sp in specs):
        return None
    like = torch.empty(0, device=dev)
    r = C.csv_parse_device(str(path), specs, _literal(delim or ","), skip_header, int(rank), int(world), like)
    if r is None:       # a number the device could not round for certain: the host parser (strtod)
        return None
    cols, n, _bad, _total, r0, starts, ends, fbytes = r
    ld = pad16(n)
    cdt = torch.uint16 if wide else torch.uint8
    codes = (torch.stack([c[:ld] for c in cols[: len(binned)]]) if binned
             else torch.zeros((0, ld), dtype=cdt, device=dev))
    num = torch.zeros((len(numeric), ld), dtype=torch.float32, device=dev)
    for i, c in enumerate(cols[len(binned): len(binned) + len(numeric)]):
        num[i, :n] = c[:n]
    labels = cols[-1][:ld] if cls_f is not None else None
    idf = schema.id_field
    ids = None
    if idf is not None:
        lit = _literal(delim or ",")
        ids = LazyColumn(lambda: C.CsvFile(str(path), lit, skip_header, nthreads), idf.ordinal, r0, r0 + n)
    lines = None
    if keep_lines:
        from .lines import LineSpans
        lines = LineSpans.from_file(str(path), starts, ends)
        lines.dev = (fbytes, starts, ends - starts)      # the device formatter reads the uploaded bytes
    return Table(schema, n, codes, binned, num, numeric, labels, cls_f, ids, lines, r0, meta={"parser": "device"})


def _py_lines_of(path, skip_header: bool) -> list[str]:
    """Non-blank lines of one file or a list of files (pure-Python path)."""
    out: list[str] = []
    for p in (path if isinstance(path, (list, tuple)) else [path]):
        with open(p) as fh:
            out += [ln.rstrip("\r\n") for ln in fh if ln.strip()]
    return out[1:] if skip_header else out


def _distinct_py(lines: list[str], ordinal: int, delim: str) -> list[str]:
    split = split_regex(delim or ",")
    seen: dict[str, None] = {}
    for ln in lines:
        r = split(ln)
        if ordinal < len(r):
            seen.setdefault(r[ordinal].strip(), None)
    return list(seen)


def _float(s: str) -> float:
    try:
        return float(s)
    except ValueError:
        return math.nan


def _encode_py(f: FeatureField, s: str, missing: int = MISSING) -> int:
    s = s.strip()
    if f.is_categorical:
        try:
            return f.cardinality.index(s)
        except ValueError:
            return missing
    v = _float(s)
    if math.isnan(v):
        return missing
    b = int(math.floor(v / f.bucket_width)) - f.bucket_offset
    return b if 0 <= b < min(missing, f.num_bins) else missing


def from_arrays(schema: FeatureSchema, columns: dict[int, Sequence], device="cpu") -> Table:
    """Build a Table from in-memory columns keyed by ordinal (strings or numbers)."""
    feats = schema.feature_fields
    cls_f = schema.find_class_attr_field()
    binned = [f for f in feats if f.is_binned]
    numeric = [f for f in feats if not f.is_binned and f.is_numeric]
    n = len(next(iter(columns.values())))
    ld = pad16(n)
    cdt = _CODE_DTYPE[code_width(binned)]
    miss = _MISSING_OF[cdt]
    codes = torch.full((len(binned), ld), miss, dtype=cdt)
    for j, f in enumerate(binned):
        lut = {v: i for i, v in enumerate(f.cardinality)} if f.is_categorical else None
        vals = ([lut.get(str(v).strip(), miss) for v in columns[f.ordinal]] if lut is not None
                else [_encode_py(f, str(v), miss) for v in columns[f.ordinal]])
        codes[j, :n] = torch.tensor(vals, dtype=torch.int64).to(codes.dtype)
    num = torch.zeros((len(numeric), ld), dtype=torch.float32)
    for j, f in enumerate(numeric):
        num[j, :n] = torch.tensor(np.asarray(columns[f.ordinal], dtype=np.float32))
    labels = None
    if cls_f is not None and cls_f.ordinal in columns:
        labels = torch.full((ld,), MISSING, dtype=torch.uint8)
        labels[:n] = torch.tensor([_encode_py(cls_f, str(v)) for v in columns[cls_f.ordinal]],
                                  dtype=torch.uint8)
    idf = schema.id_field
    ids = [str(v) for v in columns[idf.ordinal]] if idf is not None and idf.ordinal in columns else None
    return Table(schema, n, codes, binned, num, numeric, labels, cls_f, ids).to(device)
