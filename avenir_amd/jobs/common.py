"""Shared plumbing of the CLI jobs: registry, config, sharded text input, rank-aware output.

Every reference job is launched as ``<class> -Dconf.path=<props> in out`` (Hadoop) or
``<object> in out <hocon>`` (Spark, ``getCommandLineArgs(args, 3)``, e.g.
S/util/LinearMapper.scala:40-99).  Here a job is a function ``fn(ctx)`` registered under the
reference's job name; ``ctx`` (a :class:`JobContext`) carries the typed config (``.properties``
with the job's key prefix, or the HOCON app block), the input shard of this rank and the output
writer.

Distributed semantics (one process per GPU under ``torchrun``; RCCL collectives):

* map-only jobs (predictors, samplers, transforms) read a contiguous block of the input lines
  per rank and write their own ``part-NNNNN`` file (Hadoop's one-file-per-mapper) when the output
  is a directory, or gather their lines to rank 0 (rank order) when it is a single file;
* reducing jobs (models, statistics) build dense partial tensors per rank, all-reduce them once
  and write from rank 0 only.
"""
from __future__ import annotations

import json
import sys
from collections import Counter
from pathlib import Path
from typing import Callable, Iterable, Sequence

import torch

JOBS: dict[str, tuple[Callable, str]] = {}

#: input bytes this process read through ``JobContext.records`` (per-rank byte-range evidence for
#: the data-parallel tests; a Hadoop-style counter)
IO_STATS = {"bytes_read": 0}


def job(name: str, help_: str, aliases: Sequence[str] = ()):
    def deco(fn):
        JOBS[name] = (fn, help_)
        for a in aliases:
            JOBS[a] = (fn, f"alias of {name}")
        return fn
    return deco


def parse_defines(defs: Sequence[str] | None) -> dict[str, str]:
    """``-D key=value`` overrides (Hadoop's generic ``-D`` option)."""
    out = {}
    for d in defs or []:
        if "=" not in d:
            raise SystemExit(f"-D expects key=value, got {d!r}")
        k, v = d.split("=", 1)
        out[k.strip()] = v
    return out


class JobContext:
    """Per-job view of the CLI arguments: config, device, communicator, I/O helpers."""

    def __init__(self, args, prefix: str = "", app: str | None = None):
        from ..parallel.comm import get_comm
        from ..utils.config import JobConfig
        self.args = args
        app = getattr(args, "app", None) or app
        if getattr(args, "config", None):
            if str(args.config).endswith(".conf") and app is None:
                # a HOCON file with a block named after the job (the Spark appName)
                from ..utils.config import read_hocon
                if getattr(args, "job", None) in read_hocon(args.config):
                    app = args.job
            self.cfg = JobConfig.from_file(args.config, prefix, app if str(args.config).endswith(".conf") else None)
        else:
            self.cfg = JobConfig({}, prefix)
        self.cfg.update(parse_defines(getattr(args, "define", None)))
        self.comm = get_comm()
        dev = getattr(args, "device", None)
        self.device = torch.device(dev) if dev else torch.device("cuda" if torch.cuda.is_available() else "cpu")

    # -- config shortcuts ---------------------------------------------------------------------
    def __getattr__(self, name):
        # cfg.get_int / get_str / ... reachable as ctx.get_int(...)
        if name.startswith("get") or name == "has":
            return getattr(self.cfg, name)
        raise AttributeError(name)

    @property
    def delim_in(self) -> str:
        return self.cfg.get_str("field.delim.regex", None) or self.cfg.get_str("field.delim.in", None) or ","

    @property
    def delim_out(self) -> str:
        return self.cfg.get_str("field.delim.out", None) or self.cfg.get_str("field.delim", None) or ","

    @property
    def split(self) -> Callable[[str], list[str]]:
        from ..data.table import split_regex
        return split_regex(self.delim_in)

    def path(self, key: str | None = None, arg: str | None = None, default=None) -> str:
        """A side-file path: the CLI flag ``arg`` if given, else config ``key`` (made relative to the
        config file's directory when it does not exist as given)."""
        v = getattr(self.args, arg, None) if arg else None
        if not v and key is not None:
            v = self.cfg.get_str(key, default)
        if v is None:
            raise SystemExit(f"missing path: --{arg or ''} / {self.cfg.prefix}{key}")
        p = Path(v)
        if not p.exists() and getattr(self.args, "config", None):
            alt = Path(self.args.config).parent / v
            if alt.exists():
                return str(alt)
        return str(p)

    def schema(self, key: str = "feature.schema.file.path"):
        from ..utils.schema import FeatureSchema
        p = getattr(self.args, "schema", None) or self.cfg.get_str(key, None)
        if not p:
            for k in ("feature.schema.file.path", "schema.file.path"):
                p = p or self.cfg.get_str(k, None)
        if not p:
            raise SystemExit("a feature schema is required (--schema or *.schema.file.path)")
        return FeatureSchema.from_json(Path(self.path(None, None, p) if not Path(p).exists() else p))

    def adhoc_schema(self, cat_ords, class_ord: int | None = None, num_ords=()):
        """A schema built from config ordinals (jobs whose reference reads ordinals, not a schema
        file): categorical features with dictionaries discovered from the data, optional numeric
        features and class attribute."""
        from ..utils.schema import FeatureField, FeatureSchema
        fields = [FeatureField(f"f{o}", o, "categorical", feature=True) for o in cat_ords]
        fields += [FeatureField(f"f{o}", o, "double", feature=True) for o in num_ords]
        if class_ord is not None:
            fields.append(FeatureField(f"f{class_ord}", class_ord, "categorical", extra={"classAttribute": True}))
        return FeatureSchema(fields)

    # -- input --------------------------------------------------------------------------------
    def all_lines(self, path: str | None = None) -> list[str]:
        """Every non-blank line of ``path`` (side files read whole by every rank)."""
        from ..data.records import shard_lines
        return shard_lines(path or self.args.input, None, shard=False)

    def lines(self, path: str | None = None, shard: bool = True) -> list[str]:
        """This rank's lines: the native byte-range shard of the input (a rank reads only the bytes of
        its range; a line belongs to the rank whose range holds its first byte).  All lines when
        ``shard=False`` or not distributed."""
        from ..data.records import shard_lines
        return shard_lines(path or self.args.input, self.comm, shard=shard)

    def rows(self, path: str | None = None, shard: bool = True, keep_empty: bool = True) -> list[list[str]]:
        sp = self.split
        return [sp(l) for l in self.lines(path, shard)]

    def records(self, path: str | None = None, shard: bool = True, **kw):
        """This rank's CSR token table of the input (data/records.py): one native pass (device
        tokenizer on a GPU), dictionary merged over ranks.  ``kw``: modes / tail_mode / sub_delim /
        numeric / trim / delims (default: the job's literal field delimiter)."""
        from ..data.records import read_records
        from ..data.table import _literal
        if "delims" not in kw:
            lit = _literal(self.delim_in)
            if lit is None or len(lit) != 1:
                raise SystemExit(f"native record input needs a one-character field delimiter, got {self.delim_in!r}")
            kw["delims"] = lit
        rec = read_records(path or self.args.input, comm=self.comm, device=self.device, shard=shard, **kw)
        IO_STATS["bytes_read"] += int(rec.stats.get("bytes", 0))
        return rec

    def native_delim(self) -> str | None:
        """The job's field delimiter when it is one literal character (native tokenizers), else None."""
        from ..data.table import _literal
        lit = _literal(self.delim_in)
        return lit if lit is not None and len(lit) == 1 else None

    def try_records(self, path: str | None = None, shard: bool = True, **kw):
        """:meth:`records` when the input delimiter is one literal character, else None (the job
        then takes its split-row path)."""
        if self.native_delim() is None:
            return None
        return self.records(path, shard=shard, **kw)

    def numeric_matrix(self, ords, dtype=torch.float64, path: str | None = None, shard: bool = True, **kw):
        """(X [n, len(ords)] on the job's device, Records or None): fields ``ords`` parsed as
        numbers — natively (mode 'n' at those fields, the rest skipped; ``kw`` adds modes for other
        fields, e.g. ``extra={0: 'd'}``) or, for a regex delimiter, from split rows (then the
        second value is the row list)."""
        ords = list(ords)
        extra = dict(kw.pop("extra", {}))
        rec = self.try_records(path, shard=shard, modes=field_modes({**{o: "n" for o in ords}, **extra}),
                               tail_mode="x", numeric=True, **kw)
        if rec is None:
            rows = self.rows(path, shard)
            X = torch.tensor([[float(r[o]) for o in ords] for r in rows], dtype=dtype).view(len(rows), len(ords))
            return X.to(self.device), rows
        if not ords:
            return torch.zeros((rec.n_lines, 0), dtype=dtype, device=rec.device), rec
        return torch.stack([rec.field(o, numeric=True) for o in ords], 1).to(dtype), rec

    def line_base(self, n_local: int) -> int:
        """Global index of this rank's first line (exclusive scan of the line counts)."""
        if not self.comm.is_distributed:
            return 0
        counts = self.comm.all_gather_object(int(n_local))
        return int(sum(counts[: self.comm.rank]))

    def table(self, raw_numeric: bool = False, path: str | None = None, schema=None, shard: bool = True):
        from ..data.table import load_csv
        comm = self.comm
        path = str(path or self.args.input)
        files = input_files(path)
        src = [str(f) for f in files] if len(files) != 1 else str(files[0])
        return load_csv(src, schema or self.schema(), self.delim_in,
                        rank=comm.rank if shard else 0, world=comm.world if shard else 1,
                        device=self.device, keep_lines=True, raw_numeric=raw_numeric)

    # -- collectives on host objects ------------------------------------------------------------
    def union(self, items: Iterable) -> list:
        """Sorted union of a set of hashable keys over all ranks (shared vocabulary)."""
        s = set(items)
        if self.comm.is_distributed:
            for part in self.comm.all_gather_object(sorted(s, key=str)):
                s.update(part)
        return sorted(s, key=str)

    def sum_counts(self, c: Counter | dict) -> Counter:
        """Merge a host ``Counter`` over ranks (sparse string-keyed reductions)."""
        out = Counter(c)
        if self.comm.is_distributed:
            out = Counter()
            for part in self.comm.all_gather_object(dict(c)):
                out.update(part)
        return out

    def all_reduce(self, *ts: torch.Tensor) -> None:
        if self.comm.is_distributed:
            self.comm.all_reduce_coalesced(list(ts))

    def gather_lines(self, lines: list[str]) -> list[str]:
        if not self.comm.is_distributed:
            return lines
        out = []
        for part in self.comm.all_gather_object(lines):
            out += part
        return out

    @property
    def is_root(self) -> bool:
        return self.comm.rank == 0

    # -- output -------------------------------------------------------------------------------
    def check(self) -> None:
        """Output gate: raise P2PError if a peer-mapped sum of this rank failed (local; waits for
        the last one), so no output is ever written from a failed collective.  Every emit method
        calls it; jobs that write files themselves call it first."""
        self.comm.check()

    def _target(self, out: str | None = None) -> tuple[Path, bool]:
        p = Path(out or self.args.output)
        is_dir = p.is_dir() or (p.suffix == "" and not p.exists())
        return p, is_dir

    def emit(self, lines: list[str], out: str | None = None) -> Path | None:
        """Map-side output: per-rank part file into a directory, or rank-ordered single file."""
        self.check()
        p, is_dir = self._target(out)
        if is_dir:
            p.mkdir(parents=True, exist_ok=True)
            t = p / f"part-{self.comm.rank:05d}"
            _write_text(t, lines)
            return t
        lines = self.gather_lines(lines)
        if self.is_root:
            _write_text(p, lines)
            return p
        return None

    def emit_text(self, text: bytes, out: str | None = None) -> Path | None:
        """Map-side output of pre-formatted text (data/records.format_lines): this rank's part file
        into a directory, or the rank-ordered concatenation written by rank 0."""
        self.check()
        p, is_dir = self._target(out)
        if is_dir:
            p.mkdir(parents=True, exist_ok=True)
            t = p / f"part-{self.comm.rank:05d}"
            t.write_bytes(text)
            return t
        if self.comm.is_distributed:
            text = b"".join(self.comm.all_gather_object(text))
        if self.is_root:
            p.parent.mkdir(parents=True, exist_ok=True)
            p.write_bytes(text)
            return p
        return None

    def emit_columns(self, cols: list, n: int, out: str | None = None) -> Path | None:
        """Map-side output of ``data/records.format_lines`` columns: this rank's part file into a
        directory (or the whole file when not distributed) written straight from the native
        formatter's threads; a single-file output of several ranks is gathered to rank 0."""
        self.check()
        from ..data.records import format_lines
        p, is_dir = self._target(out)
        if is_dir or not self.comm.is_distributed:
            if is_dir:
                p.mkdir(parents=True, exist_ok=True)
                p = p / f"part-{self.comm.rank:05d}"
            else:
                p.parent.mkdir(parents=True, exist_ok=True)
            format_lines(cols, n, self.delim_out, path=str(p))
            return p
        return self.emit_text(format_lines(cols, n, self.delim_out), out)

    def emit_root_columns(self, cols: list, n: int, out: str | None = None, name: str = "part-00000") -> Path | None:
        """Reduce-side output of ``format_lines`` columns: rank 0 writes them."""
        self.check()
        from ..data.records import format_lines
        if not self.is_root:
            return None
        p, is_dir = self._target(out)
        if is_dir:
            p.mkdir(parents=True, exist_ok=True)
            p = p / name
        p.parent.mkdir(parents=True, exist_ok=True)
        format_lines(cols, n, self.delim_out, path=str(p))
        return p

    def emit_root_text(self, text: bytes, out: str | None = None, name: str = "part-00000") -> Path | None:
        """Reduce-side output of pre-formatted text: rank 0 writes it."""
        self.check()
        if not self.is_root:
            return None
        p, is_dir = self._target(out)
        if is_dir:
            p.mkdir(parents=True, exist_ok=True)
            p = p / name
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_bytes(text)
        return p

    def emit_root(self, lines: list[str], out: str | None = None, name: str = "part-00000") -> Path | None:
        """Reduce-side output: rank 0 writes the (already reduced) result."""
        self.check()
        if not self.is_root:
            return None
        p, is_dir = self._target(out)
        if is_dir:
            p.mkdir(parents=True, exist_ok=True)
            p = p / name
        _write_text(p, lines)
        return p

    def emit_json(self, obj, out: str | None = None) -> None:
        self.check()
        if self.is_root:
            p = Path(out or self.args.output)
            p.parent.mkdir(parents=True, exist_ok=True)
            p.write_text(json.dumps(obj, indent=1))

    def report(self, obj: dict) -> None:
        """Counters / summary line on stdout (Hadoop job counters)."""
        if self.is_root:
            print(json.dumps(obj, default=str), flush=True)


def _write_text(p: Path, lines: list[str]) -> None:
    p.parent.mkdir(parents=True, exist_ok=True)
    p.write_text("\n".join(lines) + ("\n" if lines else ""))


def read_lines(path: str | Sequence[str]) -> list[str]:
    """Non-empty lines of a file, or of every visible file of a directory (sorted, Hadoop part
    files), or of a comma-separated list of those (``FileInputFormat.addInputPaths``)."""
    paths = [path] if isinstance(path, (str, Path)) else list(path)
    out: list[str] = []
    for ps in paths:
        for one in str(ps).split(",") if not Path(str(ps)).exists() else [str(ps)]:
            p = Path(one)
            files = (sorted(f for f in p.iterdir() if f.is_file() and not f.name.startswith((".", "_")))
                     if p.is_dir() else [p])
            for f in files:
                out += [l for l in f.read_text().splitlines() if l.strip()]
    return out


def input_files(path: str) -> list[Path]:
    """The files behind an input path (comma list / directory / file)."""
    out = []
    for one in str(path).split(","):
        p = Path(one)
        out += (sorted(f for f in p.iterdir() if f.is_file() and not f.name.startswith((".", "_")))
                if p.is_dir() else [p])
    return out


def field_modes(spec: dict[int, str], default: str = "x") -> str:
    """Per-field tokenizer mode string (``data/records.read_records``) from ``{field: mode}``."""
    if not spec:
        return ""
    return "".join(spec.get(j, default) for j in range(max(spec) + 1))


def field_columns(spans, width: int, delims: str, replace: dict | None = None, drop=()) -> list:
    """``format_lines`` columns re-emitting fields ``0..width-1`` of each raw line (byte spans),
    with ``replace[j]`` columns (one column or a list) in place of field j and ``drop`` removed."""
    replace = replace or {}
    cols = []
    for j in range(width):
        if j in replace:
            r = replace[j]
            cols += r if isinstance(r, list) else [r]
        elif j not in drop:
            cols.append(spans.column("rf", j, delims))
    return cols


def fmt(x: float, prec: int = 3) -> str:
    """``BasicUtils.formatDouble(x, prec)``."""
    return f"{x:.{prec}f}"


def die(msg: str) -> None:
    print(msg, file=sys.stderr)
    raise SystemExit(2)
