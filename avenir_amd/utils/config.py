"""Unified configuration system (SURVEY.md §5.6 / layer N2).

Reads all three legacy configuration dialects of the reference, unchanged:

1. **Java ``.properties``** with per-job key prefixes (``dtb.``, ``bad.``, ``nen.`` ...) and global
   keys (``field.delim.regex``, ``num.reducer``, ``debug.on``), as loaded by chombo's
   ``Utility.setConfiguration(conf, "avenir")`` (reference: e.g.
   ``src/main/java/org/avenir/tree/DecisionTreeBuilder.java:75``).  Prefixed lookup falls back to
   the un-prefixed key, mirroring ``dtb.num.reducer`` -> ``num.reducer``
   (``DecisionTreeBuilder.java:89-91``).
2. **HOCON** application blocks used by the Spark jobs (``resource/opt.conf``, ``samp.conf``):
   ``appName { key = value ... nested { ... } }``, arrays ``["a","b"]``, quoted/unquoted strings,
   ``#`` and ``//`` comments.
3. **jprops-style Python configs** (``python/lib/mlutil.py:34-231``): a defaults table
   ``{key: (default, error_if_missing)}``, ``_`` means "use default", ``none`` means None, typed
   getters return ``(value, is_default)``, programmatic ``set_param``/``override``.
"""
from __future__ import annotations

import json
import re
from pathlib import Path
from typing import Any, Iterable

__all__ = ["read_properties", "parse_properties", "parse_hocon", "read_hocon", "JobConfig",
           "Configuration"]


# --------------------------------------------------------------------------------------------
# Java properties
# --------------------------------------------------------------------------------------------
def parse_properties(text: str) -> dict[str, str]:
    """Parse Java ``.properties`` text (``=``/``:``/whitespace separators, ``#``/``!`` comments,
    backslash line continuation and escapes)."""
    out: dict[str, str] = {}
    lines = text.splitlines()
    i = 0
    while i < len(lines):
        line = lines[i].lstrip()
        i += 1
        if not line or line[0] in "#!":
            continue
        while line.endswith("\\") and not line.endswith("\\\\") and i < len(lines):
            line = line[:-1] + lines[i].lstrip()
            i += 1
        # find the separator (first unescaped '=', ':' or whitespace)
        key_chars = []
        j = 0
        while j < len(line):
            ch = line[j]
            if ch == "\\" and j + 1 < len(line):
                key_chars.append(line[j + 1])
                j += 2
                continue
            if ch in "=:" or ch.isspace():
                break
            key_chars.append(ch)
            j += 1
        rest = line[j:].lstrip()
        if rest[:1] in ("=", ":"):
            rest = rest[1:].lstrip()
        value = rest.replace("\\t", "\t").replace("\\n", "\n").replace("\\\\", "\\")
        out["".join(key_chars)] = value.rstrip()
    return out


def read_properties(path: str | Path) -> dict[str, str]:
    return parse_properties(Path(path).read_text())


# --------------------------------------------------------------------------------------------
# HOCON (the subset used by the reference's Spark configs)
# --------------------------------------------------------------------------------------------
_TOKEN = re.compile(r'\s*(?:(#[^\n]*|//[^\n]*)|("(?:[^"\\]|\\.)*")|([{}\[\],=:\n])|([^\s{}\[\],=:"#]+(?:[ \t]+[^\s{}\[\],=:"#]+)*))')


def _hocon_tokens(text: str) -> list[tuple[str, str]]:
    toks: list[tuple[str, str]] = []
    pos = 0
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m or m.end() == pos:
            if text[pos:].strip() == "":
                break
            raise ValueError(f"HOCON parse error near: {text[pos:pos + 40]!r}")
        pos = m.end()
        if m.group(1):
            continue
        if m.group(2) is not None:
            toks.append(("str", json.loads(m.group(2))))
        elif m.group(3) is not None:
            toks.append(("sym", m.group(3)))
        elif m.group(4) is not None:
            toks.append(("word", m.group(4)))
    return toks


def _hocon_scalar(word: str) -> Any:
    lw = word.lower()
    if lw == "true":
        return True
    if lw == "false":
        return False
    if lw == "null":
        return None
    try:
        return int(word)
    except ValueError:
        pass
    try:
        return float(word)
    except ValueError:
        return word


def parse_hocon(text: str) -> dict[str, Any]:
    toks = _hocon_tokens(text)
    pos = 0

    def skip_nl():
        nonlocal pos
        while pos < len(toks) and toks[pos] == ("sym", "\n"):
            pos += 1

    def parse_value():
        nonlocal pos
        skip_nl()
        kind, val = toks[pos]
        if kind == "sym" and val == "{":
            pos += 1
            return parse_object(end="}")
        if kind == "sym" and val == "[":
            pos += 1
            arr = []
            while True:
                skip_nl()
                if toks[pos] == ("sym", "]"):
                    pos += 1
                    return arr
                arr.append(parse_value())
                skip_nl()
                if toks[pos] == ("sym", ","):
                    pos += 1
        pos += 1
        return val if kind == "str" else _hocon_scalar(val)

    def set_path(obj: dict, key: str, value: Any):
        # the reference's keys are flat dotted names ("max.num.iterations"): keep them flat
        if isinstance(value, dict) and isinstance(obj.get(key), dict):
            obj[key].update(value)
        else:
            obj[key] = value

    def parse_object(end: str | None):
        nonlocal pos
        obj: dict[str, Any] = {}
        while True:
            skip_nl()
            if pos >= len(toks):
                if end is None:
                    return obj
                raise ValueError("HOCON: unterminated object")
            kind, val = toks[pos]
            if kind == "sym" and val == end:
                pos += 1
                return obj
            if kind == "sym" and val == ",":
                pos += 1
                continue
            key = val
            pos += 1
            skip_nl()
            if toks[pos] in (("sym", "="), ("sym", ":")):
                pos += 1
            set_path(obj, key, parse_value())

    return parse_object(end=None)


def read_hocon(path: str | Path) -> dict[str, Any]:
    return parse_hocon(Path(path).read_text())


# --------------------------------------------------------------------------------------------
# JobConfig: typed access to one job's flat properties (Java MR style) or one HOCON app block
# --------------------------------------------------------------------------------------------
_MISSING = object()


class JobConfig:
    """Typed view over a flat key/value config with an optional per-job key prefix.

    ``cfg.get_int("num.reducer", 1)`` looks up ``<prefix>num.reducer`` then ``num.reducer``.
    Works for Java ``.properties`` dicts and for HOCON app blocks (whose values may already be
    typed).  Missing mandatory keys raise ``KeyError`` with the key name (like chombo's
    ``getMandatory*Param``).
    """

    def __init__(self, values: dict[str, Any] | None = None, prefix: str = ""):
        self.values: dict[str, Any] = dict(values or {})
        self.prefix = prefix

    # -- construction --------------------------------------------------------------------------
    @classmethod
    def from_file(cls, path: str | Path, prefix: str = "", app: str | None = None) -> "JobConfig":
        p = Path(path)
        if p.suffix == ".conf":
            data = read_hocon(p)
            if app is not None:
                if app not in data:
                    raise KeyError(f"HOCON file {p} has no block {app!r}")
                data = data[app]
            return cls(_flatten(data), prefix)
        if p.suffix == ".json":
            return cls(json.loads(p.read_text()), prefix)
        return cls(read_properties(p), prefix)

    def with_prefix(self, prefix: str) -> "JobConfig":
        return JobConfig(self.values, prefix)

    def set(self, key: str, value: Any) -> None:
        self.values[key] = value

    def update(self, kv: dict[str, Any]) -> None:
        self.values.update(kv)

    # -- lookup --------------------------------------------------------------------------------
    def _raw(self, key: str, default: Any = _MISSING) -> Any:
        for k in ((self.prefix + key) if self.prefix else None, key):
            if k is not None and k in self.values:
                return self.values[k]
        if default is _MISSING:
            raise KeyError(f"missing mandatory config key: {self.prefix}{key}")
        return default

    def has(self, key: str) -> bool:
        return self._raw(key, None) is not None

    def get(self, key: str, default: Any = _MISSING) -> Any:
        return self._raw(key, default)

    def get_str(self, key: str, default: Any = _MISSING) -> str | None:
        v = self._raw(key, default)
        return None if v is None else str(v)

    def get_int(self, key: str, default: Any = _MISSING) -> int | None:
        v = self._raw(key, default)
        if v is None:
            return None
        if isinstance(v, str):
            v = v.strip()
            return int(float(v)) if ("." in v or "e" in v.lower()) else int(v)
        return int(v)

    def get_float(self, key: str, default: Any = _MISSING) -> float | None:
        v = self._raw(key, default)
        return None if v is None else float(v)

    def get_bool(self, key: str, default: Any = _MISSING) -> bool | None:
        v = self._raw(key, default)
        if v is None or isinstance(v, bool):
            return v
        return str(v).strip().lower() in ("true", "1", "yes", "on")

    def get_list(self, key: str, default: Any = _MISSING, delim: str = ",", typ=str) -> list | None:
        v = self._raw(key, default)
        if v is None:
            return None
        if isinstance(v, (list, tuple)):
            return [typ(x) for x in v]
        s = str(v).strip()
        if not s:
            return []
        return [typ(x.strip()) for x in s.split(delim)]

    def get_int_list(self, key: str, default: Any = _MISSING, delim: str = ",") -> list[int] | None:
        return self.get_list(key, default, delim, int)

    def get_float_list(self, key: str, default: Any = _MISSING, delim: str = ",") -> list[float] | None:
        return self.get_list(key, default, delim, float)

    # reference-wide conventions
    @property
    def field_delim_in(self) -> str:
        d = self.get_str("field.delim.regex", None) or self.get_str("field.delim.in", None) or ","
        return _regex_to_delim(d)

    @property
    def field_delim_out(self) -> str:
        return self.get_str("field.delim.out", ",") or ","

    @property
    def debug(self) -> bool:
        return bool(self.get_bool("debug.on", False))

    def dump(self) -> str:
        return "\n".join(f"{k}={self.values[k]}" for k in sorted(self.values))

    def __contains__(self, key: str) -> bool:
        return self.has(key)

    def __repr__(self) -> str:
        return f"JobConfig(prefix={self.prefix!r}, {len(self.values)} keys)"


def _regex_to_delim(d: str) -> str:
    """The reference passes a *regex* for splitting; map the common ones to a literal char."""
    table = {"\\s+": " ", "\\t": "\t", "\\|": "|", "\\.": "."}
    if d in table:
        return table[d]
    return d.replace("\\", "") or ","


def _flatten(d: dict[str, Any], prefix: str = "") -> dict[str, Any]:
    """Flatten nested HOCON objects into dotted keys while also keeping the nested dicts (so
    ``cfg.get('thompsonSampler')`` returns the sub-block)."""
    out: dict[str, Any] = {}
    for k, v in d.items():
        key = f"{prefix}{k}"
        out[key] = v
        if isinstance(v, dict):
            out.update(_flatten(v, key + "."))
    return out


# --------------------------------------------------------------------------------------------
# Python-side Configuration (jprops semantics)
# --------------------------------------------------------------------------------------------
class Configuration:
    """Defaults-table configuration with the reference Python semantics
    (``python/lib/mlutil.py:34-231``): every getter returns ``(value, is_default)``; a value of
    ``_`` selects the default, ``none`` yields None; a default whose second element is a message
    means the key is mandatory."""

    def __init__(self, config: str | Path | dict[str, str] | None, defaults: dict[str, tuple],
                 verbose: bool = False):
        if config is None:
            configs: dict[str, str] = {}
        elif isinstance(config, dict):
            configs = {k: str(v) for k, v in config.items()}
        else:
            configs = read_properties(config)
        # keys only present in the defaults table behave as "_"
        for k in defaults:
            configs.setdefault(k, "_")
        self.configs = configs
        self.defaults = defaults
        self.verbose = verbose

    def override(self, config: str | Path | dict[str, str]) -> None:
        upd = read_properties(config) if not isinstance(config, dict) else config
        self.configs.update({k: str(v) for k, v in upd.items()})

    def set_param(self, name: str, value: Any) -> None:
        self.configs[name] = str(value)

    setParam = set_param

    def is_none(self, name: str) -> bool:
        return self.configs.get(name, "_").strip().lower() == "none"

    def is_default(self, name: str) -> bool:
        return self.configs.get(name, "_").strip() == "_"

    def _default(self, name: str):
        if name not in self.defaults:
            raise KeyError(f"no value and no default for {name}")
        val, err = self.defaults[name]
        if err is not None:
            raise ValueError(err)
        return val

    def _get(self, name: str, conv):
        if self.is_none(name):
            return None, False
        if self.is_default(name):
            return self._default(name), True
        return conv(self.configs[name].strip()), False

    def get_string(self, name: str):
        return self._get(name, str)

    def get_int(self, name: str):
        return self._get(name, lambda s: int(float(s)))

    def get_float(self, name: str):
        return self._get(name, float)

    def get_boolean(self, name: str):
        return self._get(name, lambda s: s.lower() == "true")

    def get_int_list(self, name: str, delim: str = ","):
        return self._get(name, lambda s: [int(x) for x in s.split(delim)])

    def get_float_list(self, name: str, delim: str = ","):
        return self._get(name, lambda s: [float(x) for x in s.split(delim)])

    def get_string_list(self, name: str, delim: str = ","):
        return self._get(name, lambda s: s.split(delim))

    # reference-compatible camelCase aliases
    getStringConfig = get_string
    getIntConfig = get_int
    getFloatConfig = get_float
    getBooleanConfig = get_boolean
    getIntListConfig = get_int_list
    getFloatListConfig = get_float_list
    getStringListConfig = get_string_list

    def either_or(self, first: str, second: str, getter: str = "get_string"):
        g = getattr(self, getter)
        fn, sn = self.is_none(first), self.is_none(second)
        if not fn and not sn:
            raise ValueError(f"only one of {first} and {second} should be set")
        if fn and sn:
            raise ValueError(f"at least one of {first} and {second} should be set")
        return (g(first)[0], None) if not fn else (None, g(second)[0])

    def items(self) -> Iterable[tuple[str, str]]:
        return self.configs.items()
