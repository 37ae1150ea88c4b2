"""Loader for the in-tree native extension ``avenir_amd/_C.so``.

Policy (fail loudly): GPU tensors ALWAYS go through the hand-written HIP kernels.  If the
extension is missing or failed to load, any GPU op raises instead of silently falling back to a
PyTorch implementation.  CPU tensors use small, readable PyTorch reference implementations (the
"golden oracles" of SURVEY.md §4.3) so the whole framework is testable on machines without a GPU.
"""
from __future__ import annotations

import importlib
import os
import threading

import torch  # noqa: F401  (must be imported first: _C links against torch's HIP runtime)

_lock = threading.Lock()
_mod = None
_err: BaseException | None = None


def _load():
    global _mod, _err
    with _lock:
        if _mod is not None or _err is not None:
            return
        try:
            _mod = importlib.import_module("avenir_amd._C")
        except BaseException as exc:  # noqa: BLE001
            if os.environ.get("AVENIR_AUTOBUILD", "1") == "1":
                try:
                    from . import _build
                    _build.build()
                    _mod = importlib.import_module("avenir_amd._C")
                    return
                except BaseException as exc2:  # noqa: BLE001
                    _err = exc2
                    return
            _err = exc


def available() -> bool:
    _load()
    return _mod is not None


def C():
    """Return the native module or raise (used by every GPU path)."""
    _load()
    if _mod is None:
        raise RuntimeError(
            "avenir_amd native extension (_C.so) is not available; build it with "
            "`python -m avenir_amd._build` (hipcc --offload-arch=gfx950). Original error: "
            f"{_err!r}")
    return _mod


def host():
    """Native host runtime (CSV parser, ring buffer, checkpoint I/O); None if not built."""
    _load()
    return _mod
