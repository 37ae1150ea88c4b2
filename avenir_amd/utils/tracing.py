"""Lightweight tracing: roctx ranges + device-event phase timers with bandwidth / FLOP rates.

The reference has no instrumentation.  ``trace("phase", bytes=..., flops=...)``
wraps a region: on the GPU it pushes a roctx range (``torch.cuda.nvtx`` maps to roctx on ROCm, so
rocprofv3 ``--marker-trace`` shows the phases) and records a pair of HIP events; on the CPU it uses
``perf_counter``.  Nothing is synchronised inside the region — ``report()`` resolves the events
once at the end — so tracing does not serialise the stream.  Enabled by ``AVENIR_TRACE=1`` or
``Tracer.enable()``; disabled tracing costs one attribute check.
"""
from __future__ import annotations

import contextlib
import json
import os
import time
from collections import defaultdict

import torch


class Tracer:
    def __init__(self):
        self.enabled = os.environ.get("AVENIR_TRACE", "0") == "1"
        self.records: list[tuple[str, object, object, float, float, bool]] = []

    def enable(self, on: bool = True):
        self.enabled = on
        return self

    def clear(self):
        self.records.clear()

    @contextlib.contextmanager
    def range(self, name: str, nbytes: float = 0.0, flops: float = 0.0, device=None):
        if not self.enabled:
            yield
            return
        cuda = torch.cuda.is_available() and (device is None or torch.device(device).type == "cuda")
        if cuda:
            torch.cuda.nvtx.range_push(name)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            try:
                yield
            finally:
                e.record()
                torch.cuda.nvtx.range_pop()
                self.records.append((name, s, e, nbytes, flops, True))
        else:
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self.records.append((name, t0, time.perf_counter(), nbytes, flops, False))

    def report(self) -> dict[str, dict]:
        """Per phase: calls, total ms, mean ms, GB/s, TFLOP/s (if bytes / flops were given)."""
        if any(r[5] for r in self.records):
            torch.cuda.synchronize()
        agg = defaultdict(lambda: {"calls": 0, "ms": 0.0, "bytes": 0.0, "flops": 0.0})
        for name, s, e, nb, fl, cuda in self.records:
            ms = s.elapsed_time(e) if cuda else (e - s) * 1e3
            a = agg[name]
            a["calls"] += 1
            a["ms"] += ms
            a["bytes"] += nb
            a["flops"] += fl
        out = {}
        for name, a in agg.items():
            sec = a["ms"] / 1e3
            r = {"calls": a["calls"], "total_ms": round(a["ms"], 4), "mean_ms": round(a["ms"] / a["calls"], 4)}
            if a["bytes"] and sec > 0:
                r["GB_per_s"] = float(f"{a['bytes'] / sec / 1e9:.4g}")
            if a["flops"] and sec > 0:
                r["TFLOP_per_s"] = float(f"{a['flops'] / sec / 1e12:.4g}")
            out[name] = r
        return out

    def dump(self, path=None) -> str:
        s = json.dumps(self.report(), indent=1)
        if path:
            with open(path, "w") as f:
                f.write(s)
        return s


TRACER = Tracer()


def trace(name: str, nbytes: float = 0.0, flops: float = 0.0, device=None):
    return TRACER.range(name, nbytes, flops, device)


def traced(name: str, nbytes=None, flops=None, device=None):
    """Decorator form: ``@traced("nb.fit", nbytes=lambda self, t, *a, **k: t.n * 6)``.  The byte /
    FLOP callables and ``device`` (a callable too) see the call's arguments; disabled tracing
    costs one attribute check per call."""
    import functools

    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*args, **kw):
            if not TRACER.enabled:
                return fn(*args, **kw)
            try:
                nb = float(nbytes(*args, **kw)) if nbytes else 0.0
                fl = float(flops(*args, **kw)) if flops else 0.0
                dv = device(*args, **kw) if device else None
            except Exception:
                nb, fl, dv = 0.0, 0.0, None
            with TRACER.range(name, nb, fl, dv):
                return fn(*args, **kw)
        return wrapper
    return deco


@contextlib.contextmanager
def torch_profile(path: str | None = None, cuda: bool | None = None):
    """torch.profiler wrapper for the NN paths; writes a Chrome trace when ``path`` is given."""
    acts = [torch.profiler.ProfilerActivity.CPU]
    if (cuda if cuda is not None else torch.cuda.is_available()):
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts, record_shapes=False) as prof:
        yield prof
    if path:
        prof.export_chrome_trace(path)
