"""HIP-graph capture for the framework's replayed inner loops (GBT trees, SMO step blocks, training
steps).

``torch.cuda.graph(g)`` runs ``torch.cuda.synchronize()``, ``gc.collect()`` and
``torch.cuda.empty_cache()`` before every capture.  The last one hands every cached block of the
process back to the driver, so a model that captures a graph per fit (GBT) in a process that holds
gigabytes of cached tensors pays the hipFree of all of them and then fresh hipMallocs for
everything that follows: measured 0.031 s -> 0.122 s for a 64 k-row GBT fit and 19.8 -> 38 ms for
the next SVM fit when run after the 16.7 M-row benchmarks.  ``capturing`` is the same capture on a
side stream without the flush.
"""
from __future__ import annotations

import contextlib

import torch


@contextlib.contextmanager
def capturing(graph: "torch.cuda.CUDAGraph", stream: "torch.cuda.Stream | None" = None,
              device: "torch.device | int | str | None" = None):
    """Capture the work issued inside the block into ``graph`` (on ``stream`` or a new side stream
    ordered after the current one); the current stream waits for the side stream afterwards.
    ``device``: the device of the captured work (default: ``stream``'s, else the current device) —
    the side stream, the ordering and the capture all happen with that device current, so work on
    a device other than the current one is captured rather than launched outside the graph."""
    if device is None:
        device = stream.device if stream is not None else torch.cuda.current_device()
    with torch.cuda.device(device):
        s = stream if stream is not None else torch.cuda.Stream(device=device)
        cur = torch.cuda.current_stream(device)
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            graph.capture_begin()
            try:
                yield graph
            finally:
                graph.capture_end()
        cur.wait_stream(s)
