"""Helpers to run multi-rank (gloo, CPU) tests in-process via torch.multiprocessing."""
from __future__ import annotations

import os
import pickle
import socket
import traceback

import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make_comm(kind: str):
    """``gloo:cpu`` (default), ``gloo:cuda`` (device tensors over a gloo group: ranks share the
    GPU), ``rccl-emul:cpu`` / ``rccl-emul:cuda`` (Comm.emulated_rccl: the RCCL-only code paths
    over a gloo group)."""
    from avenir_amd.parallel import comm as C
    be, dev = (kind.split(":") + ["cpu"])[:2]
    c = C.Comm.emulated_rccl(device=dev) if be == "rccl-emul" else C.Comm(backend="gloo", device=dev)
    if dev == "cuda":   # every rank on the one visible GPU
        import torch
        torch.cuda.set_device(0)
        c.device = torch.device("cuda", 0)
    C.set_comm(c)
    return c


def _worker(rank, world, port, fn, args, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    try:
        from avenir_amd.parallel import comm as C
        C.set_comm(None)
        c = _make_comm(os.environ.get("AVMI_TEST_COMM", "gloo:cpu"))
        res = fn(rank, world, *args)
        # pickled by value here: the queue's default tensor pickler shares storage by fd, which
        # breaks when this rank exits before the parent has received it (connection reset)
        q.put((rank, "ok", pickle.dumps(res)))
        c.barrier()
        c.shutdown()
    except Exception:  # noqa: BLE001
        q.put((rank, "err", traceback.format_exc()))


def run_world(fn, world: int, *args, timeout: float = 120.0, comm: str = "gloo:cpu"):
    """Run ``fn(rank, world, *args)`` on ``world`` ranks (``comm``: see _make_comm); return the
    results ordered by rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker_env, args=(r, world, port, fn, args, q, {"AVMI_TEST_COMM": comm}))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, status, res = q.get(timeout=timeout)
            if status != "ok":
                raise AssertionError(f"rank {rank} failed:\n{res}")
            out[rank] = pickle.loads(res)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return [out[r] for r in range(world)]


def _worker_env(rank, world, port, fn, args, q, env):
    os.environ.update(env or {})
    _worker(rank, world, port, fn, args, q)


def run_world_outcome(fn, world: int, *args, env: dict | None = None, timeout: float = 120.0):
    """Like ``run_world`` but tolerant of failing ranks (fault-injection tests): returns
    ``(results_by_rank, errors_by_rank, exitcodes)``; every rank process is fresh (spawn)."""
    import queue as _queue
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker_env, args=(r, world, port, fn, args, q, env)) for r in range(world)]
    for p in procs:
        p.start()
    res, errs = {}, {}
    import time as _t
    deadline = _t.monotonic() + timeout
    while len(res) + len(errs) < world and _t.monotonic() < deadline:
        try:
            rank, status, payload = q.get(timeout=1.0)
        except _queue.Empty:
            if all(not p.is_alive() for p in procs) and q.empty():
                break
            continue
        (res if status == "ok" else errs)[rank] = pickle.loads(payload) if status == "ok" else payload
    for p in procs:
        p.join(timeout=10)
        if p.is_alive():
            p.kill()
            p.join(timeout=10)
    return res, errs, [p.exitcode for p in procs]
