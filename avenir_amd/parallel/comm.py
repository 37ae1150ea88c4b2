"""Collective communication layer (N4): RCCL over xGMI via ``torch.distributed``.

Every shuffle / broadcast / collect of the reference maps onto one of these ops (SURVEY.md
§2.24, §2.26):

* Hadoop combiner + reducer sum, Spark ``reduceByKey`` on dense keys  -> ``all_reduce`` (sum)
* HDFS side files read in every mapper's ``setup()``, Spark ``broadcast`` -> ``broadcast``
* Spark ``collect``/``collectAsMap``, cascade-SVM support vectors     -> ``all_gather_v``
* key-partitioned shuffles (joins, group-by-entity)                   -> ``all_to_all_v``
* bucket-pair replication for all-pairs similarity                    -> ``ring_pass``

One process per GPU; backend ``nccl`` (== RCCL on ROCm) for GPU tensors, ``gloo`` on CPU (tests,
CI).  With world size 1 every op is a no-op, so single-GPU code paths are the same code.

Design notes for xGMI (7 point-to-point links per MI355X): the payloads here are small dense count
tensors (KB..tens of MB), so ops are issued ONCE per model/iteration on coalesced flat buffers
(``all_reduce_coalesced``) rather than per key; RCCL picks its one-shot/tree algorithms for small
messages and multi-ring for large ones.

Deterministic small-message all-reduce, two variants, both bit-identical on every rank and run:

* ``algo="p2p"``: the hand-written peer-mapped kernels of ``csrc/kernels/comm.hip``
  (``parallel/p2p.py``).  Each rank stages its operand in an IPC-exported buffer; ONE kernel per
  rank waits on per-block epoch flags raised by its peers and sums every peer's staging in rank
  order (one-shot up to 256 KiB, reduce-scatter + all-gather through result stagings above, up to
  the 8 MiB staging capacity; larger messages take the library collective).  No ring steps, no
  proxy thread.  Device sums of float32 / float64 / int32 / int64 only; other cases fall back to
  the library collective.  Tested with 2 and 4 processes sharing one GPU
  (tests/test_p2p_allreduce.py) — the multi-process path through the same code a multi-GPU node
  takes over xGMI.
* ``algo="oneshot"``: an all-gather of every rank's buffer (RCCL's collective) followed by a local
  sum in rank order; any reduction op, any device.

Selection of sum reductions up to ``AVMI_ONESHOT_MAX_BYTES`` (default 64 KiB) when the caller names
no algorithm: ``AVMI_SMALL_ALLREDUCE`` = ``auto`` (default) | ``p2p`` | ``oneshot`` | ``rccl``.
``auto``: at the first such all-reduce of a device tensor on a multi-rank communicator, every rank
runs the same probe (:meth:`Comm._auto_small_allreduce`): build the peer-mapped state (agreed over
ranks; unavailable -> the library collective), check it exact on integer sums, time it against
the library collective at the message's size, and take it only if every rank found it exact and
it is faster (max over ranks).  The choice is cached per communicator.

Failure reporting of the p2p path is loud (``parallel/p2p.py``): a checked call raises
``P2PError`` on the rank whose wait failed and on the late peer; unchecked calls (the NB
side-stream overlap) are checked at the next collective of this communicator (non-blocking) and
by :meth:`Comm.check` — which every job output method calls before writing
(``jobs/common.py``) — so no job writes output computed from a failed sum.
"""
from __future__ import annotations

import datetime as _dt
import os
import time
from contextlib import contextmanager
from typing import Any, Sequence

import torch
import torch.distributed as dist

from ..utils import logging as alog
from ..utils.tracing import traced

_COMM: "Comm | None" = None
_SMALL_ENV = os.environ.get("AVMI_SMALL_ALLREDUCE", "auto").strip().lower() or "auto"
if _SMALL_ENV not in ("auto", "p2p", "oneshot", "rccl"):
    raise ValueError(f"AVMI_SMALL_ALLREDUCE={_SMALL_ENV!r}: expected auto, p2p, oneshot or rccl")
_ONESHOT_MAX_BYTES = int(os.environ.get("AVMI_ONESHOT_MAX_BYTES", str(64 << 10)))
_PROBE_TIMEOUT_S = float(os.environ.get("AVMI_P2P_PROBE_TIMEOUT_S", "10"))


class CollectiveTimeout(RuntimeError):
    pass


class Comm:
    def __init__(self, backend: str | None = None, timeout_s: float | None = None,
                 device: str | None = None, port: int | None = None):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", str(self.rank)))
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        if device == "cuda":
            n = torch.cuda.device_count()
            torch.cuda.set_device(self.local_rank % max(1, n))
            self.device = torch.device("cuda", torch.cuda.current_device())
        else:
            self.device = torch.device("cpu")
        self.timeout_s = float(timeout_s or os.environ.get("AVENIR_COMM_TIMEOUT", "600"))
        self.backend = backend or ("nccl" if self.device.type == "cuda" else "gloo")
        # the process group's real backend; ``backend`` picks the algorithmic path (equal except in
        # the RCCL emulation of tests: see emulated_rccl)
        self.pg_backend = self.backend
        self._owns_pg = False
        if self.world > 1 and not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            # torchrun exports MASTER_PORT; AVENIR_MASTER_PORT (or Comm(port=...)) overrides the
            # fallback used when a job starts its own ranks
            os.environ.setdefault("MASTER_PORT", str(port or os.environ.get("AVENIR_MASTER_PORT", "29533")))
            kw = {}
            if self.backend == "nccl":
                kw["device_id"] = self.device
            dist.init_process_group(self.backend, rank=self.rank, world_size=self.world,
                                    timeout=_dt.timedelta(seconds=self.timeout_s), **kw)
            self._owns_pg = True
        if dist.is_initialized():
            self.world = dist.get_world_size()
            self.rank = dist.get_rank()
            self.pg_backend = dist.get_backend()
        self.stats = {"calls": 0, "bytes": 0, "seconds": 0.0}
        # parallel/p2p.P2PAllReduce, created by the first p2p all-reduce; False once its agreed
        # construction failed (no peer mapping on this node): the library collective from then on
        self._p2p = None
        self._p2p_unchecked = False     # an unchecked p2p call may not have been checked yet
        # algorithm of sum all-reduces up to _ONESHOT_MAX_BYTES when the caller names none:
        # None (library collective), "oneshot", "p2p", or "auto" (probe at the first one: see
        # _auto_small_allreduce); env AVMI_SMALL_ALLREDUCE, or set by a tuner such as bench.py's
        self.small_allreduce = {"rccl": None}.get(_SMALL_ENV, _SMALL_ENV)
        self.small_allreduce_probe: dict | None = None

    @classmethod
    def emulated_rccl(cls, device: str | None = None, **kw) -> "Comm":
        """A communicator that takes every RCCL-only code path (``backend == "nccl"``: side-stream
        overlap of the NB all-reduce, device-resident collective buffers) while its process group
        is gloo — so those paths run in multi-process tests on a CPU host or on ONE GPU shared by
        several ranks.  Tensors cross the gloo group through host copies (``_prep``)."""
        c = cls(backend="gloo", device=device, **kw)
        c.backend = "nccl"
        return c

    # ------------------------------------------------------------------------------------------
    @property
    def is_distributed(self) -> bool:
        return self.world > 1

    @property
    def is_root(self) -> bool:
        return self.rank == 0

    def _account(self, t: torch.Tensor, t0: float) -> None:
        self.stats["calls"] += 1
        self.stats["bytes"] += t.numel() * t.element_size()
        self.stats["seconds"] += time.perf_counter() - t0

    def _prep(self, t: torch.Tensor) -> tuple[torch.Tensor, bool]:
        """gloo only handles CPU tensors, RCCL only GPU tensors: move if needed (a host tensor
        handed to an RCCL group — a job's small host-side counters — goes through the device)."""
        if self.pg_backend == "gloo" and t.is_cuda:
            return t.cpu(), True
        if self.pg_backend == "nccl" and not t.is_cuda and self.device.type == "cuda":
            return t.to(self.device), True
        return t, False

    # ------------------------------------------------------------------------------------------
    @traced("comm.all_reduce", nbytes=lambda self, t, *a, **k: t.numel() * t.element_size(), device=lambda self, t, *a, **k: t.device)
    def all_reduce(self, t: torch.Tensor, op: str = "sum", algo: str | None = None,
                   checked: bool = True) -> torch.Tensor:
        """In-place all-reduce (sum|max|min|prod); returns ``t``.  ``algo``: None (library
        collective, or the selected small-message path), "ring" (library), "oneshot" (all-gather +
        rank-ordered local reduction), "p2p" (hand-written peer-mapped kernel, sums of device
        tensors; anything else falls back to the library collective).  ``checked=False`` lets a
        p2p sum stay asynchronous (see the module docstring)."""
        if not self.is_distributed:
            return t
        self._guard()
        small = t.numel() * t.element_size() <= _ONESHOT_MAX_BYTES
        if algo is None and op == "sum" and small and self.small_allreduce:
            if self.small_allreduce == "auto":
                if self._auto_eligible(t):
                    self._auto_small_allreduce(t)
                    algo = self.small_allreduce
            else:
                algo = self.small_allreduce
        if algo == "p2p":
            if op == "sum" and self._all_reduce_p2p(t, checked) is not None:
                return t
            algo = None                       # not a device sum the kernel takes: the library collective
        if algo == "oneshot":
            return self._all_reduce_oneshot(t, op)
        t0 = time.perf_counter()
        x, moved = self._prep(t)
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN,
               "prod": dist.ReduceOp.PRODUCT}[op]
        dist.all_reduce(x, op=rop)
        if moved:
            t.copy_(x)
        self._account(t, t0)
        return t

    # ---- peer-mapped path: construction, selection, failure gate ------------------------------
    def p2p(self):
        """The peer-mapped all-reduce state (``parallel/p2p.py``), created on first use — a
        collective: every rank reaches its first p2p all-reduce together.  None when it is
        unavailable on this node (the agreed construction failed on some rank: every rank gets None
        together, and remembers it, so later calls take the library collective at once)."""
        if self._p2p is None:
            from .p2p import P2PAllReduce, P2PError
            try:
                self._p2p = P2PAllReduce(self, self.device)
            except P2PError as e:
                alog.get_logger("comm").warning("peer-mapped all-reduce unavailable: %s", e)
                self._p2p = False
                if self.small_allreduce in ("p2p", "auto"):
                    self.small_allreduce = None
        return self._p2p or None

    def _auto_eligible(self, t: torch.Tensor) -> bool:
        from .p2p import P2PAllReduce
        return self.device.type == "cuda" and P2PAllReduce.supports(t) and t.device == self.device

    def _auto_small_allreduce(self, like: torch.Tensor) -> str | None:
        """Collective, once per communicator: pick the small-sum algorithm (module docstring).
        Every rank reaches it at the same all-reduce (same size, same dtype class by the collective
        contract) and takes the same branch: construction and the verdict are both agreed."""
        info: dict = {"bytes": like.numel() * like.element_size()}
        choice = None
        p = self.p2p()
        if p is None:
            info["p2p"] = "unavailable"
        else:
            exact, t_p2p, t_lib = self._probe_p2p(p, like)
            info.update(exact_here=exact, p2p_us_here=t_p2p * 1e6, lib_us_here=t_lib * 1e6)
            use, t_p2p, t_lib = self._agree_small_choice(exact, t_p2p, t_lib)
            info.update(p2p_us=t_p2p * 1e6, lib_us=t_lib * 1e6)
            choice = "p2p" if use else None
        info["chosen"] = choice or "library"
        self.small_allreduce = choice
        self.small_allreduce_probe = info
        alog.get_logger("comm").info("small all-reduce selection: %s", info)
        return choice

    def _probe_p2p(self, p, like: torch.Tensor, rounds: int = 8, iters: int = 30) -> tuple[bool, float, float]:
        """This rank's measurements: the kernel exact on integer sums of ``like``'s size, then the
        mean time of the kernel and of the library collective at that size.

        The exactness rounds start behind a barrier and run under a short wait bound
        (``AVMI_P2P_PROBE_TIMEOUT_S``, 10 s): a node whose peer mapping does not deliver (flags
        never seen across devices, a peer gone) fails HERE, in seconds, instead of at the job's
        first real sum after the full wait bound.  A P2PError in these rounds is caught; exactness
        is then agreed over the ranks (one library all-reduce) BEFORE the timing rounds, so every
        rank runs the same collectives, and an inexact verdict anywhere retires the kernel on every
        rank (closed together; later small sums take the library collective)."""
        from .p2p import P2PError
        W = self.world
        n = max(1, like.numel())
        xi = torch.empty(n, dtype=torch.int64, device=like.device)
        exact = True
        old = p.timeout_s
        self.barrier()
        try:
            p.set_timeout(min(old, _PROBE_TIMEOUT_S))
            for i in range(rounds):
                xi.fill_(self.rank + 1 + i)
                p.all_reduce(xi)
                exact &= bool((xi == W * (W + 1) // 2 + W * i).all().item())
        except P2PError as e:
            alog.get_logger("comm").warning("peer-mapped all-reduce failed its probe: %s", e)
            exact = False
        dev = self.device if self.pg_backend == "nccl" else "cpu"
        f = torch.tensor([0.0 if exact else 1.0], dtype=torch.float64, device=dev)
        self.all_reduce(f, "max", algo="ring")
        if float(f.item()) != 0.0:
            try:
                p.close()                     # collective: every rank reaches it (agreed verdict)
            finally:
                self._p2p = False
            return False, float("inf"), 0.0
        p.set_timeout(old)
        x = torch.ones_like(like).contiguous()

        def timed(fn) -> float:
            for _ in range(3):
                fn()
            torch.cuda.synchronize(like.device)
            self.barrier()
            t0 = time.perf_counter()
            for _ in range(iters):
                fn()
            torch.cuda.synchronize(like.device)
            return (time.perf_counter() - t0) / iters

        t_lib = timed(lambda: self.all_reduce(x, algo="ring"))
        t_p2p = timed(lambda: p.all_reduce(x, checked=False))
        p.check(block=True)
        return exact, t_p2p, t_lib

    def _agree_small_choice(self, exact: bool, t_p2p: float, t_lib: float) -> tuple[bool, float, float]:
        """One max all-reduce of (not exact, p2p time, library time) over the ranks: the kernel is
        chosen only if it was exact on EVERY rank and faster by the slowest rank's clock."""
        dev = self.device if self.pg_backend == "nccl" else "cpu"
        f = torch.tensor([0.0 if exact else 1.0, float(t_p2p), float(t_lib)], dtype=torch.float64, device=dev)
        self.all_reduce(f, "max", algo="ring")
        bad, tp, tl = f.tolist()
        return (bad == 0.0 and tp < tl), tp, tl

    def _all_reduce_p2p(self, t: torch.Tensor, checked: bool = True) -> torch.Tensor | None:
        """The hand-written peer-mapped sum (comm.hip); None when ``t`` does not qualify (host
        tensor, unsupported dtype, larger than the staging capacity, peer mapping unavailable) —
        the caller then takes the library collective.  The decision depends only on shape / dtype /
        device type and agreed state, which every rank shares, so all ranks take the same path."""
        from .p2p import P2PAllReduce
        if not P2PAllReduce.supports(t) or self.device.type != "cuda":
            return None
        p = self.p2p()
        if p is None or t.numel() * t.element_size() > p.cap_bytes:
            return None
        t0 = time.perf_counter()
        _maybe_delay_p2p(self.rank)
        p.all_reduce(t, checked=checked)
        if not checked:
            self._p2p_unchecked = True
        self._account(t, t0)
        return t

    @property
    def p2p_calls(self) -> int:
        """Number of peer-mapped all-reduce kernels this communicator launched."""
        return sum(self._p2p.calls.values()) if self._p2p else 0

    def _guard(self) -> None:
        """Entry of every collective: raise P2PError if an unchecked p2p call of this rank has
        failed (non-blocking: only kernels that already finished are seen)."""
        if self._p2p_unchecked and self._p2p:
            self._p2p.check(block=False)

    def check(self, block: bool = True) -> None:
        """Raise P2PError if any p2p all-reduce of this rank failed.  ``block`` waits for the last
        one first.  Local (no collective): the job output methods call it before writing, so a
        rank never writes output computed from a failed sum; the peers of a failed rank fail on
        their own (poisoned flags) or at their next collective."""
        if self._p2p:
            self._p2p.check(block=block)
            if block:
                self._p2p_unchecked = False

    def _all_reduce_oneshot(self, t: torch.Tensor, op: str) -> torch.Tensor:
        """One all-gather of every rank's buffer, then the reduction over ranks in rank order."""
        t0 = time.perf_counter()
        g = self.all_gather(t.contiguous())                       # [world, *t.shape]
        if op == "sum":
            r = g[0].clone()
            for k in range(1, self.world):
                r += g[k]
        elif op == "max":
            r = g.amax(0)
        elif op == "min":
            r = g.amin(0)
        elif op == "prod":
            r = g[0].clone()
            for k in range(1, self.world):
                r *= g[k]
        else:
            raise ValueError(op)
        t.copy_(r)
        self._account(t, t0)
        return t

    def all_reduce_coalesced(self, tensors: Sequence[torch.Tensor], op: str = "sum") -> None:
        """All-reduce several tensors of one dtype with a single collective (flat buffer)."""
        if not self.is_distributed or not tensors:
            return
        by_dtype: dict[torch.dtype, list[torch.Tensor]] = {}
        for t in tensors:
            by_dtype.setdefault(t.dtype, []).append(t)
        for ts in by_dtype.values():
            flat = torch.cat([t.reshape(-1) for t in ts])
            self.all_reduce(flat, op)
            o = 0
            for t in ts:
                k = t.numel()
                t.copy_(flat[o:o + k].view_as(t))
                o += k

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if not self.is_distributed:
            return t
        self._guard()
        t0 = time.perf_counter()
        x, moved = self._prep(t)
        dist.broadcast(x, src)
        if moved:
            t.copy_(x)
        self._account(t, t0)
        return t

    def broadcast_object(self, obj: Any, src: int = 0) -> Any:
        if not self.is_distributed:
            return obj
        self._guard()
        box = [obj]
        dist.broadcast_object_list(box, src)
        return box[0]

    def all_gather_object(self, obj: Any) -> list[Any]:
        if not self.is_distributed:
            return [obj]
        self._guard()
        out: list[Any] = [None] * self.world
        dist.all_gather_object(out, obj)
        return out

    @traced("comm.all_gather", nbytes=lambda self, t, *a, **k: t.numel() * t.element_size() * self.world, device=lambda self, t, *a, **k: t.device)
    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """Equal-shape all-gather -> [world, *t.shape]."""
        if not self.is_distributed:
            return t.unsqueeze(0)
        self._guard()
        x, moved = self._prep(t.contiguous())
        flat = torch.empty((self.world * x.numel(),), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(flat, x.reshape(-1))
        out = flat.view((self.world,) + tuple(x.shape))
        return out.to(t.device) if moved else out

    def all_gather_v(self, t: torch.Tensor) -> torch.Tensor:
        """Variable-length all-gather along dim 0 (RCCL has no AllGatherV: exchange counts,
        pad to the max, all-gather, strip)."""
        if not self.is_distributed:
            return t
        n = torch.tensor([t.shape[0]], dtype=torch.long, device=t.device)
        counts = self.all_gather(n).view(-1).tolist()
        m = max(counts)
        pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[: t.shape[0]] = t
        g = self.all_gather(pad)
        return torch.cat([g[r, : counts[r]] for r in range(self.world)], dim=0)

    def all_to_all_v(self, chunks: list[torch.Tensor]) -> list[torch.Tensor]:
        """Send ``chunks[r]`` to rank r; receive one tensor from every rank (dim-0 variable): one
        all-to-all of the row counts, one ``all_to_all_single`` of the payload (RCCL over xGMI on
        GPUs; gloo runs the same call on host copies)."""
        if not self.is_distributed:
            return [chunks[0]]
        dev = chunks[0].device
        tail = tuple(chunks[0].shape[1:])
        send, moved = self._prep(torch.cat(chunks, dim=0).contiguous())
        sizes = torch.tensor([c.shape[0] for c in chunks], dtype=torch.long, device=send.device)
        recv_sizes = torch.empty_like(sizes)
        t0 = time.perf_counter()
        dist.all_to_all_single(recv_sizes, sizes)
        rs = recv_sizes.tolist()
        recv = torch.empty((int(sum(rs)),) + tail, dtype=send.dtype, device=send.device)
        dist.all_to_all_single(recv, send, rs, sizes.tolist())
        self._account(recv, t0)
        if moved:
            recv = recv.to(dev)
        return list(torch.split(recv, rs))

    def fetch_rows(self, gids: torch.Tensor, tables: list[torch.Tensor], base: int, sizes: list[int]) -> list[torch.Tensor]:
        """Rows ``gids`` (global row ids; -1 = none -> zeros) of row-sharded ``tables`` (this rank holds
        global rows [base, base + len)), ``sizes`` = every rank's row count.  Two all-to-alls (the
        requests, then the rows) instead of an all-gather of every table: O(requested rows)."""
        dev = gids.device
        g = gids.long().view(-1)
        if not self.is_distributed:
            li = (g - base).clamp(0, max(0, tables[0].shape[0] - 1)) if tables and tables[0].shape[0] else g.clamp_min(0)
            out = []
            for t in tables:
                v = t[li] if t.shape[0] else torch.zeros((g.numel(),) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
                out.append(torch.where((g >= 0).view((-1,) + (1,) * (t.dim() - 1)), v, torch.zeros_like(v)))
            return out
        starts = torch.tensor([sum(sizes[:r]) for r in range(self.world)], dtype=torch.long, device=dev)
        owner = (torch.searchsorted(starts, g.clamp_min(0), right=True) - 1).clamp_min(0)
        owner = torch.where(g >= 0, owner, torch.full_like(owner, self.rank))
        order = torch.argsort(owner, stable=True)
        counts = torch.bincount(owner, minlength=self.world).tolist()
        req = self.all_to_all_v(list(torch.split(g[order], counts)))          # ids others want from me
        want = torch.cat(req) if req else torch.zeros(0, dtype=torch.long, device=dev)
        li = (want - base).clamp(0, max(0, tables[0].shape[0] - 1))
        back_counts = [r.shape[0] for r in req]
        out = []
        for t in tables:
            v = t[li] if t.shape[0] else torch.zeros((want.numel(),) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
            v = torch.where((want >= 0).view((-1,) + (1,) * (t.dim() - 1)), v, torch.zeros_like(v))
            got = torch.cat(self.all_to_all_v(list(torch.split(v, back_counts))))  # in my request order
            res = torch.empty_like(got)
            res[order] = got
            out.append(res)
        return out

    def ring_pass(self, t: torch.Tensor) -> torch.Tensor:
        """Send ``t`` to rank+1 and receive from rank-1 (systolic all-pairs schedule).  Shapes may
        differ between ranks: the dim-0 length travels first.  Both exchanges are batched P2P groups
        (at world 2 the send and the receive share one peer, and a lone RCCL send of a large
        buffer would wait for a receive queued behind it)."""
        if not self.is_distributed:
            return t
        n_out = torch.tensor([t.shape[0]], dtype=torch.long, device=t.device)
        n_in = self.ring_pass_finish(self.ring_pass_start(n_out, 1))
        return self.ring_pass_finish(self.ring_pass_start(t, int(n_in.item())))

    def ring_pass_start(self, t: torch.Tensor, recv_rows: int):
        """Post the send of ``t`` to rank+1 and the receive of ``recv_rows`` rows (same trailing
        shape / dtype) from rank-1; returns a handle for :meth:`ring_pass_finish`.  Issued as one
        batched P2P group (``batch_isend_irecv``: no send/recv ordering deadlock on RCCL) so the
        caller can compute while the transfer is in flight."""
        nxt, prv = (self.rank + 1) % self.world, (self.rank - 1) % self.world
        x, moved = self._prep(t.contiguous())
        recv = torch.empty((int(recv_rows),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        ops = [dist.P2POp(dist.isend, x, nxt), dist.P2POp(dist.irecv, recv, prv)]
        reqs = dist.batch_isend_irecv(ops)
        return reqs, recv, x, (t.device if moved else None)

    def ring_pass_finish(self, handle) -> torch.Tensor:
        reqs, recv, _keepalive, dev = handle
        for r in reqs:
            r.wait()
        return recv.to(dev) if dev is not None else recv

    def ring_iter(self, tensors: list[torch.Tensor]):
        """Systolic ring over every rank's block: yields ``(owner, block)`` W times, starting with
        this rank's own ``tensors`` (a list sharing dim 0 per tensor, any dtypes), then the blocks of
        rank-1, rank-2, ... .  The block sizes are exchanged once up front; the transfer of the
        next block (``ring_pass_start``, one batched P2P group per tensor) is posted BEFORE the
        current block is yielded, so the caller's compute on it overlaps the xGMI transfer.  With
        world size 1: the own block once."""
        if not self.is_distributed:
            yield self.rank, tensors
            return
        W, me = self.world, self.rank
        n = torch.tensor([t.shape[0] for t in tensors], dtype=torch.long,
                         device=self.device if self.pg_backend == "nccl" else "cpu")
        sizes = self.all_gather(n).view(W, -1).tolist()
        cur = [t.contiguous() for t in tensors]
        for step in range(W):
            owner = (me - step) % W
            pend = None
            if step + 1 < W:
                src = (me - step - 1) % W
                pend = [self.ring_pass_start(t, sizes[src][k]) for k, t in enumerate(cur)]
            yield owner, cur
            if pend is not None:
                cur = [self.ring_pass_finish(h) for h in pend]

    def barrier(self) -> None:
        if self.is_distributed:
            self._guard()
            if self.pg_backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def reduce_max_scalar(self, v: float) -> float:
        if not self.is_distributed:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=self.device if self.pg_backend == "nccl" else "cpu")
        self.all_reduce(t, "max")
        return float(t.item())

    def shutdown(self) -> None:
        if self._p2p:
            self.check()                      # a failed sum surfaces before a clean exit
            self._p2p.close()
        self._p2p = None
        if self._owns_pg and dist.is_initialized():
            dist.destroy_process_group()
            self._owns_pg = False


def get_comm(**kw) -> Comm:
    """The process's communicator.  ``AVENIR_COMM_BACKEND`` = gloo / nccl / rccl-emul overrides the
    default backend (rccl-emul: the RCCL code paths over a gloo group, so several ranks can share
    one GPU in a rehearsal of a multi-GPU run)."""
    global _COMM
    if _COMM is None:
        be = os.environ.get("AVENIR_COMM_BACKEND", "")
        if be == "rccl-emul" and "backend" not in kw:
            _COMM = Comm.emulated_rccl(**kw)
        else:
            if be in ("gloo", "nccl"):
                kw.setdefault("backend", be)
            _COMM = Comm(**kw)
    return _COMM


def set_comm(c: Comm | None) -> None:
    global _COMM
    _COMM = c


@contextmanager
def timed_collective(name: str, warn_s: float = 30.0):
    """Watchdog-style timing of a collective phase: logs a warning when a phase is slow (a hung
    peer shows up here long before RCCL's own timeout fires)."""
    t0 = time.perf_counter()
    yield
    dt = time.perf_counter() - t0
    if dt > warn_s:
        alog.get_logger("comm").warning("collective %s took %.1fs", name, dt)


def _maybe_delay_p2p(rank: int) -> None:
    """Fault injection for the peer-mapped path (tests): ``AVMI_FAULT_P2P_SLEEP_RANK`` sleeps
    ``AVMI_FAULT_P2P_SLEEP_S`` seconds before each of its p2p launches — a rank late past the
    peers' wait bound, as a slow shard read would make it."""
    r = os.environ.get("AVMI_FAULT_P2P_SLEEP_RANK")
    if r is not None and int(r) == rank:
        time.sleep(float(os.environ.get("AVMI_FAULT_P2P_SLEEP_S", "0")))


def maybe_inject_fault(iteration: int, rank: int | None = None) -> None:
    """Env-driven fault injection for recovery tests: when
    ``AVMI_FAULT_RANK`` == this rank and ``AVMI_FAULT_ITER`` == iteration, raise."""
    fr = os.environ.get("AVMI_FAULT_RANK")
    fi = os.environ.get("AVMI_FAULT_ITER")
    if fr is None or fi is None:
        return
    r = rank if rank is not None else int(os.environ.get("RANK", "0"))
    if int(fr) == r and int(fi) == iteration:
        mode = os.environ.get("AVMI_FAULT_MODE", "raise")
        if mode == "exit":
            os._exit(17)
        raise RuntimeError(f"injected fault at rank {r} iteration {iteration}")


class Watchdog:
    """Failure detector for long collective phases: the training / iteration loop
    calls ``beat()``; if no beat arrives within ``timeout_s`` the watchdog logs the stall and
    (``abort=True``) terminates this rank with exit code 75 so ``torchrun --max-restarts`` can
    relaunch the job, which then resumes from its last iteration checkpoint.  RCCL's own async
    error handling (``TORCH_NCCL_ASYNC_ERROR_HANDLING=1``, set here if unset) aborts a hung
    communicator from inside the process group as a second line of defence."""

    def __init__(self, timeout_s: float = 300.0, abort: bool = True, on_stall=None):
        import threading
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        self.timeout_s, self.abort, self.on_stall = timeout_s, abort, on_stall
        self._last = time.monotonic()
        self._stop = threading.Event()
        self.stalled = False
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def beat(self) -> None:
        self._last = time.monotonic()

    def _run(self):
        while not self._stop.wait(min(1.0, self.timeout_s / 4)):
            if time.monotonic() - self._last > self.timeout_s:
                self.stalled = True
                alog.get_logger("comm").error("watchdog: no progress for %.0fs", self.timeout_s)
                if self.on_stall is not None:
                    self.on_stall()
                if self.abort:
                    os._exit(75)
                return

    def stop(self) -> None:
        self._stop.set()


def health_check(comm: "Comm | None" = None) -> bool:
    """One tiny all-reduce that every rank must answer: True when the world is healthy."""
    comm = comm or get_comm()
    if not comm.is_distributed:
        return True
    t = torch.ones(1, device=comm.device if comm.backend == "nccl" else "cpu")
    comm.all_reduce(t)
    return int(t.item()) == comm.world
