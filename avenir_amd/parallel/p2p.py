"""Peer-mapped small-message all-reduce: the Python side of ``csrc/kernels/comm.hip``.

Every counting model of the reference ends a pass with a combiner + reducer shuffle of a KB-scale
count table (e.g. ``src/main/java/org/avenir/bayesian/BayesianDistribution.java:72-79``).  Here the
table is summed by ONE hand-written kernel per rank that reads the peers' staged copies directly:

* at construction every rank allocates its staging region (4 x ``cap_bytes``) and an uncached
  flag array, exports both with ``hipIpcGetMemHandle``, exchanges the handles ONCE through the
  process group (``all_gather_object``: gloo or RCCL) and maps every peer's regions with
  ``hipIpcOpenMemHandle`` — over xGMI between GPUs of one node, or through the same HBM when several
  ranks share one device (the multi-process rehearsal available on single-GPU boxes);
* each call bumps an epoch that every rank counts identically (collectives are called in the same
  order everywhere) and launches the one-shot kernel (messages up to ``oneshot_max`` bytes: every
  rank reads all W stagings) or the two-shot kernel (reduce-scatter + all-gather through the
  result stagings: 2 (W-1)/W of the message read per rank);
* the sum is taken in rank order, so the result is bit-identical on every rank and every run —
  the same contract as ``Comm._all_reduce_oneshot`` but without the all-gather round;
* waits are bounded in the kernel (``timeout_s``: ``AVMI_P2P_TIMEOUT_S``, else the communicator's
  process-group timeout, 600 s by default — ranks minutes apart in host work are ordinary).  A
  timed-out wait records status 1 in a pinned host-mapped word and POISONS the flag it raised for
  the late peer, whose kernel then records status 2 when it arrives; a rank whose status is set
  raises poisoned flags on every later call.  Every call is CHECKED by default: the host waits for
  the kernel's event and raises :class:`P2PError` (after poisoning every peer's flags) when the
  status is set — a garbage sum is never returned.  ``checked=False`` (the NB side-stream overlap)
  leaves the check to the communicator's next collective or output gate (``Comm.check``).

Staging memory is uncached when any peer sits on another device (``AVMI_P2P_UNCACHED`` overrides):
peers read it over xGMI while the owner's kernel is still running, so no line may linger in an
L2; ranks that share one device keep the cached default (same L2, release / acquire fences).

Teardown is collective too: :meth:`close` unmaps the peers' regions, barriers, then frees the
rank's own region (a peer must never read freed memory).
"""
from __future__ import annotations

import os

import torch

from .. import _native

_DTYPES = (torch.float32, torch.float64, torch.int32, torch.int64)


_MAX_EPOCH = 0x3FFFFFFF   # avk::P2P_MAX_EPOCH: 2 * epoch stays below the poison bit


class P2PError(RuntimeError):
    pass


def _device_identity(device: torch.device) -> str:
    """Host name + device UUID (or PCI bus id): equal for ranks sharing one GPU."""
    import socket
    try:
        props = torch.cuda.get_device_properties(device)
        uid = getattr(props, "uuid", None)
        if uid is None:
            uid = f"{getattr(props, 'pci_bus_id', '?')}:{getattr(props, 'pci_device_id', '?')}"
    except Exception:  # noqa: BLE001 - no device runtime (CPU tests): the ordinal stands in
        uid = str(device)
    return f"{socket.gethostname()}/{uid}"


def _agree(comm, ok: bool) -> bool:
    """All ranks' ``ok`` AND-ed (one min all-reduce through the library collective)."""
    f = torch.tensor([1 if ok else 0], dtype=torch.int32,
                     device=comm.device if getattr(comm, "pg_backend", "nccl") == "nccl" else "cpu")
    comm.all_reduce(f, "min", algo="ring")
    return bool(f.item())


class P2PAllReduce:
    """One communicator's peer-mapped all-reduce state.  Construct on every rank together."""

    def __init__(self, comm, device: torch.device, cap_bytes: int | None = None,
                 oneshot_max: int | None = None, timeout_s: float | None = None):
        if device.type != "cuda":
            raise ValueError("the peer-mapped all-reduce needs device tensors")
        cap = int(cap_bytes or os.environ.get("AVMI_P2P_CAP", str(8 << 20)))
        self.oneshot_max = int(oneshot_max or os.environ.get("AVMI_P2P_ONESHOT_MAX", str(256 << 10)))
        self.comm = comm
        self.device = device
        self.world, self.rank = comm.world, comm.rank
        if timeout_s is None:
            timeout_s = float(os.environ.get("AVMI_P2P_TIMEOUT_S", getattr(comm, "timeout_s", 600.0)))
        self.timeout_s = float(timeout_s)
        env_unc = os.environ.get("AVMI_P2P_UNCACHED")
        if env_unc is not None:
            uncached = env_unc == "1"
        else:                      # peers on other devices read our staging mid-kernel over xGMI
            ids = comm.all_gather_object(_device_identity(device))
            uncached = any(i != ids[0] for i in ids)
        self.uncached = uncached
        # every step that can fail on ONE rank (allocation, export, mapping a peer) is followed by
        # an agreement all-reduce, so all ranks raise together and the collective sequence of the
        # caller stays aligned (a rank leaving early would pair its next collective with a peer's
        # barrier here)
        self._h, err = None, None
        try:
            self._h = _native.C().P2PComm(device.index, cap, uncached)
            self.cap_bytes = int(self._h.cap_bytes)
            self._h.set_timeout(self.timeout_s)
            mine = bytes(self._h.handles())
        except Exception as e:     # noqa: BLE001 - reported through the agreement below
            err, mine = e, b""
        handles = comm.all_gather_object(mine)
        if err is None and all(handles):
            try:
                self._h.open(list(handles), self.rank, self.world)
            except Exception as e:  # noqa: BLE001
                err = e
        elif err is None:
            err = P2PError("a peer could not export its staging region")
        if not _agree(comm, err is None):
            h, self._h = self._h, None
            if h is not None:
                try:
                    h.close_peers()
                except Exception:  # noqa: BLE001 - nothing mapped yet
                    pass
            comm.barrier()         # every rank: no peer still maps this rank's region
            if h is not None:
                h.release()
            raise P2PError(f"rank {self.rank}: peer-mapped all-reduce unavailable "
                           f"({err!r} here)" if err is not None else
                           f"rank {self.rank}: peer-mapped all-reduce unavailable on another rank")
        self.epoch = 0
        self.failed = 0
        self.calls = {"oneshot": 0, "twoshot": 0}

    @staticmethod
    def supports(t: torch.Tensor) -> bool:
        return t.is_cuda and t.dtype in _DTYPES

    def all_reduce(self, t: torch.Tensor, algo: str | None = None, checked: bool = True) -> torch.Tensor:
        """In-place sum of ``t`` over all ranks (stream-ordered on the current stream); returns ``t``.
        ``algo``: None (by size), "oneshot" or "twoshot".  ``checked``: wait for the kernel and
        raise :class:`P2PError` if a wait failed (default); otherwise the caller checks later."""
        if self._h is None:
            raise P2PError(f"rank {self.rank}: the peer-mapped all-reduce is closed")
        self.check(block=False)                 # a failure seen since the last call: never launch on it
        if t.numel() == 0:
            return t
        nbytes = t.numel() * t.element_size()
        if nbytes > self.cap_bytes:
            raise ValueError(f"p2p all-reduce: {nbytes} bytes exceed the staging capacity {self.cap_bytes}")
        if self.epoch >= _MAX_EPOCH:
            raise P2PError(f"rank {self.rank}: p2p epoch space exhausted; rebuild the communicator")
        two = (algo == "twoshot") if algo is not None else nbytes > self.oneshot_max
        x = t
        if not t.is_contiguous() or t.data_ptr() % 16 != 0:
            x = t.contiguous().clone()
        self.epoch += 1
        self._h.all_reduce(x, self.epoch, two)
        self.calls["twoshot" if two else "oneshot"] += 1
        if x is not t:
            t.copy_(x)
        if checked:
            self.check(block=True)
        return t

    def set_timeout(self, seconds: float) -> None:
        """Bound of every later kernel wait (the selection probe runs under a short one)."""
        self.timeout_s = float(seconds)
        if self._h is not None:
            self._h.set_timeout(self.timeout_s)

    def status(self, block: bool = False) -> int:
        """0 healthy, 1 a wait of this rank timed out, 2 a peer reported a failure.  ``block``
        waits for the last call's kernel first; otherwise only finished kernels are seen."""
        if self._h is None:
            return 0
        if block:
            self._h.sync_last()
        return int(self._h.host_status())

    def ok(self) -> bool:
        """True when no wait of this rank's kernels failed (waits for the last call; local)."""
        return self.status(block=True) == 0

    def check(self, block: bool = True) -> None:
        """Raise :class:`P2PError` if a wait of this rank's kernels failed, after poisoning every
        peer's flags so their next wait on this rank fails at once instead of timing out."""
        st = self.status(block)
        if st != 0:
            self.failed = st
            try:
                self._h.poison()
            except Exception:  # noqa: BLE001 - the channel is already broken; the raise matters
                pass
            what = "a wait timed out here" if st == 1 else "a peer reported a failure"
            raise P2PError(f"rank {self.rank}: peer-mapped all-reduce failed at epoch <= {self.epoch} "
                           f"({what}); the ranks are out of step or a peer is gone")

    def close(self) -> None:
        """Collective: unmap peers, barrier, free this rank's region."""
        if self._h is None:
            return
        torch.cuda.synchronize(self.device)
        self._h.close_peers()   # even after a failure: the barrier keeps every rank's region mapped
                                # until no peer's kernel can still read it
        self.comm.barrier()
        self._h.release()
        self._h = None
