"""Per-iteration robustness for the iterative algorithms.

The reference makes its iterative jobs restartable through the state files each driver iteration
leaves behind: the coefficient file that ``LogisticRegressionJob`` appends one line to per
iteration (J/regress/LogisticRegressionJob.java:220-255, main loop :279-289), the decision-path
JSON ``DecisionTreeBuilder`` rewrites per tree level (J/tree/DecisionTreeBuilder.java:713-725,
R/detr.sh:34-54), the cluster files of ``KmeansCluster``.  A failed Hadoop task is re-attempted
(``mapreduce.map.maxattempts``) and the driver restarts from the last completed iteration.

Here every iterative loop (k-means Lloyd, logistic-regression Newton / GD, tree levels, GBT
rounds, SA / GA generations, Apriori levels) runs inside an ``IterationLoop``:

* ``restore()`` returns the last committed iteration's tensors from
  ``<dir>/<algo>.ckpt`` (the CRC-checked container of ``utils/checkpoint``), so a job started
  fresh after a crash — new processes — continues where the previous one stopped and produces the
  same result as an uninterrupted run.  Replicated state (rank 0 writes it) resumes at any world
  size: k-means, logistic regression and Apriori state does not depend on the sharding; GBT
  checkpoints its trees and global loss sums and every rank replays the trees over its own rows
  to rebuild the raw scores; SA chains and GA islands are keyed by GLOBAL chain / island index
  (their random streams too), so rank 0 checkpoints all of them and a resuming job re-deals them
  over its own ranks.  Sharded state (``<algo>.rank<r>.ckpt`` per rank; SA over a generic domain,
  whose torch generator is per rank) is only valid at the world size that wrote it: ``restore()``
  checks the recorded world size and the set of rank files on every rank and refuses a resume at
  a different world size with :class:`WorldSizeMismatch` instead of letting some ranks resume and
  others start over;
* ``step(it)`` wraps one iteration: it beats the ``Watchdog`` (a stalled collective aborts the rank
  with exit code 75 so ``torchrun --max-restarts`` relaunches it), runs the env-driven fault
  injector (``AVMI_FAULT_RANK`` / ``AVMI_FAULT_ITER`` / ``AVMI_FAULT_MODE``) and opens a tracer
  range (roctx on the GPU) named ``<algo>.iter``;
* ``commit(it, tensors)`` writes the iteration's state (rank 0 only unless ``sharded``; atomic
  tmp + rename, so a crash mid-write leaves the previous checkpoint intact).

Configuration: explicit arguments, or the environment (``AVENIR_CKPT_DIR``, ``AVENIR_RESUME``
= 0/1, ``AVENIR_CKPT_EVERY``, ``AVENIR_WATCHDOG_S``), which is how the CLI's ``--checkpoint-dir`` /
``--resume`` flags reach library code.  With no directory configured the loop only traces and
injects faults (no I/O).
"""
from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass
from pathlib import Path

import torch

from . import checkpoint as ckpt
from .tracing import TRACER


@dataclass
class RecoveryConfig:
    directory: str | None = None
    resume: bool = True
    every: int = 1
    watchdog_s: float | None = None

    @classmethod
    def from_env(cls) -> "RecoveryConfig":
        wd = os.environ.get("AVENIR_WATCHDOG_S")
        return cls(os.environ.get("AVENIR_CKPT_DIR") or None,
                   os.environ.get("AVENIR_RESUME", "1") != "0",
                   int(os.environ.get("AVENIR_CKPT_EVERY", "1")),
                   float(wd) if wd else None)


class WorldSizeMismatch(RuntimeError):
    """A sharded checkpoint was written at a different world size than the resuming job's."""


class IterationLoop:
    """Checkpoint / resume + watchdog + fault injection + tracing around one iterative algorithm.

    ``algo`` names the checkpoint file; use a distinct name per independent loop of one job
    (e.g. ``kmeans.g0``, ``kmeans.g1`` for two launch groups)."""

    def __init__(self, algo: str, config: RecoveryConfig | None = None, comm=None,
                 sharded: bool = False, device=None):
        from ..parallel.comm import get_comm
        self.algo = algo
        self.cfg = config or RecoveryConfig.from_env()
        self.comm = comm or get_comm()
        self.sharded = sharded
        self.device = device
        self.restored_from: int | None = None
        self._wd = None
        if self.cfg.watchdog_s:
            from ..parallel.comm import Watchdog
            self._wd = Watchdog(self.cfg.watchdog_s, abort=True)

    # ------------------------------------------------------------------------------------------
    @property
    def enabled(self) -> bool:
        return self.cfg.directory is not None

    @property
    def path(self) -> Path | None:
        if not self.enabled:
            return None
        suffix = f".rank{self.comm.rank}" if self.sharded else ""
        return Path(self.cfg.directory) / f"{self.algo}{suffix}.ckpt"

    def restore(self, device=None) -> tuple[int, dict | None, dict | None]:
        """(next_iteration, tensors, meta) of the last committed iteration, or (0, None, None)."""
        p = self.path
        if p is None or not self.cfg.resume:
            return 0, None, None
        if self.sharded:
            self._check_shard_set()
            # no rank may commit its first shard while another is still listing the directory
            # (a fast rank's fresh rank<r>.ckpt would read as a foreign partial shard set)
            if self.comm.world > 1:
                self.comm.barrier()
        if not p.exists():
            return 0, None, None
        t, m = ckpt.load(p, device or self.device or "cpu")
        if m.get("algorithm") != self.algo:
            raise IOError(f"checkpoint {p} belongs to {m.get('algorithm')!r}, not {self.algo!r}")
        if self.sharded and int(m.get("world_size", self.comm.world)) != self.comm.world:
            raise WorldSizeMismatch(f"sharded checkpoint {p} was written at world size {m.get('world_size')}; "
                                    f"resuming at world size {self.comm.world} would mix resumed and fresh ranks "
                                    f"(re-run at world size {m.get('world_size')} or clear {self.cfg.directory})")
        self.restored_from = int(m["iteration"])
        return self.restored_from + 1, t, m

    def _check_shard_set(self) -> None:
        """Every rank sees the same directory: the rank files present must be exactly ranks
        0..world-1 (or none).  A world-2 checkpoint resumed at world 4 (ranks 2, 3 without a file)
        or at world 1 (an orphaned rank-1 file) is refused on every rank alike."""
        d = Path(self.cfg.directory)
        found = set()
        pre = f"{self.algo}.rank"
        if d.is_dir():
            for f in d.iterdir():
                if f.name.startswith(pre) and f.name.endswith(".ckpt"):
                    mid = f.name[len(pre):-len(".ckpt")]
                    if mid.isdigit():
                        found.add(int(mid))
        if found and found != set(range(self.comm.world)):
            raise WorldSizeMismatch(f"sharded checkpoint of {self.algo!r} has rank files {sorted(found)}; this job "
                                    f"runs {self.comm.world} ranks (re-run at world size {max(found) + 1} or clear "
                                    f"{self.cfg.directory})")

    @contextlib.contextmanager
    def step(self, it: int, nbytes: float = 0.0, flops: float = 0.0):
        from ..parallel.comm import maybe_inject_fault
        if self._wd is not None:
            self._wd.beat()
        maybe_inject_fault(it, self.comm.rank)
        with TRACER.range(f"{self.algo}.iter", nbytes, flops, self.device):
            yield

    def commit(self, it: int, tensors: dict[str, torch.Tensor], meta: dict | None = None,
               force: bool = False) -> bool:
        if not self.enabled:
            return False
        if not force and (it + 1) % max(1, self.cfg.every) != 0:
            return False
        if not self.sharded and self.comm.rank != 0:
            return False
        m = {"algorithm": self.algo, "iteration": it, "world_size": self.comm.world}
        m.update(meta or {})
        ckpt.save(self.path, tensors, m)
        return True

    def close(self) -> None:
        if self._wd is not None:
            self._wd.stop()
            self._wd = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False


def loop(algo: str, **kw) -> IterationLoop:
    return IterationLoop(algo, **kw)
