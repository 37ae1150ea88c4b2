"""Online multi-armed-bandit serving loop (replaces the Storm topology + Redis queues).

Reference: ``ReinforcementLearnerTopology`` (J/storm/ReinforcementLearnerTopology.java:45-88) with
``RedisSpout`` RPOP of ``eventID,roundNum`` (J/storm/RedisSpout.java:86-100),
``ReinforcementLearnerBolt.process`` (J/storm/ReinforcementLearnerBolt.java:97-129: read rewards,
``setReward``, ``nextActions``, write actions), ``RedisRewardReader`` (LINDEX walk) and
``RedisActionWriter`` (LPUSH ``eventID,actions``); the load generator ``P/app/lead_gen.py``.

MI355X design: one process owns a device-resident :class:`~avenir_amd.models.bandit.BanditBank`
(G independent learners x A arms).  Producers push events / rewards into lock-free native SPSC
rings (``_C.SpscRing``); the serving loop drains them in micro-batches: ALL pending rewards are one
scatter-add, and ALL pending events are answered by ONE K20 selection launch (events of the same
group get distinct draws of the same round).  Unlike the reference's shuffle-grouped bolts, there
is exactly one learner per group, so no event stream is split between independent learners.
"""
from __future__ import annotations

import collections
import threading
import time
from pathlib import Path
from typing import Sequence

import torch

from .. import _native
from ..models.bandit import BanditBank

REWARD_SCALE = 1_000_000       # rewards travel through the int64 ring in fixed point


class _PyRing:
    """Fallback queue with the SpscRing interface (used when the native module is unavailable)."""

    def __init__(self, cap: int, rec_len: int):
        self.q = collections.deque(maxlen=cap)
        self.rec_len = rec_len

    def push(self, rec):
        if len(self.q) == self.q.maxlen:
            return False
        self.q.append(list(rec))
        return True

    def pop_batch(self, n):
        out = []
        while self.q and len(out) < n:
            out.append(self.q.popleft())
        return torch.tensor(out, dtype=torch.long).view(-1, self.rec_len)

    def size(self):
        return len(self.q)


def _ring(cap: int, rec_len: int):
    if _native.available():
        return _native.C().SpscRing(cap, rec_len)
    return _PyRing(cap, rec_len)


class BanditService:
    def __init__(self, bank: BanditBank, capacity: int = 1 << 16, max_batch: int = 4096):
        self.bank = bank
        self.events = _ring(capacity, 2)          # (event_id, group)
        self.rewards = _ring(capacity, 3)         # (group, action, reward * REWARD_SCALE)
        self.max_batch = max_batch
        self.out: collections.deque = collections.deque()
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self.stats = {"events": 0, "rewards": 0, "batches": 0}

    # -- producers -------------------------------------------------------------------------------
    def submit_event(self, event_id: int, group: int = 0) -> bool:
        return self.events.push([int(event_id), int(group)])

    def submit_reward(self, action: int | str, reward: float, group: int = 0) -> bool:
        a = self.bank.actions.index(action) if isinstance(action, str) else int(action)
        return self.rewards.push([int(group), a, int(round(reward * REWARD_SCALE))])

    # -- serving loop ----------------------------------------------------------------------------
    def step(self) -> int:
        """Drain rewards then events once; returns the number of events answered."""
        rw = self.rewards.pop_batch(self.max_batch)
        if rw.shape[0]:
            self.bank.set_rewards(rw[:, 0], rw[:, 1], rw[:, 2].double() / REWARD_SCALE)
            self.stats["rewards"] += int(rw.shape[0])
        ev = self.events.pop_batch(self.max_batch)
        n = int(ev.shape[0])
        if n == 0:
            return 0
        groups = ev[:, 1].clamp(0, self.bank.G - 1)
        # rank of each event within its group -> column of the selection batch
        order = torch.argsort(groups, stable=True)
        g_sorted = groups[order]
        first = torch.searchsorted(g_sorted, g_sorted, right=False)
        col = torch.empty_like(order)
        col[order] = torch.arange(n) - first
        width = int(col.max()) + 1
        acts = self.bank.next_actions(width).cpu()                  # [G, width]
        chosen = acts[groups, col]
        with self._lock:
            for eid, a in zip(ev[:, 0].tolist(), chosen.tolist()):
                self.out.append((eid, self.bank.actions[a]))
        self.stats["events"] += n
        self.stats["batches"] += 1
        return n

    def run_forever(self, idle_sleep_s: float = 0.0005):
        while not self._stop.is_set():
            if self.step() == 0:
                time.sleep(idle_sleep_s)

    def start(self):
        self._stop.clear()
        self._thread = threading.Thread(target=self.run_forever, daemon=True)
        self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)

    def actions(self, max_n: int | None = None) -> list[tuple[int, str]]:
        """Drain answered events as (event_id, action) — the reference's action-queue records."""
        out = []
        with self._lock:
            while self.out and (max_n is None or len(out) < max_n):
                out.append(self.out.popleft())
        return out

    # -- checkpoint ------------------------------------------------------------------------------
    def checkpoint(self, path):
        Path(path).write_text("\n".join(self.bank.get_model()) + "\n")

    def restore(self, path):
        self.bank.build_model([l for l in Path(path).read_text().splitlines() if l.strip()])


def simulate_lead_generation(service: BanditService, ctr: dict[str, float], n_rounds: int = 100,
                             events_per_round: int = 50, reward_value: float = 100.0, seed: int = 0) -> dict:
    """Load generator (P/app/lead_gen.py): post events, read actions, reward clicks with the
    per-action click-through rate; returns the click rate per action and overall."""
    g = torch.Generator().manual_seed(seed)
    eid = 0
    shown = collections.Counter()
    clicks = collections.Counter()
    for _ in range(n_rounds):
        for _ in range(events_per_round):
            service.submit_event(eid, 0)
            eid += 1
        service.step()
        for _, a in service.actions():
            shown[a] += 1
            if float(torch.rand(1, generator=g)) < ctr[a]:
                clicks[a] += 1
                service.submit_reward(a, reward_value)
            else:
                service.submit_reward(a, 0.0)
    total = sum(shown.values())
    return {"shown": dict(shown), "clicks": dict(clicks), "ctr": sum(clicks.values()) / max(total, 1)}
