"""Concrete search domains: task scheduling, meeting scheduling, feature-subset selection.

* :class:`TaskScheduleSearch` — employees -> tasks (J/examples/TaskScheduleSearch.java:45-305 with
  the JSON model J/examples/TaskSchedule.java, R/taskSched.json).  Per (task, employee) component
  cost = mean of normalised travel (round-trip drive below ``airTravelDistThreshold`` miles, else the
  quadratic air-fare estimator), per-diem, hotel and skill-mismatch costs (:169-224); two tasks
  given to one employee must be ``minDaysGap`` days apart (:263-305).  Compiled once into an
  :class:`AssignmentDomain` cost table + conflict matrix, so the K22 SA kernel prices a move in
  O(1).  Notes: the reference divides per-diem/hotel by ``duration * maxRate`` and multiplies by
  ``duration``, which is 0/0 for a same-day task; the ratio is used directly here.  Geo distance
  is haversine in miles (chombo ``BasicUtils.getGeoDistance`` is external: parity unpinned).
* :class:`MeetingScheduleDomain` — (day, hour, minute) per meeting (P/app/mesched.py:53-227),
  fully vectorised: participant overlap, blocked hours and ordering constraints as [P, M, M]
  masks; per-person cost = 8 - mean free slot hours (the free-slot sum telescopes to
  10h - booked time per day), weighted by role.
* :class:`FeatureSubsetDomain` — feature selection (P/app/fesel.py) as a binary mask over F
  features with a size range and tied feature groups; the built-in evaluator scores EVERY
  candidate subset of a population with one GEMM over per-feature naive-Bayes log-likelihoods
  ([P, F] x [F, N*C]) instead of retraining a classifier per candidate.
"""
from __future__ import annotations

import json
import math
import re
from datetime import datetime
from typing import Sequence

import torch

from .domain import AssignmentDomain, SearchDomain

EARTH_RADIUS_MILES = 3958.8


def geo_distance(lat1, lon1, lat2, lon2) -> torch.Tensor:
    """Haversine great-circle distance in miles (broadcasting)."""
    lat1, lon1, lat2, lon2 = (torch.as_tensor(x, dtype=torch.float64) * (math.pi / 180) for x in (lat1, lon1, lat2, lon2))
    a = torch.sin((lat2 - lat1) / 2) ** 2 + torch.cos(lat1) * torch.cos(lat2) * torch.sin((lon2 - lon1) / 2) ** 2
    return 2 * EARTH_RADIUS_MILES * torch.asin(torch.sqrt(a.clamp(0, 1)))


def read_lenient_json(path: str) -> dict:
    """JSON with trailing commas (R/taskSched.json ends with ``,\\n}``)."""
    with open(path) as fh:
        text = fh.read()
    return json.loads(re.sub(r",(\s*[}\]])", r"\1", text))


def _java_date_format(fmt: str) -> str:
    return fmt.replace("yyyy", "%Y").replace("MM", "%m").replace("dd", "%d").replace("HH", "%H").replace("mm", "%M")


class TaskScheduleSearch(AssignmentDomain):
    def __init__(self, sched: dict, device="cpu"):
        self.sched = sched
        locs = {l["id"]: l for l in sched["locations"]}
        tasks, emps = sched["tasks"], sched["employees"]
        self.task_ids = [t["id"] for t in tasks]
        self.employee_ids = [e["id"] for e in emps]
        T, E = len(tasks), len(emps)
        tg = torch.tensor([locs[t["location"]]["gps"] for t in tasks], dtype=torch.float64)
        eg = torch.tensor([locs[e["location"]]["gps"] for e in emps], dtype=torch.float64)
        dist = geo_distance(tg[:, 0:1], tg[:, 1:2], eg[:, 0].view(1, -1), eg[:, 1].view(1, -1))   # [T, E]
        a = sched["airFareEstimator"]
        travel = torch.where(dist < sched["airTravelDistThreshold"], 2 * dist * sched["perMileDriveCost"],
                             a[0] * dist * dist + a[1] * dist + a[2])
        scale = float(sched["costScale"])
        travel = travel / sched["maxTravelCost"] * scale
        per_diem = torch.tensor([locs[t["location"]]["perDiemCost"] / sched["maxPerDiemRate"] * scale for t in tasks],
                                dtype=torch.float64).view(-1, 1)
        hotel = torch.tensor([locs[t["location"]]["hotelCost"] / sched["maxHotelRate"] * scale for t in tasks],
                             dtype=torch.float64).view(-1, 1)
        skill = torch.zeros((T, E), dtype=torch.float64)
        for i, t in enumerate(tasks):
            req = set(t["skills"])
            for j, e in enumerate(emps):
                match = sum(1 for s in e["skills"] if s in req)
                skill[i, j] = (len(t["skills"]) - match) * scale / len(t["skills"])
        self.components = {"travel": travel, "perDiem": per_diem.expand(T, E), "hotel": hotel.expand(T, E),
                           "skill": skill}
        cost = (travel + per_diem + hotel + skill) / 4.0
        # conflicts: same employee on two tasks closer than minDaysGap days (ms arithmetic as in :266)
        fmt = _java_date_format(sched.get("dateFormat", "MM-dd-yyyy"))
        day_ms = 86400000
        st = [int(datetime.strptime(t["startDate"], fmt).timestamp() * 1000) for t in tasks]
        en = [int(datetime.strptime(t["endDate"], fmt).timestamp() * 1000) for t in tasks]
        min_gap = sched["minDaysGap"] * day_ms - 4
        conflict = torch.zeros((T, T), dtype=torch.bool)
        for i in range(T):
            for j in range(T):
                if i != j:
                    conflict[i, j] = not ((st[j] - en[i]) >= min_gap or (st[i] - en[j]) >= min_gap)
        super().__init__(cost.float().to(device), conflict.to(device),
                         invalid_cost=float(sched.get("inavlidSolutionCost", sched.get("invalidSolutionCost", 150))),
                         swap_moves=True, values=self.employee_ids)

    @classmethod
    def from_json(cls, path: str, device="cpu") -> "TaskScheduleSearch":
        return cls(read_lenient_json(path), device)

    def to(self, device):
        return TaskScheduleSearch(self.sched, device)

    def format_solution(self, row: Sequence[int], comp_delim: str = ";", item_delim: str = ":") -> str:
        """Reference string form ``task:employee;task:employee...`` (BasicSearchDomain delims :47-48)."""
        return comp_delim.join(f"{t}{item_delim}{self.employee_ids[int(e)]}" for t, e in zip(self.task_ids, row))

    def parse_solution(self, text: str, comp_delim: str = ";", item_delim: str = ":") -> list[int]:
        m = dict(c.split(item_delim) for c in text.split(comp_delim))
        return [self.employee_ids.index(m[t]) for t in self.task_ids]


class MeetingScheduleDomain(SearchDomain):
    """Solution = [day, hour, minute] x M meetings (value tables from ``mesched.properties``:
    days 1..5, hours 8..16, minutes 0/30)."""

    SEC_MIN, SEC_HOUR, SEC_DAY = 60, 3600, 86400

    def __init__(self, participants: Sequence[Sequence[int]], durations: Sequence[int], n_people: int,
                 ordered: Sequence[tuple[int, int]] = (), blocked: dict | None = None,
                 role_weight: Sequence[float] | None = None, days=range(1, 6), hours=range(8, 17), minutes=(0, 30),
                 device="cpu"):
        dev = torch.device(device)
        M = len(participants)
        self.M = M
        self.days, self.hours, self.minutes = (torch.tensor(list(x), dtype=torch.float32, device=dev)
                                               for x in (days, hours, minutes))
        self.cards = torch.tensor([len(self.days), len(self.hours), len(self.minutes)] * M, dtype=torch.long, device=dev)
        self.comp_size = 3
        mem = torch.zeros((n_people, M), dtype=torch.bool)
        for m, ps in enumerate(participants):
            mem[list(ps), m] = True
        self.member = mem.to(dev)                                                   # [people, M]
        self.share = ((mem.float().T @ mem.float()) > 0).to(dev) & ~torch.eye(M, dtype=torch.bool, device=dev)
        self.dur = torch.tensor([float(d) for d in durations], device=dev) * self.SEC_MIN
        self.ordered = list(ordered)
        self.blocked = blocked or {}
        self.role_w = torch.tensor(role_weight if role_weight is not None else [1.0] * n_people, device=dev)
        self.invalid_cost = float("inf")

    @classmethod
    def random_instance(cls, n_meetings: int, n_people: int, seed: int = 0, device="cpu"):
        """Random instance like MeetingScheduleCost.__init__ (mesched.py:57-110)."""
        g = torch.Generator().manual_seed(seed)
        parts = []
        for _ in range(n_meetings):
            k = int(torch.randint(2, 7, (1,), generator=g))
            parts.append(torch.randperm(n_people, generator=g)[:k].tolist())
        dvals, dw = [30, 60, 90, 120], torch.tensor([80.0, 100, 60, 40])
        durs = [dvals[int(i)] for i in torch.multinomial(dw, n_meetings, True, generator=g)]
        order = [tuple(torch.randperm(n_meetings, generator=g)[:2].tolist())]
        blocked = {}
        for p in torch.randperm(n_people, generator=g)[:2].tolist():
            blocked[p] = (int(torch.randint(1, 6, (1,), generator=g)), int(torch.randint(8, 16, (1,), generator=g)),
                          int(torch.randint(1, 4, (1,), generator=g)))
        rw = [1.0] * n_people
        mans = torch.randperm(n_people, generator=g)[: max(1, int(0.2 * n_people))].tolist()
        for m in mans:
            rw[m] = 1.3
        rw[mans[0]] = 1.8
        return cls(parts, durs, n_people, order, blocked, rw, device=device)

    def times(self, sol):
        P = sol.shape[0]
        s3 = sol.view(P, self.M, 3)
        day = self.days[s3[..., 0]]
        start = (day - 1) * self.SEC_DAY + self.hours[s3[..., 1]] * self.SEC_HOUR + self.minutes[s3[..., 2]] * self.SEC_MIN
        return day, start, start + self.dur.view(1, -1)

    def decode(self, sol):
        P = sol.shape[0]
        s3 = sol.view(P, self.M, 3)
        return torch.stack([self.days[s3[..., 0]], self.hours[s3[..., 1]], self.minutes[s3[..., 2]]], -1).view(P, -1)

    def valid(self, sol):
        day, st, en = self.times(sol)
        overlap = (st.unsqueeze(2) < en.unsqueeze(1)) & (st.unsqueeze(1) < en.unsqueeze(2))     # [P, M, M]
        ok = ~(overlap & self.share.unsqueeze(0)).flatten(1).any(1)
        for p, (bd, bh, bdur) in self.blocked.items():
            bs = (bd - 1) * self.SEC_DAY + bh * self.SEC_HOUR
            be = bs + bdur * self.SEC_HOUR
            mine = self.member[p].view(1, -1)
            ok &= ~((st < be) & (bs < en) & mine).any(1)
        for a, b in self.ordered:
            ok &= en[:, a] <= st[:, b]
        return ok

    def cost(self, sol):
        day, st, en = self.times(sol)
        P = sol.shape[0]
        nd = len(self.days)
        dayi = sol.view(P, self.M, 3)[..., 0]                                      # [P, M] day index
        onehot = torch.nn.functional.one_hot(dayi, nd).float()                     # [P, M, D]
        mem = self.member.float()                                                  # [people, M]
        cnt = torch.einsum("qm,pmd->pqd", mem, onehot)                             # meetings per person-day
        booked = torch.einsum("qm,pmd->pqd", mem, onehot * self.dur.view(1, -1, 1))
        active = cnt > 0
        free = torch.where(active, 10 * self.SEC_HOUR - booked, torch.zeros_like(booked)).sum(2)
        nslots = torch.where(active, cnt + 1, torch.zeros_like(cnt)).sum(2)
        has = nslots > 0
        pcost = 8 - free / nslots.clamp_min(1) / self.SEC_HOUR                     # [P, people]
        w = self.role_w.view(1, -1) * has.float()
        return (pcost * w).sum(1) / w.sum(1).clamp_min(1e-12)


class FeatureSubsetDomain(SearchDomain):
    """Binary include mask over F features, size in [min_size, max_size], tied groups.

    ``cost`` defaults to the naive-Bayes validation error of each subset: with per-row, per-feature,
    per-class log-likelihoods ``LL [N, F, C]`` and class log-priors, a subset's class scores are
    ``mask @ LL`` — the whole population is scored by ONE [P, F] x [F, N*C] GEMM."""

    def __init__(self, n_features: int, min_size: int = 1, max_size: int | None = None, groups=None,
                 loglik: torch.Tensor | None = None, log_prior: torch.Tensor | None = None,
                 labels: torch.Tensor | None = None, cost_fn=None, device="cpu"):
        dev = torch.device(device)
        self.F = n_features
        self.cards = torch.full((n_features,), 2, dtype=torch.long, device=dev)
        self.min_size, self.max_size = min_size, max_size or n_features
        self.groups = groups
        self.loglik = None if loglik is None else loglik.to(dev).float()
        self.log_prior = None if log_prior is None else log_prior.to(dev).float()
        self.labels = None if labels is None else labels.to(dev).long()
        self.cost_fn = cost_fn
        self.invalid_cost = 1.0

    @classmethod
    def from_naive_bayes(cls, nb, table, labels, **kw):
        """Per-feature log-likelihoods from a fitted :class:`~avenir_amd.models.bayes.NaiveBayes`."""
        ll, lp = nb.feature_loglik(table)
        return cls(ll.shape[1], loglik=ll, log_prior=lp, labels=labels, device=ll.device, **kw)

    def valid(self, sol):
        n = sol.sum(1)
        return (n >= self.min_size) & (n <= self.max_size)

    def cost(self, sol):
        if self.cost_fn is not None:
            return torch.as_tensor(self.cost_fn(sol), device=sol.device).float()
        N, F, C = self.loglik.shape
        scores = sol.float() @ self.loglik.permute(1, 0, 2).reshape(F, N * C)            # [P, N*C]
        scores = scores.view(-1, N, C) + self.log_prior.view(1, 1, C)
        pred = scores.argmax(2)
        return (pred != self.labels.view(1, -1)).float().mean(1)

    def decode(self, sol):
        return [row.nonzero().view(-1).tolist() for row in sol]
