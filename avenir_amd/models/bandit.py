"""Multi-armed bandits: 11 online learners as one batched, device-resident bank of independent
learners, plus the batch (MapReduce-style) bandits.

Reference: ``MultiArmBanditLearner`` SPI and its factory (``J/reinforce/MultiArmBanditLearnerFactory
.java:30-79``): randomGreedy, upperConfidenceBoundOne, upperConfidenceBoundTwo, softMax,
thompsonSampler, optimisticThompsonSampler, intervalEstimator, actionPursuit, rewardComparison,
exponentialWeight, exponentialWeightExpert; ``min.trial`` forcing, ``decision.batch.size``,
``reward.scale``, text model get/build and ``merge`` (``MultiArmBanditLearner.java:98-307``); the batch
bandits ``GreedyRandomBandit``, ``AuerDeterministic``, ``SoftMaxBandit``, ``RandomFirstGreedyBandit``
(``J/reinforce/*Bandit.java``); the Spark per-group bandit (``S/reinforce/MultiArmBandit.scala``).

A ``BanditBank`` holds G learners x A arms as SoA tensors; ``next_actions`` decides for every group in
ONE K20 kernel launch (one wavefront per group); rewards are applied with batched scatter updates.
Documented divergence: the reference RandomGreedyLearner explores when ``curProb < random()``
(i.e. with probability 1 - eps, ``RandomGreedyLearner.java:88``); here exploration happens with
probability eps as the algorithm intends.
"""
from __future__ import annotations

import math
from typing import Sequence

import numpy as np
import torch

from .. import _native
from ..ops.random import philox4x32, u32_to_unit

ALGOS = {
    "randomGreedy": 0, "upperConfidenceBoundOne": 1, "upperConfidenceBoundTwo": 2, "softMax": 3,
    "thompsonSampler": 4, "optimisticThompsonSampler": 5, "intervalEstimator": 6,
    "actionPursuit": 100, "rewardComparison": 100, "exponentialWeight": 100, "exponentialWeightExpert": 100,
}
_RED = {"none": 0, "linear": 1, "logLinear": 2}


class BanditBank:
    def __init__(self, algo: str, actions: Sequence[str], n_groups: int = 1, config: dict | None = None,
                 device="cpu", seed: int = 0, experts: torch.Tensor | None = None):
        if algo not in ALGOS:
            raise ValueError(f"unknown learner type {algo}")
        cfg = dict(config or {})
        self.algo, self.code = algo, ALGOS[algo]
        self.actions = list(actions)
        self.G, self.A = n_groups, len(actions)
        self.cfg = cfg
        self.dev = torch.device(device)
        self.seed = seed
        self.round = int(cfg.get("current.decision.round", 0))
        self.batch = int(cfg.get("decision.batch.size", 1))
        self.reward_scale = float(cfg.get("reward.scale", 1.0))
        G, A, dev = self.G, self.A, self.dev
        self.trials = torch.zeros((G, A), dtype=torch.int32, device=dev)
        self.rsum = torch.zeros((G, A), dtype=torch.float32, device=dev)
        self.bin_width = float(cfg.get("bin.width", 1.0))
        nb = int(math.ceil(float(cfg.get("max.reward", 100)) / self.bin_width)) if algo in (
            "thompsonSampler", "optimisticThompsonSampler", "intervalEstimator") else 1
        self.nb = max(nb, 1)
        self.hist = torch.zeros((G, A, self.nb), dtype=torch.int32, device=dev)
        self.probs = torch.full((G, A), 1.0 / A, dtype=torch.float32, device=dev)
        self.pref = torch.zeros((G, A), dtype=torch.float32, device=dev)
        self.weight = torch.ones((G, A), dtype=torch.float32, device=dev)
        self.ref_reward = torch.full((G,), float(cfg.get("intial.reference.reward", 100.0)), device=dev)
        self.gstate = torch.zeros((G, 4), dtype=torch.float32, device=dev)
        self.gstate[:, 0] = float(cfg.get("temp.constant", 100.0))
        self.gstate[:, 1] = float(cfg.get("confidence.limit", 90.0))
        self.istate = torch.zeros((G, 4), dtype=torch.int32, device=dev)
        self.istate[:, 0] = -1
        self.epochs = torch.zeros((G, A), dtype=torch.int32, device=dev)
        self.experts = experts.float().to(dev) if experts is not None else None   # [E, A]
        if self.experts is not None:
            self.expert_w = torch.ones((G, self.experts.shape[0]), dtype=torch.float32, device=dev)
        f = torch.zeros(8, dtype=torch.float32)
        i = torch.zeros(8, dtype=torch.int32)
        i[0] = int(cfg.get("min.trial", -1))
        if algo == "randomGreedy":
            f[0] = float(cfg.get("random.selection.prob", 0.5))
            f[1] = float(cfg.get("prob.reduction.constant", 1.0))
            f[2] = float(cfg.get("min.prob", -1.0))
            i[1] = _RED[cfg.get("prob.reduction.algorithm", "linear")]
        elif algo == "upperConfidenceBoundTwo":
            f[0] = float(cfg.get("alpha", 0.1))
        elif algo in ("thompsonSampler", "optimisticThompsonSampler"):
            i[2] = int(cfg.get("min.sample.size", 0))
        self.fparam, self.iparam = f.to(dev), i.to(dev)
        self._refresh_probs()

    # ------------------------------------------------------------------------------------------
    def _refresh_probs(self) -> None:
        a = self.algo
        if a == "rewardComparison":
            self.probs = torch.softmax(self.pref, 1)
        elif a == "exponentialWeight":
            g = float(self.cfg.get("distr.constant", 0.1))
            self.probs = (1 - g) * self.weight / self.weight.sum(1, keepdim=True) + g / self.A
        elif a == "exponentialWeightExpert":
            g = float(self.cfg.get("distr.constant", 0.1))
            mix = (self.expert_w @ self.experts) / self.expert_w.sum(1, keepdim=True)
            self.probs = (1 - g) * mix / mix.sum(1, keepdim=True) + g / self.A

    def next_actions(self, batch: int | None = None) -> torch.Tensor:
        """Action index per group: int32 [G, batch]."""
        b = batch or self.batch
        if self.dev.type == "cuda":
            out = _native.C().bandit_select(self.code, b, self.trials, self.rsum, self.probs.contiguous(), self.hist,
                                            self.bin_width, self.fparam, self.iparam, self.gstate, self.istate,
                                            self.epochs, self.seed, self.round)
        else:
            out = self._select_ref(b)
        self.round += 1
        self._after_round()
        return out

    def _after_round(self) -> None:
        cfg = self.cfg
        if self.algo == "softMax":
            r = self.round - max(int(cfg.get("min.trial", 0)), 0)
            red = cfg.get("temp.reduction.algorithm", "linear")
            if r > 1 and red != "none":
                t = self.gstate[:, 0]
                t = t / r if red == "linear" else t * math.log(r) / r
                mn = float(cfg.get("min.temp.constant", -1.0))
                if mn > 0:
                    t = t.clamp_min(mn)
                self.gstate[:, 0] = t
        elif self.algo == "intervalEstimator":
            step = float(cfg.get("confidence.limit.reduction.step", 0.0))
            iv = int(float(cfg.get("confidence.limit.reduction.round.interval", 0)) or 0)
            if step > 0 and iv > 0 and self.round % iv == 0:
                mn = float(cfg.get("min.confidence.limit", 50.0))
                self.gstate[:, 1] = (self.gstate[:, 1] - step).clamp_min(mn)

    # ------------------------------------------------------------------------------------------
    def set_rewards(self, groups: torch.Tensor, actions: torch.Tensor, rewards: torch.Tensor) -> None:
        dev = self.dev
        g = groups.long().to(dev)
        a = actions.long().to(dev)
        r = rewards.float().to(dev)
        flat = g * self.A + a
        self.trials.view(-1).index_add_(0, flat, torch.ones_like(flat, dtype=torch.int32))
        sr = r / self.reward_scale
        self.rsum.view(-1).index_add_(0, flat, sr)
        if self.nb > 1:
            bi = (r / self.bin_width).long().clamp(0, self.nb - 1)
            self.hist.view(-1).index_add_(0, flat * self.nb + bi, torch.ones_like(bi, dtype=torch.int32))
        algo = self.algo
        if algo == "actionPursuit":
            lr = float(self.cfg.get("pursuit.learning.rate", 0.05))
            mean = self.rsum / self.trials.clamp_min(1)
            best = mean.argmax(1, keepdim=True)
            is_best = torch.zeros_like(self.probs).scatter_(1, best, 1.0)
            touched = torch.zeros(self.G, dtype=torch.bool, device=dev)
            touched[g] = True
            upd = torch.where(is_best > 0, self.probs + lr * (1 - self.probs), self.probs - lr * self.probs)
            self.probs = torch.where(touched.view(-1, 1), upd, self.probs)
        elif algo == "rewardComparison":
            pc = float(self.cfg.get("preference.change.rate", 0.01))
            rc = float(self.cfg.get("reference.reward.change.rate", 0.01))
            mean = (self.rsum / self.trials.clamp_min(1)).view(-1)[flat]
            self.pref.view(-1).index_add_(0, flat, pc * (mean - self.ref_reward[g]))
            self.ref_reward.index_add_(0, g, rc * (mean - self.ref_reward[g]))
        elif algo == "exponentialWeight":
            gam = float(self.cfg.get("distr.constant", 0.1))
            p = self.probs.view(-1)[flat].clamp_min(1e-12)
            self.weight.view(-1).index_copy_(0, flat, self.weight.view(-1)[flat] * torch.exp(gam * (sr / p) / self.A))
        elif algo == "exponentialWeightExpert":
            gam = float(self.cfg.get("distr.constant", 0.1))
            p = self.probs.view(-1)[flat].clamp_min(1e-12)
            xhat = self.experts[:, a].T * (sr / p).view(-1, 1)      # [M, E]
            self.expert_w.index_copy_(0, g, self.expert_w[g] * torch.exp(gam * xhat / self.A))
        self._refresh_probs()

    # ------------------------------------------------------------------------------------------
    def _select_ref(self, batch: int) -> torch.Tensor:
        """Host reference of the K20 kernel (same Philox streams)."""
        G, A = self.G, self.A
        trials = self.trials.cpu().numpy()
        rsum = self.rsum.cpu().numpy()
        probs = self.probs.cpu().numpy().astype(np.float32)
        hist = self.hist.cpu().numpy()
        f, i = self.fparam.cpu().numpy(), self.iparam.cpu().numpy()
        gst, ist, ep = self.gstate.cpu().numpy(), self.istate.cpu().numpy(), self.epochs.cpu().numpy()
        out = np.zeros((G, batch), dtype=np.int32)
        code = self.code
        # arm k on lane k % 64, slot k // 64; E slots (a power of two, as the kernel's template)
        E = 1
        while E * 64 < A:
            E *= 2
        for g in range(G):
            n = trials[g].astype(np.int64)
            mean = np.where(n > 0, rsum[g] / np.maximum(n, 1), 0.0).astype(np.float32)
            total = int(n.sum())
            for b in range(batch):
                idx = np.uint64((g * batch + b) * E * 64) + np.arange(E * 64, dtype=np.uint64)
                x, y, _, _ = philox4x32(self.seed, self.round, idx)
                u_lane, v_lane = u32_to_unit(x), u32_to_unit(y)
                u_a, u_b = float(u32_to_unit(x[:1])[0]), float(u32_to_unit(y[:1])[0])
                action = -1
                if code != 100 and i[0] > 0:
                    under = np.nonzero(n < i[0])[0]
                    if under.size:
                        action = int(under[0])
                if action < 0:
                    score = None
                    if code == 0:
                        t = max(total, 1)
                        eps = f[0] if i[1] == 0 else (f[0] * f[1] / t if i[1] == 1 else f[0] * f[1] * math.log(t) / t)
                        eps = min(eps, f[0])
                        if f[2] > 0:
                            eps = max(eps, f[2])
                        if u_a < eps:
                            action = min(int(u_b * A), A - 1)
                        score = mean
                    elif code == 1:
                        t = max(total, 1)
                        score = np.where(n > 0, mean + np.sqrt(2 * math.log(t) / np.maximum(n, 1)), np.inf)
                    elif code == 2:
                        if ist[g, 0] >= 0 and ist[g, 1] < ist[g, 2]:
                            action = int(ist[g, 0])
                        else:
                            tao = np.where(ep[g] == 0, 1.0, (1 + f[0]) ** ep[g])
                            aa = (1 + f[0]) * np.log(math.e * max(total, 1) / tao) / (2 * tao)
                            score = mean + np.sqrt(np.maximum(aa, 0))
                    elif code == 3:
                        w = np.exp(mean / max(gst[g, 0], 1e-6))
                        action = _pick(w, u_a)
                    elif code in (4, 5):
                        if total < i[2]:
                            action = min(int(u_a * A), A - 1)
                        else:
                            score = np.array([_thompson(hist[g, k], self.bin_width, float(u_lane[k]), float(v_lane[k]))
                                              for k in range(A)], dtype=np.float32)
                            if code == 5:
                                score = np.maximum(score, mean)
                    elif code == 6:
                        conf = gst[g, 1]
                        score = np.array([_interval_ub(hist[g, k], self.bin_width, conf) for k in range(A)])
                    elif code == 100:
                        action = _pick(probs[g], u_a)
                    if action < 0:
                        action = int(np.argmax(score))
                out[g, b] = action
                if code == 2:
                    if ist[g, 0] == action and ist[g, 1] < ist[g, 2]:
                        ist[g, 1] += 1
                    else:
                        e = ep[g, action]
                        es = int(round((1 + f[0]) ** (e + 1) - (1 + f[0]) ** e))
                        ist[g, 0], ist[g, 1], ist[g, 2] = action, 1, max(es, 1)
                        ep[g, action] = e + 1
        if code == 2:
            self.istate.copy_(torch.from_numpy(ist))
            self.epochs.copy_(torch.from_numpy(ep))
        return torch.from_numpy(out)

    # ------------------------------------------------------------------------------------------
    def get_model(self, delim: str = ",") -> list[str]:
        """Per group and action: ``group,action,count,sum,mean`` (getMeanRewardStatModel)."""
        t, s = self.trials.cpu(), self.rsum.cpu()
        lines = []
        for g in range(self.G):
            for a, name in enumerate(self.actions):
                n = int(t[g, a])
                lines.append(delim.join([str(g), name, str(n), f"{float(s[g, a]):.6f}",
                                         f"{float(s[g, a]) / n if n else 0.0:.6f}"]))
        return lines

    def build_model(self, lines: list[str], delim: str = ",") -> None:
        for ln in lines:
            g, name, n, s, _ = ln.split(delim)
            a = self.actions.index(name)
            self.trials[int(g), a] = int(n)
            self.rsum[int(g), a] = float(s)
        self._refresh_probs()

    def merge(self, other: "BanditBank") -> "BanditBank":
        self.trials += other.trials.to(self.dev)
        self.rsum += other.rsum.to(self.dev)
        self.hist += other.hist.to(self.dev)
        self._refresh_probs()
        return self

    def best_actions(self) -> torch.Tensor:
        return (self.rsum / self.trials.clamp_min(1)).argmax(1)


def _pick(w: np.ndarray, u: float) -> int:
    w = w.astype(np.float32)
    cum = np.cumsum(w, dtype=np.float32)
    tot = float(cum[-1])
    hit = np.nonzero((cum > u * tot) & (w > 0))[0]
    return int(hit[0]) if hit.size else len(w) - 1


def _thompson(h: np.ndarray, bw: float, u: float, v: float) -> float:
    tot = int(h.sum())
    if tot == 0:
        return v * bw
    cum = np.cumsum(h.astype(np.float32))
    k = np.nonzero(cum >= np.float32(u) * np.float32(tot))[0]
    return (float(k[0]) + v) * bw if k.size else (len(h) - 1 + v) * bw


def _interval_ub(h: np.ndarray, bw: float, conf: float) -> float:
    tot = int(h.sum())
    if tot == 0:
        return math.inf
    cum = np.cumsum(h.astype(np.float32))
    k = np.nonzero(cum >= (0.5 + 0.5 * conf / 100.0) * tot)[0]
    return (float(k[0]) + 1.0) * bw if k.size else (len(h) - 0.5) * bw


# ================================================================================================
# batch bandits (MR map-only jobs over per-group item state)
# ================================================================================================
def batch_select(counts: torch.Tensor, rewards: torch.Tensor, batch_size: int, strategy: str = "auerGreedy",
                 round_num: int = 1, epsilon: float = 0.1, temp: float = 1.0, explore_count: int = 0,
                 seed: int = 0, group_base: int = 0) -> torch.Tensor:
    """Select ``batch_size`` distinct items per group from (count, total reward) state [G, I]:
    ``auerGreedy``/``auerDeterministic`` (UCB1 ranking), ``linear``/``logLinear`` eps-greedy
    (GreedyRandomBandit), ``softMax`` (SoftMaxBandit, sampling without replacement via Gumbel
    top-k), ``randomFirst`` (RandomFirstGreedyBandit: explore uniformly for the first
    ``explore_count`` rounds, then exploit by mean reward).  The random draws are counter-based
    (Philox keyed by (seed + round, global group ``group_base + g``, item)), so a group's selection
    does not depend on which other groups share the call — a rank's block of groups selects
    exactly what a single process selects."""
    G, I = counts.shape
    n = counts.double()
    mean = torch.where(n > 0, rewards.double() / n.clamp_min(1), torch.zeros_like(n))
    import numpy as np
    from ..ops.random import philox4x32
    idx = ((np.arange(G, dtype=np.uint64) + np.uint64(group_base))[:, None] * np.uint64(I)
           + np.arange(I, dtype=np.uint64)[None, :]).reshape(-1)
    x, y, _, _ = philox4x32(seed + round_num, 0, idx)
    u = ((x.astype(np.uint64) << np.uint64(21)) | (y.astype(np.uint64) >> np.uint64(11))).astype(np.float64)
    noise = torch.from_numpy((u + 0.5) / float(1 << 53)).view(G, I).to(counts.device)
    k = min(batch_size, I)
    if strategy in ("auerGreedy", "auerDeterministic"):
        tot = n.sum(1, keepdim=True).clamp_min(1)
        score = torch.where(n > 0, mean + torch.sqrt(2 * torch.log(tot) / n.clamp_min(1)), torch.full_like(n, math.inf))
        return torch.topk(score + 1e-9 * noise, k, 1).indices
    if strategy in ("linear", "logLinear"):
        t = max(round_num, 1)
        eps = epsilon / t if strategy == "linear" else epsilon * math.log(t + 1) / t
        explore = noise[:, :1] < eps
        rand_rank = torch.topk(noise, k, 1).indices
        greedy = torch.topk(mean + 1e-9 * noise, k, 1).indices
        return torch.where(explore, rand_rank, greedy)
    if strategy == "softMax":
        gumbel = -torch.log(-torch.log(noise.clamp(1e-12, 1 - 1e-12)))
        return torch.topk(mean / max(temp, 1e-9) + gumbel, k, 1).indices
    if strategy == "randomFirst":
        if round_num <= explore_count:
            return torch.topk(noise, k, 1).indices
        return torch.topk(mean + 1e-9 * noise, k, 1).indices
    raise ValueError(strategy)


def pac_exploration_count(n_items: int, epsilon: float, delta: float) -> int:
    """PAC-bound exploration rounds (ExplorationCounter): (4 / eps^2) ln(2 n / delta)."""
    return int(math.ceil(4.0 / (epsilon * epsilon) * math.log(2.0 * n_items / delta)))
