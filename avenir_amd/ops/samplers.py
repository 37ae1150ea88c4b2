"""Random samplers (``python/lib/sampler.py`` parity) backed by the K21 device kernel.

Every sampler has ``sample()`` (one value, the reference API) and ``sample_n(n)`` (a batch drawn on
``device`` by ONE kernel launch from counter-based Philox, so batches are reproducible and can be
sharded across ranks by offset).  ``create_sampler("a:b:...:type:dtype")`` parses the reference's
sampler spec strings (``sampler.py:863``).
"""
from __future__ import annotations

import math
from typing import Sequence

import numpy as np
import torch

from .. import _native
from .random import philox4x32, u32_to_unit

UNIFORM, NORMAL, EXPONENTIAL, LOGNORMAL, GAMMA, POISSON, PARETO, TRIANGULAR, BERNOULLI, TABLE, UNIFORM_INT = range(11)

_stream_counter = [0]


def _next_offset() -> int:
    _stream_counter[0] += 1
    return _stream_counter[0]


def device_sample(dist: int, n: int, params: Sequence[float], device="cpu", seed: int = 0,
                  offset: int | None = None, table: torch.Tensor | None = None) -> torch.Tensor:
    """n draws of a distribution (float32 [n]).  GPU: K21 kernel; CPU: the same Philox stream and
    transforms in numpy."""
    off = _next_offset() if offset is None else offset
    p = list(params) + [0.0] * (3 - len(params))
    dev = torch.device(device)
    if dev.type == "cuda":
        pt = torch.tensor(p, dtype=torch.float32, device=dev)
        tb = table.float().to(dev).contiguous() if table is not None else None
        return _native.C().sample(int(dist), int(n), pt, tb, int(seed), int(off))
    idx = np.arange(n, dtype=np.uint64)
    x, y, z, w = philox4x32(seed, off, idx)
    u1, u2 = u32_to_unit(x).astype(np.float64), u32_to_unit(y).astype(np.float64)
    nrm = np.sqrt(-2 * np.log(u1)) * np.cos(2 * np.pi * u2)
    if dist == UNIFORM:
        v = p[0] + (p[1] - p[0]) * (u1 - 0.5 / 16777216)
    elif dist == NORMAL:
        v = p[0] + p[1] * nrm
    elif dist == EXPONENTIAL:
        v = -np.log(u1) / p[0]
    elif dist == LOGNORMAL:
        v = np.exp(p[0] + p[1] * nrm)
    elif dist == GAMMA:
        v = np.random.default_rng(seed * 1000003 + off).gamma(p[0], p[1], n)
    elif dist == POISSON:
        v = np.random.default_rng(seed * 1000003 + off).poisson(p[0], n).astype(np.float64)
    elif dist == PARETO:
        v = p[1] / u1 ** (1.0 / p[0])
    elif dist == TRIANGULAR:
        lo, md, hi = p
        fc = (md - lo) / (hi - lo)
        v = np.where(u1 < fc, lo + np.sqrt(u1 * (hi - lo) * (md - lo)), hi - np.sqrt((1 - u1) * (hi - lo) * (hi - md)))
    elif dist == BERNOULLI:
        v = (u1 <= p[0]).astype(np.float64)
    elif dist == TABLE:
        cdf = table.double().cpu().numpy()
        k = np.minimum(np.searchsorted(cdf, u1, side="left"), len(cdf) - 1)
        v = p[0] + (k + u2 - 0.5 / 16777216) * p[1]
    elif dist == UNIFORM_INT:
        span = p[1] - p[0] + 1
        v = p[0] + np.minimum(np.floor(u1 * span - 0.5 / 16777216 * span), span - 1)
    else:
        raise ValueError(dist)
    return torch.from_numpy(v.astype(np.float32))


# ================================================================================================
# sampler classes
# ================================================================================================
class Sampler:
    device = "cpu"
    seed = 0

    def sample_n(self, n: int) -> torch.Tensor:
        raise NotImplementedError

    def sample(self):
        v = self.sample_n(1)
        return v[0].item() if isinstance(v, torch.Tensor) and v.dim() == 1 else v[0]

    def on(self, device, seed: int | None = None) -> "Sampler":
        self.device = device
        if seed is not None:
            self.seed = seed
        return self


class _Param(Sampler):
    dist = UNIFORM
    as_int = False

    def __init__(self, *params):
        self.params = [float(x) for x in params]

    def sample_n(self, n):
        v = device_sample(self.dist, n, self.params, self.device, self.seed)
        return torch.round(v) if self.as_int else v

    def sampleAsInt(self):
        self.as_int = True
        return self


class UniformNumericSampler(_Param):
    def __init__(self, lo, hi):
        super().__init__(lo, hi)
        self.is_int = isinstance(lo, int) and isinstance(hi, int)
        self.dist = UNIFORM_INT if self.is_int else UNIFORM


class NormalSampler(_Param):
    dist = NORMAL


GaussianRejectSampler = NormalSampler


class ExponentialSampler(_Param):
    dist = EXPONENTIAL


class LogNormalSampler(_Param):
    dist = LOGNORMAL


class GammaSampler(_Param):
    dist = GAMMA


class PoissonSampler(_Param):
    dist = POISSON


class ParetoSampler(_Param):
    dist = PARETO


class TriangularRejectSampler(_Param):
    dist = TRIANGULAR


class BernoulliTrialSampler(_Param):
    dist = BERNOULLI


class UniformCategoricalSampler(Sampler):
    def __init__(self, values: Sequence):
        self.values = list(values)

    def sample_n(self, n):
        k = device_sample(UNIFORM_INT, n, [0, len(self.values) - 1], self.device, self.seed).long()
        return [self.values[i] for i in k.tolist()]

    def sample_idx(self, n):
        return device_sample(UNIFORM_INT, n, [0, len(self.values) - 1], self.device, self.seed).long()


class NonParamRejectSampler(Sampler):
    """Histogram sampler: bins of width ``bin_width`` starting at ``lo`` with weights."""

    def __init__(self, lo: float, bin_width: float, weights: Sequence[float]):
        w = torch.tensor([float(x) for x in weights], dtype=torch.float64)
        self.cdf = (torch.cumsum(w, 0) / w.sum()).float()
        self.lo, self.bw = float(lo), float(bin_width)

    def sample_n(self, n):
        return device_sample(TABLE, n, [self.lo, self.bw], self.device, self.seed, table=self.cdf)


class DiscreteRejectSampler(Sampler):
    """Discrete values lo..hi (step) with weights (sampler.py:401)."""

    def __init__(self, lo: int, hi: int, step: int, weights: Sequence[float]):
        self.values = list(range(lo, hi + 1, step))
        w = torch.tensor([float(x) for x in weights], dtype=torch.float64)
        self.cdf = (torch.cumsum(w, 0) / w.sum()).float()

    def sample_idx(self, n):
        return device_sample(TABLE, n, [0.0, 1.0], self.device, self.seed, table=self.cdf).floor().long()

    def sample_n(self, n):
        vals = torch.tensor(self.values)
        return vals[self.sample_idx(n).cpu().clamp(0, len(self.values) - 1)]


class CategoricalRejectSampler(DiscreteRejectSampler):
    def __init__(self, values_weights: dict):
        self.values = list(values_weights)
        w = torch.tensor([float(values_weights[v]) for v in self.values], dtype=torch.float64)
        self.cdf = (torch.cumsum(w, 0) / w.sum()).float()

    def sample_n(self, n):
        return [self.values[i] for i in self.sample_idx(n).cpu().clamp(0, len(self.values) - 1).tolist()]


class NormalSamplerWithTrendCycle(Sampler):
    """Normal noise + linear trend + cyclic component over a step counter (sampler.py:309)."""

    def __init__(self, mean, sd, trend: float = 0.0, cycle: Sequence[float] = ()):
        self.mean, self.sd, self.trend, self.cycle = float(mean), float(sd), float(trend), list(cycle)
        self.step = 0

    def sample_n(self, n):
        t = torch.arange(self.step, self.step + n, dtype=torch.float32)
        v = device_sample(NORMAL, n, [self.mean, self.sd], self.device, self.seed).cpu() + self.trend * t
        if self.cycle:
            v += torch.tensor(self.cycle)[(t.long() % len(self.cycle))]
        self.step += n
        return v


class MultiVarNormalSampler(Sampler):
    def __init__(self, mean: Sequence[float], cov: Sequence[Sequence[float]]):
        self.mean = torch.tensor(mean, dtype=torch.float32)
        self.L = torch.linalg.cholesky(torch.tensor(cov, dtype=torch.float64)).float()

    def sample_n(self, n):
        d = self.mean.numel()
        z = device_sample(NORMAL, n * d, [0.0, 1.0], self.device, self.seed).view(n, d)
        return z @ self.L.to(z.device).T + self.mean.to(z.device)


JointNormalSampler = MultiVarNormalSampler


class JointNonParamRejectSampler(Sampler):
    """Joint histogram over a grid of (dim1 bins x dim2 bins ...) flattened weights."""

    def __init__(self, los: Sequence[float], widths: Sequence[float], shape: Sequence[int], weights: Sequence[float]):
        self.los, self.widths, self.shape = list(los), list(widths), list(shape)
        w = torch.tensor([float(x) for x in weights], dtype=torch.float64)
        self.cdf = (torch.cumsum(w, 0) / w.sum()).float()

    def sample_n(self, n):
        k = device_sample(TABLE, n, [0.0, 1.0], self.device, self.seed, table=self.cdf).floor().long().cpu()
        out = []
        for d in reversed(range(len(self.shape))):
            out.append(self.los[d] + (k % self.shape[d]).float() * self.widths[d])
            k = k // self.shape[d]
        return torch.stack(out[::-1], 1)


class DistrMixtureSampler(Sampler):
    def __init__(self, samplers: Sequence[Sampler], weights: Sequence[float]):
        self.samplers = list(samplers)
        self.pick = DiscreteRejectSampler(0, len(samplers) - 1, 1, weights)

    def sample_n(self, n):
        idx = self.pick.sample_idx(n).cpu()
        out = torch.zeros(n)
        for k, s in enumerate(self.samplers):
            m = idx == k
            c = int(m.sum())
            if c:
                out[m] = torch.as_tensor(s.sample_n(c), dtype=torch.float32).cpu()
        return out


class AncestralSampler(Sampler):
    """Bayesian-network ancestral sampling: parent sampler + conditional child samplers."""

    def __init__(self, parent: Sampler, children: dict, child_of_parent=lambda v: v):
        self.parent, self.children, self.key = parent, children, child_of_parent

    def sample(self):
        p = self.parent.sample()
        return p, self.children[self.key(p)].sample()

    def sample_n(self, n):
        return [self.sample() for _ in range(n)]


class ClusterSampler(Sampler):
    """Points around cluster centres (sampler.py:654)."""

    def __init__(self, centers: Sequence[Sequence[float]], sd: float, weights: Sequence[float] | None = None):
        self.centers = torch.tensor(centers, dtype=torch.float32)
        self.sd = float(sd)
        self.pick = DiscreteRejectSampler(0, len(centers) - 1, 1, weights or [1.0] * len(centers))

    def sample_n(self, n):
        k = self.pick.sample_idx(n).cpu().clamp(0, len(self.centers) - 1)
        d = self.centers.shape[1]
        z = device_sample(NORMAL, n * d, [0.0, self.sd], self.device, self.seed).cpu().view(n, d)
        return self.centers[k] + z


class PermutationSampler(Sampler):
    def __init__(self, values: Sequence):
        self.values = list(values)

    def sample_n(self, n):
        u = device_sample(UNIFORM, n * len(self.values), [0, 1], self.device, self.seed).cpu().view(n, -1)
        order = torch.argsort(u, 1)
        return [[self.values[i] for i in row] for row in order.tolist()]


class MetropolitanSampler(Sampler):
    """Metropolis MCMC with a normal proposal over a (vectorised) target density: ``chains``
    independent chains advance together on the device (sampler.py:668-762)."""

    def __init__(self, log_density, proposal_sd: float, start: float = 0.0, chains: int = 1, burn_in: int = 0):
        self.logp, self.sd, self.chains, self.burn = log_density, float(proposal_sd), chains, burn_in
        self.x = None
        self.start = float(start)
        self.accepted = 0
        self.proposed = 0

    def sample_n(self, n):
        dev = torch.device(self.device)
        if self.x is None:
            self.x = torch.full((self.chains,), self.start, device=dev)
            for _ in range(self.burn):
                self._step()
        out = torch.empty((n, self.chains), device=dev)
        for i in range(n):
            out[i] = self._step()
        return out if self.chains > 1 else out[:, 0]

    def _step(self):
        prop = self.x + device_sample(NORMAL, self.chains, [0.0, self.sd], self.device, self.seed).to(self.x.device)
        u = device_sample(UNIFORM, self.chains, [0.0, 1.0], self.device, self.seed).to(self.x.device)
        acc = torch.log(u) < (self.logp(prop) - self.logp(self.x))
        self.x = torch.where(acc, prop, self.x)
        self.accepted += int(acc.sum())
        self.proposed += self.chains
        return self.x

    @property
    def acceptance_rate(self) -> float:
        return self.accepted / max(self.proposed, 1)


class SpikeyDataSampler(Sampler):
    """Normal baseline with occasional spikes (outlier generator)."""

    def __init__(self, mean, sd, spike_prob: float, spike_size: float):
        self.mean, self.sd, self.p, self.size = float(mean), float(sd), float(spike_prob), float(spike_size)

    def sample_n(self, n):
        v = device_sample(NORMAL, n, [self.mean, self.sd], self.device, self.seed)
        s = device_sample(BERNOULLI, n, [self.p], self.device, self.seed).to(v.device)
        return v + s * self.size


def create_sampler(spec: str) -> Sampler:
    """Parse a reference sampler spec ``v1:v2:...:type:dtype`` (sampler.py:863)."""
    items = spec.split(":")
    dtype, stype = items[-1], items[-2]
    vals = items[:-2]
    if stype == "uniform":
        if dtype == "int":
            return UniformNumericSampler(int(vals[0]), int(vals[1]))
        if dtype == "float":
            return UniformNumericSampler(float(vals[0]), float(vals[1]))
        return UniformCategoricalSampler(vals)
    if stype == "normal":
        s = NormalSampler(float(vals[0]), float(vals[1]))
        return s.sampleAsInt() if dtype == "int" else s
    if stype == "nonparam":
        return NonParamRejectSampler(float(vals[0]), float(vals[1]), [float(x) for x in vals[2:]])
    if stype == "discrete":
        return DiscreteRejectSampler(int(vals[0]), int(vals[1]), int(vals[2]), [float(x) for x in vals[3:]])
    if stype == "categorical":
        return CategoricalRejectSampler({vals[i]: float(vals[i + 1]) for i in range(0, len(vals), 2)})
    if stype == "exponential":
        return ExponentialSampler(float(vals[0]))
    if stype == "lognormal":
        return LogNormalSampler(float(vals[0]), float(vals[1]))
    if stype == "gamma":
        return GammaSampler(float(vals[0]), float(vals[1]))
    if stype == "poisson":
        return PoissonSampler(float(vals[0]))
    if stype == "pareto":
        return ParetoSampler(float(vals[0]), float(vals[1]))
    if stype == "triangular":
        return TriangularRejectSampler(float(vals[0]), float(vals[1]), float(vals[2]))
    if stype == "bernoulli":
        return BernoulliTrialSampler(float(vals[0]))
    raise ValueError(f"unknown sampler type {stype}")
