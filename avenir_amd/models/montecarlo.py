"""Batched Monte-Carlo simulator and MCMC convergence diagnostics.

Reference: ``python/mlextra/mcsim.py`` — register samplers, then ``run()`` loops ``numIter``
iterations calling every sampler and a user callback per iteration; statistics: sum, mean, sd,
median, min/max, integral over bounds, tail statistics, percentile, critical values;
``python/lib/mcconverge.py`` — Geweke z-score and Raftery-Lewis.

MI355X: all ``numIter`` samples of every variable are drawn in one K21 launch each ([numIter, nVars]
on device), the callback is a VECTORISED function of that batch (torch ops on device; a scalar
per-iteration callback is still accepted and looped on the host), and iterations shard across
ranks by Philox offset with one all-gather of the outputs for the order statistics.
"""
from __future__ import annotations

import math
from typing import Callable

import torch

from ..ops import samplers as S
from ..parallel.comm import Comm, get_comm


class MonteCarloSimulator:
    def __init__(self, num_iter: int, callback: Callable, device="cpu", seed: int = 0, vectorized: bool = True,
                 comm: Comm | None = None):
        self.num_iter = num_iter
        self.callback = callback
        self.device = torch.device(device)
        self.seed = seed
        self.vectorized = vectorized
        self.samplers: list[S.Sampler] = []
        self.extra_args: list = []
        self.comm = comm
        self.output: torch.Tensor | None = None

    # -- registration (reference names) -----------------------------------------------------------
    def register(self, sampler: S.Sampler) -> "MonteCarloSimulator":
        self.samplers.append(sampler)
        return self

    def registerBernoulliTrialSampler(self, pr):
        return self.register(S.BernoulliTrialSampler(pr))

    def registerPoissonSampler(self, rate, max_samp=None):
        return self.register(S.PoissonSampler(rate))

    def registerUniformSampler(self, lo, hi):
        return self.register(S.UniformNumericSampler(lo, hi))

    def registerTriangularSampler(self, lo, hi, vertex):
        return self.register(S.TriangularRejectSampler(lo, vertex, hi))

    def registerGaussianSampler(self, mean, sd):
        return self.register(S.NormalSampler(mean, sd))

    registerNormalSampler = registerGaussianSampler

    def registerLogNormalSampler(self, mean, sd):
        return self.register(S.LogNormalSampler(mean, sd))

    def registerParetoSampler(self, mode, shape):
        return self.register(S.ParetoSampler(shape, mode))

    def registerGammaSampler(self, shape, scale):
        return self.register(S.GammaSampler(shape, scale))

    def registerDiscreteRejectSampler(self, xmin, xmax, step, *values):
        return self.register(S.DiscreteRejectSampler(xmin, xmax, step, values))

    def registerNonParametricSampler(self, lo, bin_width, *values):
        return self.register(S.NonParamRejectSampler(lo, bin_width, values))

    def registerCustomSampler(self, sampler):
        return self.register(sampler)

    def registerExtraArgs(self, *args):
        self.extra_args = list(args)
        return self

    # -- run ------------------------------------------------------------------------------------
    def _draw(self, n: int, offset: int) -> torch.Tensor:
        cols = []
        for j, s in enumerate(self.samplers):
            s.on(self.device, self.seed * 1000003 + j)
            v = s.sample_n(n)
            if not isinstance(v, torch.Tensor):
                v = torch.tensor(v, dtype=torch.float32)
            v = v.to(self.device).float()
            cols.append(v if v.dim() == 2 else v.view(-1, 1))
        return torch.cat(cols, 1)

    def run(self) -> torch.Tensor:
        comm = self.comm or get_comm()
        n_local = self.num_iter // comm.world + (1 if comm.rank < self.num_iter % comm.world else 0)
        S._stream_counter[0] = 1000 * (comm.rank + 1)   # disjoint Philox offsets per rank
        X = self._draw(n_local, 0)
        if self.vectorized:
            out = self.callback(X, *self.extra_args)
            out = torch.as_tensor(out, dtype=torch.float32, device=self.device).view(-1)
        else:
            xs = X.cpu().tolist()
            out = torch.tensor([float(self.callback(list(x) + self.extra_args + [self, i])) for i, x in enumerate(xs)])
        if comm.is_distributed:
            out = comm.all_gather_v(out.to(comm.device if comm.backend == "nccl" else "cpu"))
        self.output = out.double()
        return self.output

    # -- statistics -----------------------------------------------------------------------------
    def getSum(self):
        return float(self.output.sum())

    def getMean(self):
        return float(self.output.mean())

    def getStdDev(self):
        return float(self.output.std())

    def getMedian(self):
        return float(self.output.median())

    def getMax(self):
        return float(self.output.max())

    def getMin(self):
        return float(self.output.min())

    def getIntegral(self, bounds: float) -> float:
        """Monte-Carlo integral: mean x the volume of the sampling domain."""
        return self.getMean() * bounds

    def getPercentile(self, value: float) -> float:
        """Percent of outputs below ``value``."""
        return float((self.output < value).double().mean() * 100)

    def getLowerTailStat(self, zvalue: float) -> float:
        """Value below which ``zvalue`` percent of the outputs fall."""
        return float(torch.quantile(self.output, zvalue / 100.0))

    def getUpperTailStat(self, zvalue: float) -> float:
        return float(torch.quantile(self.output, 1 - zvalue / 100.0))

    def getCritValue(self, conf: float, lower: bool = True) -> float:
        return float(torch.quantile(self.output, (1 - conf) if lower else conf))

    def getOutput(self):
        return self.output


# ================================================================================================
# MCMC convergence (python/lib/mcconverge.py)
# ================================================================================================
def geweke_z(chain: torch.Tensor, first: float = 0.1, last: float = 0.5) -> float:
    x = chain.double().view(-1)
    n = x.numel()
    a, b = x[: int(first * n)], x[int((1 - last) * n):]
    return float((a.mean() - b.mean()) / math.sqrt(float(a.var()) / a.numel() + float(b.var()) / b.numel()))


def raftery_lewis(chain: torch.Tensor, q: float = 0.025, r: float = 0.005, s: float = 0.95) -> dict:
    """Raftery-Lewis run-length diagnostic on the indicator chain x <= quantile(q)."""
    x = chain.double().view(-1)
    thr = torch.quantile(x, q)
    z = (x <= thr).long()
    trans = torch.zeros((2, 2), dtype=torch.float64)
    for a, b in zip(z[:-1].tolist(), z[1:].tolist()):
        trans[a, b] += 1
    alpha = float(trans[0, 1] / trans[0].sum().clamp_min(1))
    beta = float(trans[1, 0] / trans[1].sum().clamp_min(1))
    from math import erf, log, sqrt
    phi = sqrt(2) * _erfinv((s + 1) / 2 * 2 - 1)
    if alpha + beta == 0:
        return {"burn_in": 0, "n_min": len(x), "dependence": 1.0}
    m = int(math.ceil(log((0.001 * (alpha + beta)) / max(alpha, beta)) / log(abs(1 - alpha - beta)))) if abs(1 - alpha - beta) > 0 else 0
    n = int(math.ceil((2 - alpha - beta) * alpha * beta * phi * phi / ((alpha + beta) ** 3 * r * r)))
    nmin = int(math.ceil(q * (1 - q) * phi * phi / (r * r)))
    return {"burn_in": max(m, 0), "n": n, "n_min": nmin, "dependence": (n + max(m, 0)) / max(nmin, 1)}


def _erfinv(y: float) -> float:
    return float(torch.erfinv(torch.tensor(y, dtype=torch.float64)))
