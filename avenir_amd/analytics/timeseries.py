"""Synthetic time-series generation (``tsgen.py``, P/app/tsgen.py:34-499).

Operations (reference op names): ``rg`` random gaussian-ish values from a sampler, ``rnp`` random
non-parametric, ``gen`` base + trend + year/week/day cycles + noise, ``rw`` random walk, ``ar``
autoregressive, ``sine`` sum of sines + noise, ``corr`` lagged linear copy of another series +
noise, ``ccorr`` piecewise cross-correlated, ``aol`` inject outliers.  Every generator produces
the whole series (or a batch of ``B`` series) as device tensors in one shot — AR uses a short
recursion over time but vectorised over series; sines/cycles are closed form.
"""
from __future__ import annotations

import math
from typing import Sequence

import torch

DAY, WEEK, YEAR = 86400, 7 * 86400, 365 * 86400


class TimeSeriesGenerator:
    def __init__(self, n: int, interval_s: float = 60.0, start_epoch: float = 1_600_000_000, series: int = 1,
                 seed: int = 0, device="cpu"):
        self.n, self.dt, self.t0, self.B = n, interval_s, start_epoch, series
        self.device = torch.device(device)
        self.g = torch.Generator(device=self.device).manual_seed(seed)

    @property
    def times(self) -> torch.Tensor:
        return self.t0 + self.dt * torch.arange(self.n, dtype=torch.float64, device=self.device)

    def _noise(self, sd: float):
        return sd * torch.randn((self.B, self.n), dtype=torch.float64, device=self.device, generator=self.g)

    def rg(self, mean: float = 0.0, sd: float = 1.0):
        return mean + self._noise(sd)

    def rnp(self, lo: float, bin_width: float, weights: Sequence[float]):
        w = torch.tensor(weights, dtype=torch.float64, device=self.device)
        k = torch.multinomial(w / w.sum(), self.B * self.n, replacement=True, generator=self.g).view(self.B, self.n)
        u = torch.rand((self.B, self.n), dtype=torch.float64, device=self.device, generator=self.g)
        return lo + (k + u) * bin_width

    def gen(self, base: float = 0.0, trend: float = 0.0, year: Sequence[float] = (), week: Sequence[float] = (),
            day: Sequence[float] = (), noise_sd: float = 0.0, trend_type: str = "linear"):
        """base + trend * step (or quadratic) + seasonal cycles + gaussian noise.  Cycle parameters
        are amplitude lists evaluated as sum_k a_k sin(2 pi (k+1) t / period)."""
        t = self.times - self.t0
        s = torch.full((self.n,), base, dtype=torch.float64, device=self.device)
        step = torch.arange(self.n, dtype=torch.float64, device=self.device)
        s = s + (trend * step if trend_type == "linear" else trend * step * step)
        for amps, period in ((year, YEAR), (week, WEEK), (day, DAY)):
            for k, a in enumerate(amps):
                s = s + a * torch.sin(2 * math.pi * (k + 1) * t / period)
        return s.view(1, -1) + (self._noise(noise_sd) if noise_sd else 0.0)

    def rw(self, init: float = 5.0, step_range: float = 1.0):
        steps = (torch.rand((self.B, self.n), dtype=torch.float64, device=self.device, generator=self.g) - 0.5) \
            * 2 * step_range
        steps[:, 0] = 0
        return init + torch.cumsum(steps, 1)

    def ar(self, coeffs: Sequence[float], noise_sd: float = 1.0, mean: float = 0.0):
        p = len(coeffs)
        c = torch.tensor(coeffs, dtype=torch.float64, device=self.device)
        x = torch.zeros((self.B, self.n + p), dtype=torch.float64, device=self.device)
        e = self._noise(noise_sd)
        for t in range(self.n):
            x[:, t + p] = (x[:, t:t + p].flip(1) * c).sum(1) + e[:, t]
        return mean + x[:, p:]

    def sine(self, comps: Sequence[tuple[float, float, float]], noise_sd: float = 0.0):
        """comps = (amplitude, period seconds, phase radians)."""
        t = self.times - self.t0
        s = torch.zeros(self.n, dtype=torch.float64, device=self.device)
        for a, per, ph in comps:
            s = s + a * torch.sin(2 * math.pi * t / per + ph)
        return s.view(1, -1) + (self._noise(noise_sd) if noise_sd else 0.0)

    def corr(self, other: torch.Tensor, scale: float = 1.0, noise_sd: float = 0.1, lag: int = 0):
        o = torch.as_tensor(other, dtype=torch.float64, device=self.device).view(-1, self.n)
        shifted = torch.roll(o, lag, 1)
        if lag > 0:
            shifted[:, :lag] = o[:, :1]
        return scale * shifted + self._noise(noise_sd)

    def ccorr(self, other: torch.Tensor, co_params: tuple[float, float], unco_params: tuple[float, float],
              period: int = 50):
        """Alternate correlated (scale, noise) and uncorrelated (mean, sd) stretches of ``period``."""
        o = torch.as_tensor(other, dtype=torch.float64, device=self.device).view(-1, self.n)
        co = co_params[0] * o + self._noise(co_params[1])
        un = unco_params[0] + self._noise(unco_params[1])
        seg = (torch.arange(self.n, device=self.device) // period) % 2 == 0
        return torch.where(seg.view(1, -1), co, un)

    def aol(self, series: torch.Tensor, percent: float = 5.0, mean: float = 0.0, sd: float = 5.0):
        """Add outliers to ``percent`` % of the points; returns (series, outlier mask)."""
        s = torch.as_tensor(series, dtype=torch.float64, device=self.device).clone().view(-1, self.n)
        m = torch.rand(s.shape, device=self.device, generator=self.g) < percent / 100.0
        sign = torch.where(torch.rand(s.shape, device=self.device, generator=self.g) < 0.5, -1.0, 1.0)
        s = torch.where(m, s + sign.double() * (mean + sd * torch.randn(s.shape, dtype=torch.float64,
                                                                         device=self.device, generator=self.g).abs()
                                                 + 3 * s.std()), s)
        return s, m

    def to_lines(self, series: torch.Tensor, precision: int = 3, time_format: str = "epoch", delim: str = ","):
        ts = self.times.tolist()
        out = []
        for b in range(series.shape[0]):
            for t, v in zip(ts, series[b].tolist()):
                out.append(f"{int(t)}{delim}{v:.{precision}f}")
        return out
