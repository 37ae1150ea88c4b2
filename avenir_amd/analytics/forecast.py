"""Additive time-series forecaster with changepoints, seasonality and holidays.

Reference: ``ProphetForcaster`` (P/unsupv/profo.py:35-286) wraps fbprophet (piecewise-linear trend
with changepoints, Fourier seasonalities, holiday effects; train / validate / save / forecast).
fbprophet is not available, so this is a compact re-implementation of the same additive model
solved as ONE regularised least-squares problem on the device (MAP estimate with a Laplace-like
L1 prior on changepoint deltas approximated by ridge):

    y(t) = k t + m + sum_j delta_j (t - s_j)_+ + sum_seasons Fourier(t) + sum_h beta_h 1[t in h]

Uncertainty intervals (``train.uncertainty.samples``, ``train.interval.width``,
``train.mcmc.samples`` of P/unsupv/profo.py:58-60), drawn as fbprophet does, all samples as one
device batch:
* future trend: every future time point is a new changepoint with the history's changepoint rate,
  its rate change ~ Laplace(0, mean |delta_j|) (fbprophet's ``sample_predictive_trend``);
* observation noise ~ N(0, sigma) (the residual scale);
* with ``mcmc_samples`` > 0 also parameter uncertainty: the coefficients are drawn from the EXACT
  Gaussian posterior of this linear-Gaussian model, N(beta_MAP, (X'X / s^2 + Lambda)^-1), which is
  what an MCMC chain over it converges to (fbprophet runs Stan's NUTS because its Laplace
  changepoint prior is not conjugate; the ridge prior here is).
``yhat_lower`` / ``yhat_upper`` are the sample quantiles at (1 -/+ width) / 2.

``seasonality_mode="multiplicative"`` (``train.seasonality.mode``, P/unsupv/profo.py:54,276): the
seasonal and holiday terms scale the trend, y = trend(t) (1 + X_s(t) beta_s), fitted by
alternating ridge solves that are each exact given the other block — trend given the seasonal
factor (its columns weighted by 1 + X_s beta_s), seasonal given the trend (its columns weighted by
the trend) — until the relative change is below 1e-10.  Holiday effects get their own prior
(``holidays_prior``, ``train.holidays.prior.scale``; fbprophet's ``holidays_prior_scale``).

Forecast parity with fbprophet is unpinned.  Save/load use the framework container format.
"""
from __future__ import annotations

import math
from typing import Sequence

import torch

DAY = 86400.0


class AdditiveForecaster:
    def __init__(self, n_changepoints: int = 25, changepoint_range: float = 0.8, changepoint_prior: float = 0.05,
                 yearly: int = 10, weekly: int = 3, daily: int = 0, seasonality_prior: float = 10.0,
                 holidays: dict[str, Sequence[float]] | None = None, holiday_window_s: float = DAY, device="cpu",
                 interval_width: float = 0.8, uncertainty_samples: int = 1000, mcmc_samples: int = 0, seed: int = 0,
                 seasonality_mode: str = "additive", holidays_prior: float | None = None):
        if seasonality_mode not in ("additive", "multiplicative"):
            raise ValueError(f"seasonality mode {seasonality_mode!r}: additive or multiplicative")
        self.ncp, self.cpr, self.cp_prior = n_changepoints, changepoint_range, changepoint_prior
        self.seas = [(365.25 * DAY, yearly), (7 * DAY, weekly), (DAY, daily)]
        self.s_prior = seasonality_prior
        self.h_prior = float(holidays_prior) if holidays_prior is not None else float(seasonality_prior)
        self.mode = seasonality_mode
        self.holidays = {k: list(v) for k, v in (holidays or {}).items()}
        self.hw = holiday_window_s
        self.device = torch.device(device)
        self.interval_width, self.unc_samples, self.mcmc = float(interval_width), int(uncertainty_samples), int(mcmc_samples)
        self.seed = int(seed)
        self.cov = None

    def _design(self, t: torch.Tensor) -> torch.Tensor:
        ts = (t - self.t0) / self.scale_t                       # scaled time in [0, 1] over training
        cols = [ts, torch.ones_like(ts)]
        for s in self.cps:
            cols.append((ts - s).clamp_min(0))
        for period, order in self.seas:
            for k in range(1, order + 1):
                ang = 2 * math.pi * k * t / period
                cols += [torch.sin(ang), torch.cos(ang)]
        for name, days in self.holidays.items():
            d = torch.tensor(days, dtype=torch.float64, device=t.device)
            cols.append(((t.view(-1, 1) - d.view(1, -1)).abs() < self.hw).any(1).double())
        return torch.stack(cols, 1)

    def fit(self, t, y) -> "AdditiveForecaster":
        t = torch.as_tensor(t, dtype=torch.float64, device=self.device)
        y = torch.as_tensor(y, dtype=torch.float64, device=self.device)
        self.t0, self.scale_t = float(t.min()), float(t.max() - t.min()) or 1.0
        self.y_scale = float(y.abs().max()) or 1.0
        self.cps = torch.linspace(0, self.cpr, self.ncp + 2, dtype=torch.float64)[1:-1].tolist() if self.ncp else []
        X = self._design(t)
        ys = y / self.y_scale
        # priors: changepoint deltas ~ N(0, cp_prior^2), seasonal ~ N(0, s_prior^2), holidays ~
        # N(0, h_prior^2)
        reg = torch.zeros(X.shape[1], dtype=torch.float64, device=self.device)
        reg[2:2 + len(self.cps)] = 1.0 / self.cp_prior ** 2
        reg[2 + len(self.cps):] = 1.0 / self.s_prior ** 2
        if self.holidays:
            reg[X.shape[1] - len(self.holidays):] = 1.0 / self.h_prior ** 2
        self.n_hist = int(t.numel())
        self.t_hist = t
        if self.mode == "multiplicative":
            return self._fit_multiplicative(X, ys, reg)
        # MAP: data term weighted by 1/sigma^2 (sigma from a weakly regularised first pass), so the
        # priors act relative to the observation noise as in the Bayesian model
        eye = 1e-9 * torch.eye(X.shape[1], dtype=torch.float64, device=self.device)
        XtX, Xty = X.T @ X, X.T @ ys
        b0 = torch.linalg.solve(XtX + 1e-6 * torch.diag(reg) + eye, Xty)
        s2 = float(((ys - X @ b0) ** 2).mean()) + 1e-12
        prec = XtX / s2 + torch.diag(reg) + eye
        self.beta = torch.linalg.solve(prec, Xty / s2)
        self.cov = torch.linalg.inv(prec)                     # exact posterior covariance (scaled units)
        self.cov = 0.5 * (self.cov + self.cov.T)
        resid = ys - X @ self.beta
        self.sigma = float(resid.std()) * self.y_scale
        return self

    def _fit_multiplicative(self, X: torch.Tensor, ys: torch.Tensor, reg: torch.Tensor,
                            max_iter: int = 200, tol: float = 1e-10) -> "AdditiveForecaster":
        """y = (X_t b_t) (1 + X_s b_s): alternating exact ridge solves of the two blocks; the noise
        scale of the MAP weighting is re-estimated each round.  beta = [b_t | b_s] (the design's
        column order), cov = the block-diagonal of the two conditional posteriors."""
        nt = 2 + len(self.cps)
        Xt, Xs = X[:, :nt], X[:, nt:]
        rt, rs = reg[:nt], reg[nt:]
        f64 = dict(dtype=torch.float64, device=self.device)
        eye_t, eye_s = 1e-9 * torch.eye(nt, **f64), 1e-9 * torch.eye(Xs.shape[1], **f64)
        bs = torch.zeros(Xs.shape[1], **f64)
        bt = torch.linalg.solve(Xt.T @ Xt + 1e-6 * torch.diag(rt) + eye_t, Xt.T @ ys)
        s2 = float(((ys - Xt @ bt) ** 2).mean()) + 1e-12
        prev = None
        for _ in range(max_iter):
            fac = 1.0 + Xs @ bs                                          # seasonal factor
            A = Xt * fac.view(-1, 1)
            pt = A.T @ A / s2 + torch.diag(rt) + eye_t
            bt = torch.linalg.solve(pt, A.T @ ys / s2)
            tr = Xt @ bt
            B = Xs * tr.view(-1, 1)
            ps = B.T @ B / s2 + torch.diag(rs) + eye_s
            bs = torch.linalg.solve(ps, B.T @ (ys - tr) / s2)
            fit = tr * (1.0 + Xs @ bs)
            s2 = float(((ys - fit) ** 2).mean()) + 1e-12
            cur = torch.cat([bt, bs])
            if prev is not None and float((cur - prev).norm()) <= tol * (1.0 + float(cur.norm())):
                break
            prev = cur
        self.beta = torch.cat([bt, bs])
        cov = torch.zeros((X.shape[1], X.shape[1]), **f64)
        cov[:nt, :nt] = torch.linalg.inv(pt)
        cov[nt:, nt:] = torch.linalg.inv(ps)
        self.cov = 0.5 * (cov + cov.T)
        self.sigma = float((ys - fit).std()) * self.y_scale
        return self

    def _combine(self, X: torch.Tensor, beta: torch.Tensor) -> torch.Tensor:
        """Model output in scaled units for coefficient rows beta [S, P] (or [P]) -> [S, T] / [T]."""
        nt = 2 + len(self.cps)
        tr = beta[..., :nt] @ X[:, :nt].T
        se = beta[..., nt:] @ X[:, nt:].T
        return tr * (1.0 + se) if self.mode == "multiplicative" else tr + se

    def history_times(self) -> torch.Tensor:
        return self.t_hist if getattr(self, "t_hist", None) is not None else torch.empty(0, dtype=torch.float64)

    def predict(self, t) -> dict[str, torch.Tensor]:
        t = torch.as_tensor(t, dtype=torch.float64, device=self.device)
        X = self._design(t)
        yhat = self._combine(X, self.beta) * self.y_scale
        nt = 2 + len(self.cps)
        trend = (X[:, :nt] @ self.beta[:nt]) * self.y_scale
        lo, hi = self._intervals(t, X, yhat)
        return {"yhat": yhat, "trend": trend, "seasonal": yhat - trend, "yhat_lower": lo, "yhat_upper": hi}

    def _intervals(self, t: torch.Tensor, X: torch.Tensor, yhat: torch.Tensor):
        S = self.unc_samples
        if S <= 0 or t.numel() == 0:
            return yhat.clone(), yhat.clone()
        g = torch.Generator(device=self.device).manual_seed(self.seed)
        f64 = dict(dtype=torch.float64, device=self.device)
        if self.mcmc > 0 and self.cov is not None:            # parameter draws from the posterior
            L = torch.linalg.cholesky(self.cov + 1e-12 * torch.eye(self.cov.shape[0], **f64))
            B = self.beta.view(1, -1) + torch.randn((S, self.beta.numel()), generator=g, **f64) @ L.T
            ys = self._combine(X, B) * self.y_scale                              # [S, T]
        else:
            ys = yhat.view(1, -1).expand(S, -1).clone()
        # future trend changepoints (scaled time > 1): rate p per future point, Laplace deltas
        ts = (t - self.t0) / self.scale_t
        fut = ts > 1.0
        if bool(fut.any()) and self.cps:
            deltas = self.beta[2:2 + len(self.cps)]
            lam = float(deltas.abs().mean()) + 1e-8
            p = len(self.cps) / max(1, getattr(self, "n_hist", len(self.cps) * 10))
            tf = ts[fut]
            z = (torch.rand((S, tf.numel()), generator=g, **f64) < p).double()
            u = torch.rand((S, tf.numel()), generator=g, **f64) - 0.5
            lap = -lam * torch.sign(u) * torch.log1p(-2 * u.abs())                # Laplace(0, lam)
            zd = z * lap
            add = tf.view(1, -1) * zd.cumsum(1) - (zd * tf.view(1, -1)).cumsum(1)  # sum_j d_j (t - s_j)
            ys[:, fut] = ys[:, fut] + add * self.y_scale
        ys = ys + self.sigma * torch.randn(ys.shape, generator=g, **f64)
        w = self.interval_width
        q = torch.tensor([(1 - w) / 2, (1 + w) / 2], **f64)
        qs = torch.quantile(ys, q, dim=0)
        return qs[0], qs[1]

    def future_times(self, periods: int, freq_s: float = DAY, last: float | None = None) -> torch.Tensor:
        start = last if last is not None else self.t0 + self.scale_t
        return start + freq_s * torch.arange(1, periods + 1, dtype=torch.float64, device=self.device)

    def validate(self, t, y) -> dict[str, float]:
        p = self.predict(t)["yhat"]
        y = torch.as_tensor(y, dtype=torch.float64, device=self.device)
        e = p - y
        return {"rmse": float((e * e).mean().sqrt()), "mae": float(e.abs().mean()),
                "mape": float((e.abs() / y.abs().clamp_min(1e-12)).mean() * 100)}

    def save(self, path):
        from ..utils import checkpoint as C
        C.save(path, {"beta": self.beta, "cov": self.cov, "t_hist": self.t_hist},
               {"t0": self.t0, "scale_t": self.scale_t, "y_scale": self.y_scale, "cps": self.cps, "sigma": self.sigma,
                "seas": self.seas, "holidays": self.holidays, "hw": self.hw, "n_hist": self.n_hist,
                "interval_width": self.interval_width, "unc_samples": self.unc_samples, "mcmc": self.mcmc,
                "seed": self.seed, "mode": self.mode, "s_prior": self.s_prior, "h_prior": self.h_prior})

    @classmethod
    def load(cls, path, device="cpu"):
        from ..utils import checkpoint as C
        t, m = C.load(path, device)
        f = cls(device=device)
        f.beta = t["beta"].double()
        f.t0, f.scale_t, f.y_scale, f.cps, f.sigma = m["t0"], m["scale_t"], m["y_scale"], m["cps"], m["sigma"]
        f.seas = [tuple(s) for s in m["seas"]]
        f.holidays, f.hw = m["holidays"], m["hw"]
        f.cov = t["cov"].double() if "cov" in t else None
        f.t_hist = t["t_hist"].double() if "t_hist" in t else None
        f.n_hist = int(m.get("n_hist", 0))
        f.interval_width, f.unc_samples = float(m.get("interval_width", 0.8)), int(m.get("unc_samples", 1000))
        f.mcmc, f.seed = int(m.get("mcmc", 0)), int(m.get("seed", 0))
        f.mode = m.get("mode", "additive")
        f.s_prior = float(m.get("s_prior", f.s_prior))
        f.h_prior = float(m.get("h_prior", f.s_prior))
        return f
