"""Linear models: logistic regression, linear / ridge / elastic-net regression, linear SVM (hinge),
Fisher univariate discriminant.

Reference:
* ``LogisticRegressionJob`` / ``LogisticRegressor`` (J/regress/LogisticRegressionJob.java:60-289,
  J/regress/LogisticRegressor.java:61-163): iterative batch gradient, one MR job per iteration, a
  coefficient file that gains one line per iteration, convergence by iteration limit /
  all-coefficients %-change / average %-change.  Reference bug: the reducer stores the summed
  gradient AS the new coefficients (:220-231); here the update is ``w + lr * g / n`` (or a Newton
  step), and the coefficient history keeps the reference's one-line-per-iteration format.
* ``LogisticRegressionDiscriminant`` (P/supv/lrd.py), ``LinearRegressor`` / ``ElasticNetRegressor``
  (P/supv/regress.py:38-253).
* ``FisherDiscriminant`` (J/discriminant/FisherDiscriminant.java:83-117): per attribute, pooled
  variance of the two class-conditional distributions, log prior odds and the decision boundary
  ``(m0 + m1) / 2 - logOdds * pooledVar / (m0 - m1)``.

MI355X design: features live column-major ``[D, ld]`` (the framework's SoA layout), padded to
D in {4, 8, 16, 32}; the K13 kernel produces gradient + loss (+ per-row curvature) in ONE pass over
HBM; Newton/IRLS Hessians and regression Gram matrices are one hipBLASLt GEMM; data parallelism is
one all-reduce of a [D+1] (or [D, D]) buffer per iteration.
"""
from __future__ import annotations

import math
from pathlib import Path
from typing import Sequence

import torch

from .. import _native
from ..parallel.comm import Comm, get_comm
from ..utils.resilience import IterationLoop, RecoveryConfig

MODE_LOGISTIC, MODE_SQUARED, MODE_HINGE = 0, 1, 2


def _pad_d(d: int) -> int:
    for p in (4, 8, 16, 32):
        if d <= p:
            return p
    return d


class DenseSoA:
    """Column-major padded design matrix: X [Dp, ld] (row 0 = 1 when ``intercept``), n rows."""

    def __init__(self, X: torch.Tensor, intercept: bool = True, device=None):
        X = torch.as_tensor(X)
        dev = torch.device(device) if device is not None else X.device
        n, d = X.shape
        self.n, self.d_in, self.intercept = n, d, intercept
        D = d + (1 if intercept else 0)
        self.D = D
        self.Dp = _pad_d(D)
        self.ld = max(16, ((n + 15) // 16) * 16)
        xs = torch.zeros((self.Dp, self.ld), dtype=torch.float32, device=dev)
        o = 0
        if intercept:
            xs[0, :n] = 1.0
            o = 1
        xs[o:o + d, :n] = X.to(dev, torch.float32).T
        self.X = xs

    @property
    def device(self):
        return self.X.device

    def vec(self, v: torch.Tensor) -> torch.Tensor:
        """Row vector padded to ld (float32, device)."""
        out = torch.zeros((self.ld,), dtype=torch.float32, device=self.device)
        out[: self.n] = torch.as_tensor(v, device=self.device).float().view(-1)[: self.n]
        return out

    def rows(self) -> torch.Tensor:
        return self.X[: self.D, : self.n].T


def glm_gradient(data: DenseSoA, y: torch.Tensor, w: torch.Tensor, mode: int, sw: torch.Tensor | None = None,
                 want_h: bool = False):
    """(g [Dp] f64 = sum sw*x*e, loss f64, h [n] or None) — K13 on GPU, fp64 torch on CPU."""
    wp = torch.zeros((data.Dp,), dtype=torch.float32, device=data.device)
    wp[: w.numel()] = w.to(data.device, torch.float32)
    if data.device.type == "cuda" and data.Dp <= 256:      # K13 (tiled through LDS above 32)
        hw = torch.empty((max(data.n, 1),), dtype=torch.float32, device=data.device) if want_h else None
        out = _native.C().glm_gradient(data.X, data.n, y, sw, wp, int(mode), hw)
        return out[:-1], out[-1], (hw[: data.n] if want_h else None)
    X = data.X[:, : data.n].double()
    z = wp.double() @ X
    yy = y[: data.n].double()
    s = sw[: data.n].double() if sw is not None else torch.ones_like(yy)
    if mode == MODE_LOGISTIC:
        p = torch.sigmoid(z)
        e, l, h = yy - p, torch.nn.functional.softplus(z) - yy * z, p * (1 - p)
    elif mode == MODE_SQUARED:
        e = yy - z
        l, h = 0.5 * e * e, torch.ones_like(z)
    else:
        m = yy * z
        e = torch.where(m < 1, yy, torch.zeros_like(yy))
        l, h = (1 - m).clamp_min(0), torch.zeros_like(z)
    g = X @ (e * s)
    return g, (l * s).sum(), ((h * s).float() if want_h else None)


def _converged(prev: torch.Tensor, cur: torch.Tensor, criteria: str, threshold: float) -> bool:
    """LogisticRegressor.isAllConverged / isAverageConverged (% change per coefficient)."""
    diff = ((cur - prev) * 100.0 / prev.where(prev != 0, torch.full_like(prev, 1e-12))).abs()
    if criteria == "allBelowThreshold":
        return bool((diff <= threshold).all())
    if criteria == "averageBelowThreshold":
        return float(diff.mean()) <= threshold
    return False


class LogisticRegression:
    def __init__(self, solver: str = "newton", lr: float = 1.0, max_iter: int = 25, l2: float = 0.0,
                 intercept: bool = True, criteria: str = "averageBelowThreshold", threshold: float = 0.01,
                 tol: float = 1e-8, comm: Comm | None = None, recovery: RecoveryConfig | None = None):
        self.solver, self.lr, self.max_iter, self.l2 = solver, lr, max_iter, l2
        self.recovery = recovery
        self.intercept, self.criteria, self.threshold, self.tol = intercept, criteria, threshold, tol
        self.comm = comm
        self.coef: torch.Tensor | None = None
        self.history: list[list[float]] = []
        self.losses: list[float] = []

    def fit(self, X, y, sample_weight=None, pos_class=1) -> "LogisticRegression":
        comm = self.comm or get_comm()
        data = X if isinstance(X, DenseSoA) else DenseSoA(X, self.intercept)
        yy = data.vec((torch.as_tensor(y) == pos_class).float())
        sw = data.vec(sample_weight) if sample_weight is not None else None
        D = data.D
        n_tot = torch.tensor([float(data.n) if sw is None else float(sw.sum())], dtype=torch.float64, device=data.device)
        n_tot = float(comm.all_reduce(n_tot)) if comm.is_distributed else float(n_tot)
        w = torch.zeros((D,), dtype=torch.float64, device=data.device) if self.coef is None else self.coef.double().clone()
        self.history = [w.tolist()]
        lp = IterationLoop("logistic", self.recovery, comm, device=data.device)
        it0, st, _ = lp.restore(data.device)
        if st is not None:       # the coefficient history is the reference's per-iteration state file
            self.history = st["history"].tolist()
            self.losses = st["losses"].tolist()
            w = st["history"][-1].to(data.device)
            if bool(st["done"]):
                it0 = self.max_iter
        for it in range(it0, self.max_iter):
            with lp.step(it, nbytes=float(data.X.numel() * 4)):
                w, stop = self._iterate(data, yy, sw, w, D, n_tot, comm)
            if lp.enabled:
                lp.commit(it, {"history": torch.tensor(self.history, dtype=torch.float64),
                               "losses": torch.tensor(self.losses, dtype=torch.float64),
                               "done": torch.tensor(stop)})
            if stop:
                break
        lp.close()
        self.coef = w
        return self

    def _iterate(self, data, yy, sw, w, D, n_tot, comm):
        """One gradient / Newton iteration -> (new weights, converged)."""
        g, loss, h = glm_gradient(data, yy, w.float(), MODE_LOGISTIC, sw, want_h=self.solver == "newton")
        g = g[:D].double().clone()
        buf = torch.cat([g, loss.view(1).double()])
        if self.solver == "newton":
            if data.device.type == "cuda" and D <= 1024:
                H = _native.C().weighted_gram(data.X, data.n, D, h.contiguous())   # MFMA Gram (32x32 blocks)
            else:
                Xr = data.X[:D, : data.n]
                H = (Xr * h.view(1, -1)) @ Xr.T                               # [D, D] GEMM
            buf = torch.cat([buf, H.double().reshape(-1)])
        if comm.is_distributed:
            buf = comm.all_reduce(buf)
        g, loss = buf[:D], float(buf[D])
        if self.l2:
            g = g - self.l2 * w * n_tot
            loss += 0.5 * self.l2 * n_tot * float((w * w).sum())
        self.losses.append(loss / n_tot)
        prev = w.clone()
        if self.solver == "newton":
            H = buf[D + 1:].view(D, D) + (self.l2 * n_tot + 1e-9 * n_tot) * torch.eye(D, dtype=torch.float64, device=w.device)
            w = w + torch.linalg.solve(H, g)
        else:
            w = w + self.lr * g / n_tot
        self.history.append(w.tolist())
        if float(g.abs().max()) / n_tot < self.tol:
            return w, True
        if self.criteria != "iterLimit" and _converged(prev, w, self.criteria, self.threshold):
            return w, True
        return w, False

    def decision_function(self, X) -> torch.Tensor:
        data = X if isinstance(X, DenseSoA) else DenseSoA(X, self.intercept, device=self.coef.device)
        return (self.coef.float().to(data.device) @ data.X[: data.D, : data.n])

    def predict_proba(self, X) -> torch.Tensor:
        p = torch.sigmoid(self.decision_function(X))
        return torch.stack([1 - p, p], 1)

    def predict(self, X, threshold: float = 0.5) -> torch.Tensor:
        return (self.predict_proba(X)[:, 1] >= threshold).long()

    # -- coefficient file (one line per iteration, J/regress/LogisticRegressionJob.java:233-255) --
    def coefficient_lines(self, delim: str = ",") -> list[str]:
        return [delim.join(repr(float(c)) for c in row) for row in self.history]

    def save_coefficients(self, path, delim: str = ","):
        Path(path).write_text("\n".join(self.coefficient_lines(delim)) + "\n")

    @classmethod
    def load_coefficients(cls, path, delim: str = ",", **kw) -> "LogisticRegression":
        lines = [l for l in Path(path).read_text().splitlines() if l.strip()]
        m = cls(**kw)
        m.history = [[float(x) for x in l.split(delim)] for l in lines]
        m.coef = torch.tensor(m.history[-1], dtype=torch.float64)
        return m


# ================================================================================================
# regression from sufficient statistics
# ================================================================================================
def gram(X, y, intercept: bool = True, comm: Comm | None = None):
    """Sufficient statistics of least squares: A = [X 1]^T [X 1], b = [X 1]^T y, yy, n — one GEMM,
    fp32 inputs accumulated in fp64, all-reduced across ranks."""
    comm = comm or get_comm()
    X = torch.as_tensor(X).double()
    if intercept:
        X = torch.cat([torch.ones((X.shape[0], 1), dtype=X.dtype, device=X.device), X], 1)
    y = torch.as_tensor(y, device=X.device).double().view(-1)
    D = X.shape[1]
    buf = torch.cat([(X.T @ X).reshape(-1), X.T @ y, (y @ y).view(1),
                     torch.tensor([float(X.shape[0])], dtype=torch.float64, device=X.device)])
    if comm.is_distributed:
        buf = comm.all_reduce(buf)
    return buf[: D * D].view(D, D), buf[D * D: D * D + D], float(buf[-2]), float(buf[-1])


class LinearRegression:
    """OLS / ridge by normal equations (Cholesky) on the all-reduced Gram matrix."""

    def __init__(self, alpha: float = 0.0, intercept: bool = True, comm: Comm | None = None):
        self.alpha, self.intercept, self.comm = alpha, intercept, comm
        self.coef = None

    def fit(self, X, y) -> "LinearRegression":
        A, b, _, n = gram(X, y, self.intercept, self.comm)
        D = A.shape[0]
        reg = self.alpha * torch.eye(D, dtype=A.dtype, device=A.device)
        if self.intercept:
            reg[0, 0] = 0.0
        self.coef = torch.linalg.solve(A + reg + 1e-12 * torch.eye(D, dtype=A.dtype, device=A.device), b)
        return self

    def predict(self, X) -> torch.Tensor:
        X = torch.as_tensor(X).double().to(self.coef.device)
        return (X @ self.coef[1:] + self.coef[0]) if self.intercept else X @ self.coef

    def score(self, X, y) -> float:
        y = torch.as_tensor(y).double().to(self.coef.device)
        r = y - self.predict(X)
        return 1.0 - float((r @ r) / ((y - y.mean()) @ (y - y.mean())).clamp_min(1e-300))


class ElasticNet(LinearRegression):
    """Elastic net (sklearn objective 1/(2n)||y - Xw||^2 + a*l1*|w|_1 + a*(1-l1)/2*||w||^2) by
    cyclic coordinate descent with covariance updates on the Gram matrix — O(D^2) per sweep after
    the single pass over the data."""

    def __init__(self, alpha: float = 1.0, l1_ratio: float = 0.5, max_iter: int = 1000, tol: float = 1e-8,
                 intercept: bool = True, comm: Comm | None = None):
        super().__init__(alpha, intercept, comm)
        self.l1_ratio, self.max_iter, self.tol = l1_ratio, max_iter, tol

    def fit(self, X, y) -> "ElasticNet":
        A, b, yy, n = gram(X, y, self.intercept, self.comm)
        A, b = A.cpu(), b.cpu()
        D = A.shape[0]
        if self.intercept:
            # centre analytically: A_c = A[1:,1:] - mx mx^T n, b_c = b[1:] - mx * sum(y)
            mx = A[0, 1:] / n
            my = b[0] / n
            Ac = A[1:, 1:] - n * torch.outer(mx, mx)
            bc = b[1:] - n * mx * my
        else:
            Ac, bc = A, b
        l1 = self.alpha * self.l1_ratio * n
        l2 = self.alpha * (1 - self.l1_ratio) * n
        w = torch.zeros(Ac.shape[0], dtype=torch.float64)
        diag = Ac.diagonal()
        for _ in range(self.max_iter):
            wmax = 0.0
            for j in range(Ac.shape[0]):
                if diag[j] <= 0:
                    continue
                rho = float(bc[j] - Ac[j] @ w + diag[j] * w[j])
                new = math.copysign(max(abs(rho) - l1, 0.0), rho) / float(diag[j] + l2)
                wmax = max(wmax, abs(new - float(w[j])))
                w[j] = new
            if wmax < self.tol:
                break
        if self.intercept:
            b0 = my - mx @ w
            self.coef = torch.cat([b0.view(1), w])
        else:
            self.coef = w
        return self


class LinearSVM:
    """Primal linear SVM: hinge loss + L2 by full-batch subgradient descent (Pegasos step size
    1/(lambda t)) using the K13 hinge mode; labels in {0,1} or {-1,+1}."""

    def __init__(self, lam: float = 1e-3, max_iter: int = 200, intercept: bool = True, comm: Comm | None = None):
        self.lam, self.max_iter, self.intercept, self.comm = lam, max_iter, intercept, comm
        self.coef = None

    def fit(self, X, y) -> "LinearSVM":
        comm = self.comm or get_comm()
        data = X if isinstance(X, DenseSoA) else DenseSoA(X, self.intercept)
        yv = torch.as_tensor(y).float()
        yv = torch.where(yv > 0, torch.ones_like(yv), -torch.ones_like(yv))
        ys = data.vec(yv)
        n = float(comm.all_reduce(torch.tensor([float(data.n)], dtype=torch.float64, device=data.device))) \
            if comm.is_distributed else float(data.n)
        w = torch.zeros(data.D, dtype=torch.float64, device=data.device)
        avg = w.clone()
        for t in range(1, self.max_iter + 1):
            g, loss, _ = glm_gradient(data, ys, w.float(), MODE_HINGE)
            g = g[: data.D].double().clone()
            if comm.is_distributed:
                g = comm.all_reduce(g)
            eta = 1.0 / (self.lam * t)
            w = (1 - eta * self.lam) * w + eta * g / n
            avg += (w - avg) / t
        self.coef = avg
        return self

    def decision_function(self, X):
        data = X if isinstance(X, DenseSoA) else DenseSoA(X, self.intercept, device=self.coef.device)
        return self.coef.float().to(data.device) @ data.X[: data.D, : data.n]

    def predict(self, X):
        return (self.decision_function(X) > 0).long()


# ================================================================================================
# Fisher univariate discriminant
# ================================================================================================
def fisher_discriminant(x: torch.Tensor, labels: torch.Tensor, comm: Comm | None = None) -> torch.Tensor:
    """Per attribute: [logOddsPrior, pooledVariance, discrimValue] from class-conditional moments of
    a binary class (class 0 = first class value seen by the reducer).  ``x`` [n, F] float; the
    moments are one fused reduction ([2, F, 3]: count, sum, sum of squares), all-reduced."""
    comm = comm or get_comm()
    x = torch.as_tensor(x).double()
    lab = torch.as_tensor(labels, device=x.device).long().view(-1)
    F = x.shape[1]
    m = torch.zeros((2, F, 3), dtype=torch.float64, device=x.device)
    for c in (0, 1):
        xc = x[lab == c]
        m[c, :, 0] = xc.shape[0]
        m[c, :, 1] = xc.sum(0)
        m[c, :, 2] = (xc * xc).sum(0)
    if comm.is_distributed:
        m = comm.all_reduce(m)
    cnt, mean = m[..., 0], m[..., 1] / m[..., 0].clamp_min(1)
    var = m[..., 2] / cnt.clamp_min(1) - mean * mean                 # population variance (chombo stats)
    pooled = (var[0] * cnt[0] + var[1] * cnt[1]) / (cnt[0] + cnt[1])
    log_odds = torch.log(cnt[0] / cnt[1])
    disc = (mean[0] + mean[1]) / 2 - log_odds * pooled / (mean[0] - mean[1])
    return torch.stack([log_odds, pooled, disc], 1)


def fisher_lines(result: torch.Tensor, delim: str = ",") -> list[str]:
    return [delim.join([str(a)] + [repr(float(v)) for v in row]) for a, row in enumerate(result.tolist())]
