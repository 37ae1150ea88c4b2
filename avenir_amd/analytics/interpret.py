"""Model interpretation: individual conditional expectation (ICE) and LIME.

Reference: ``Prescriptor.indCondExp`` (P/mlextra/presc.py:102-150: vary one feature of a record over
an int range / float grid / categorical values and predict each variant), the Spark
``IndividualConditionalExpectation`` job (S/interpret/IndividualConditionalExpectation.scala:100-219:
grid variations per record, **HTTP POST of each batch to a remote model service**), and
``LimeInterpreter`` (P/mlextra/interpret.py:37-111, the ``lime`` package around ``predictProb``).

MI355X design: all variations of all records form ONE [R * G, F] device batch and the model is
called in-process once (no HTTP hop); LIME draws the perturbation batch on the device, scores it
with one model call, and solves the kernel-weighted ridge regression as a [F, F] GEMM + solve.
"""
from __future__ import annotations

from typing import Callable, Sequence

import torch


def ice_grid(records: torch.Tensor, feature: int, values: torch.Tensor) -> torch.Tensor:
    """[R, F] records x G grid values of one feature -> [R, G, F] variants."""
    R, F = records.shape
    G = values.numel()
    v = records.unsqueeze(1).expand(R, G, F).clone()
    v[:, :, feature] = values.to(records.dtype).view(1, G)
    return v


def individual_conditional_expectation(predict: Callable, records: torch.Tensor, feature: int,
                                       ftype: str = "float", range_val: float = 1.0, num_grid: int = 20,
                                       cat_values: Sequence[float] | None = None):
    """ICE curves: (grid [R, G], predictions [R, G]).

    int: ref-range .. ref+range step 1; float: ref-range .. ref+range in ``num_grid`` steps;
    categorical: the listed values (presc.py:102-150 semantics, grid relative to each record)."""
    X = torch.as_tensor(records).float()
    R = X.shape[0]
    ref = X[:, feature]
    if ftype == "int":
        steps = torch.arange(-int(range_val), int(range_val) + 1, device=X.device).float()
        grid = ref.view(-1, 1) + steps.view(1, -1)
    elif ftype == "float":
        steps = torch.linspace(-range_val, range_val, num_grid + 1, device=X.device)
        grid = ref.view(-1, 1) + steps.view(1, -1)
    else:
        grid = torch.tensor(cat_values, dtype=torch.float32, device=X.device).view(1, -1).expand(R, -1)
    G = grid.shape[1]
    V = X.unsqueeze(1).expand(R, G, X.shape[1]).clone()
    V[:, :, feature] = grid
    out = torch.as_tensor(predict(V.view(R * G, -1)))
    return grid, out.view(R, G, *out.shape[1:])


def partial_dependence(predict: Callable, records: torch.Tensor, feature: int, values: torch.Tensor):
    """Average of the ICE curves over the records."""
    V = ice_grid(torch.as_tensor(records).float(), feature, torch.as_tensor(values).float())
    R, G, F = V.shape
    out = torch.as_tensor(predict(V.view(R * G, F))).view(R, G, -1)
    return out.mean(0)


class LimeTabular:
    """LIME for tabular models: gaussian perturbations scaled by the training std, an exponential
    kernel on the scaled distance, and a weighted ridge surrogate per explained class."""

    def __init__(self, train: torch.Tensor, feature_names: Sequence[str] | None = None, kernel_width: float | None = None,
                 categorical: Sequence[int] = (), seed: int = 0):
        X = torch.as_tensor(train).float()
        self.mean, self.std = X.mean(0), X.std(0).clamp_min(1e-12)
        self.F = X.shape[1]
        self.names = list(feature_names) if feature_names else [f"f{i}" for i in range(self.F)]
        self.kw = kernel_width or 0.75 * self.F ** 0.5
        self.cat = list(categorical)
        self.train = X
        self.seed = seed

    def explain(self, record: torch.Tensor, predict_proba: Callable, label: int = 1, num_samples: int = 5000,
                num_features: int = 10, ridge: float = 1.0):
        x = torch.as_tensor(record).float().view(-1).to(self.mean.device)
        g = torch.Generator(device=x.device).manual_seed(self.seed)
        Z = torch.randn((num_samples, self.F), device=x.device, generator=g)
        P = x + Z * self.std
        if self.cat:
            idx = torch.randint(0, self.train.shape[0], (num_samples,), device=x.device, generator=g)
            for c in self.cat:
                P[:, c] = self.train[idx, c]
        P[0] = x
        scaled = (P - x) / self.std
        d = scaled.norm(dim=1)
        w = torch.sqrt(torch.exp(-(d * d) / (self.kw ** 2)))
        y = torch.as_tensor(predict_proba(P)).float()
        y = y[:, label] if y.dim() == 2 else y
        A = torch.cat([torch.ones((num_samples, 1), device=x.device), scaled], 1).double()
        W = w.double().view(-1, 1)
        AtW = (A * W).T
        reg = ridge * torch.eye(self.F + 1, dtype=torch.float64, device=x.device)
        reg[0, 0] = 0
        coef = torch.linalg.solve(AtW @ A + reg, AtW @ y.double().view(-1, 1)).view(-1)
        pred = A @ coef
        yy = y.double()
        ybar = (W.view(-1) * yy).sum() / W.sum()
        r2 = 1 - float((W.view(-1) * (yy - pred) ** 2).sum() / (W.view(-1) * (yy - ybar) ** 2).sum().clamp_min(1e-300))
        order = torch.argsort(coef[1:].abs(), descending=True)[:num_features].tolist()
        return {"intercept": float(coef[0]), "score": r2,
                "explanation": [(self.names[i], float(coef[1 + i])) for i in order],
                "local_pred": float(pred[0])}
