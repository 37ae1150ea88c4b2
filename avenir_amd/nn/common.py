"""Shared pieces of the neural models: activation / loss / optimiser factories (reference names),
tabular data preparation, checkpoints, device selection and CUDA(HIP)-graph capture of a training
step.

Reference: ``FeedForwardNetwork.createActivation/createLossFunction/createOptimizer``
(P/supv/tnn.py:154-230), ``prepData`` (:243-268), ``saveCheckpt/restoreCheckpt`` (:262-289);
``loadDataFile``/``scaleData`` (P/lib/mlutil.py:371-384, :649).

MI355X notes: the reference models are CPU-only (tnn) or create hidden state on the CPU (lstm
:267-273).  Here every model lives on ``common.device`` (default: the GPU when present), tabular
training steps with static shapes are captured ONCE into a HIP graph and replayed (small MLPs
are launch-bound, not FLOP-bound), and data-parallel training wraps the module in DDP over RCCL.
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Callable, Sequence

import numpy as np
import torch

ACTIVATIONS = {
    "relu": lambda: torch.nn.ReLU(), "tanh": lambda: torch.nn.Tanh(), "sigmoid": lambda: torch.nn.Sigmoid(),
    "softmax": lambda: torch.nn.Softmax(dim=1), "leakyRelu": lambda: torch.nn.LeakyReLU(),
    "elu": lambda: torch.nn.ELU(), "selu": lambda: torch.nn.SELU(), "gelu": lambda: torch.nn.GELU(),
    "logSigmoid": lambda: torch.nn.LogSigmoid(), "softplus": lambda: torch.nn.Softplus(),
    "logSoftmax": lambda: torch.nn.LogSoftmax(dim=1),
}


def create_activation(name: str | None):
    if name is None or name == "none":
        return None
    if name not in ACTIVATIONS:
        raise ValueError(f"invalid activation function name {name}")
    return ACTIVATIONS[name]()


def create_loss(name: str, reduction: str = "mean"):
    table = {"mse": torch.nn.MSELoss, "ce": torch.nn.CrossEntropyLoss, "lone": torch.nn.L1Loss,
             "bce": torch.nn.BCELoss, "bcel": torch.nn.BCEWithLogitsLoss, "sm": torch.nn.SoftMarginLoss,
             "mlsm": torch.nn.MultiLabelSoftMarginLoss, "nll": torch.nn.NLLLoss, "huber": torch.nn.HuberLoss}
    if name not in table:
        raise ValueError(f"invalid loss function name {name}")
    return table[name](reduction=reduction)


def create_optimizer(params, name: str, lr: float = 1e-4, weight_decay: float = 0.0, momentum: float = 0.0,
                     eps: float = 1e-8, dampening: float = 0.0, nesterov: bool = False,
                     betas: Sequence[float] = (0.9, 0.999), alpha: float = 0.99, capturable: bool = False):
    """The reference's optimiser names (P/lib/tnn.py).  GPU parameters take torch's fused
    single-kernel Adam / AdamW: the multi-tensor (foreach) update was 4 launches, ~45 us of a
    0.55 ms LSTM training step at the reference shape (profiles/r5_lstm_fp32_v4_kernel_stats.csv).
    (A fused step does not bump the parameters' version counters; the framework's packed-parameter
    caches key on utils/params.param_epoch() as well, which every optimizer step advances.)"""
    params = list(params)
    flat = [p for g in params for p in (g["params"] if isinstance(g, dict) else [g])]
    fused = (bool(flat) and all(p.is_cuda and p.dtype == torch.float32 for p in flat)
             and os.environ.get("AVMI_FUSED_OPT", "1") != "0")           # A/B switch
    fk = {"fused": True} if fused else {}
    if name == "sgd":
        return torch.optim.SGD(params, lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                               nesterov=nesterov)
    if name == "adam":
        return torch.optim.Adam(params, lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay,
                                capturable=capturable, **fk)
    if name == "adamw":
        return torch.optim.AdamW(params, lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay,
                                 capturable=capturable, **fk)
    if name == "rmsprop":
        return torch.optim.RMSprop(params, lr=lr, alpha=alpha, eps=eps, weight_decay=weight_decay, momentum=momentum,
                                   capturable=capturable)
    raise ValueError(f"invalid optimizer name {name}")


def optimizer_from_config(params, conf, prefix: str = "train.opt.", name_key: str = "train.optimizer",
                          capturable: bool = False):
    g = lambda k, d: _cfg(conf, prefix + k, d)
    betas = g("betas", [0.9, 0.999])
    if isinstance(betas, str):
        betas = [float(x) for x in betas.split(",")]
    return create_optimizer(params, _cfg(conf, name_key, "adam"), float(g("learning.rate", 1e-4)),
                            float(g("weight.decay", 0.0)), float(g("momentum", 0.0)), float(g("eps", 1e-8)),
                            float(g("dampening", 0.0)), bool(g("momentum.nesterov", False)), betas,
                            float(g("alpha", 0.99)), capturable)


def _cfg(conf, key, default):
    """Read ``key`` from a reference-style Configuration (value, is_default) or a dict."""
    if conf is None:
        return default
    if isinstance(conf, dict) or hasattr(conf, "values") and not hasattr(conf, "defaults"):
        # a plain dict, or a CLI JobConfig (.properties strings): typed like the default
        vals = conf if isinstance(conf, dict) else conf.values
        v = vals.get(key, default)
        if v in (None, "_"):
            return default
        if isinstance(v, str) and default is not None and not isinstance(default, str):
            if isinstance(default, bool):
                return v.strip().lower() == "true"
            if isinstance(default, int):
                return int(v)
            if isinstance(default, float):
                return float(v)
            if isinstance(default, list):
                return [float(x) for x in v.split(",")]
        return v
    if key not in conf.defaults:
        conf.defaults[key] = (default, None)
        conf.configs.setdefault(key, "_")
    d = conf.defaults[key][0]
    if isinstance(d, bool):
        return conf.get_boolean(key)[0]
    if isinstance(d, int):
        return conf.get_int(key)[0]
    if isinstance(d, float):
        return conf.get_float(key)[0]
    if isinstance(d, list):
        v = conf.configs.get(key, "_")
        return d if v == "_" else [float(x) for x in str(v).split(",")]
    return conf.get_string(key)[0]


def pick_device(name: "str | torch.device | None" = None) -> torch.device:
    if isinstance(name, torch.device):
        return name
    if name in (None, "", "auto"):
        return torch.device("cuda" if torch.cuda.is_available() else "cpu")
    if name.startswith("cuda") and not torch.cuda.is_available():
        return torch.device("cpu")
    return torch.device(name)


# ------------------------------------------------------------------------------------------------
# data
# ------------------------------------------------------------------------------------------------
def load_data_file(path, delim: str = ",", field_indices: Sequence[int] | None = None,
                   feat_indices: Sequence[int] | None = None):
    """(selected columns ``field_indices`` of the file, then columns ``feat_indices`` OF THAT
    selection) as float64 arrays — mlutil.loadDataFile semantics (P/lib/mlutil.py:371-377)."""
    rows = [l.rstrip("\n").split(delim) for l in Path(path).read_text().splitlines() if l.strip()]
    data = np.array([[float(r[i]) for i in field_indices] for r in rows] if field_indices
                    else [[float(v) for v in r] for r in rows], dtype=np.float64)
    feat = data if feat_indices is None else data[:, list(feat_indices)]
    return data, feat


def scale_data(x: np.ndarray | torch.Tensor, method: str = "zscale"):
    t = torch.as_tensor(x, dtype=torch.float64)
    if method == "zscale":
        sd = t.std(0, unbiased=False)
        return ((t - t.mean(0)) / torch.where(sd > 0, sd, torch.ones_like(sd))).numpy() if isinstance(x, np.ndarray) \
            else (t - t.mean(0)) / torch.where(sd > 0, sd, torch.ones_like(sd))
    if method == "minmax":
        lo, hi = t.min(0).values, t.max(0).values
        r = torch.where(hi > lo, hi - lo, torch.ones_like(hi))
        out = (t - lo) / r
        return out.numpy() if isinstance(x, np.ndarray) else out
    raise ValueError(method)


# ------------------------------------------------------------------------------------------------
# checkpoints (state dicts only; loaded with weights_only=True)
# ------------------------------------------------------------------------------------------------
def save_checkpoint(path, model: torch.nn.Module, optimizer: torch.optim.Optimizer | None = None, **extra):
    p = Path(path)
    p.parent.mkdir(parents=True, exist_ok=True)
    state = {"state_dict": {k: v.detach().cpu() for k, v in model.state_dict().items()}}
    if optimizer is not None:
        state["optim_dict"] = optimizer.state_dict()
    state.update(extra)
    tmp = p.with_suffix(p.suffix + ".tmp")
    torch.save(state, tmp)
    os.replace(tmp, p)


def load_checkpoint(path, model: torch.nn.Module, optimizer: torch.optim.Optimizer | None = None) -> dict:
    state = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(state["state_dict"])
    if optimizer is not None and "optim_dict" in state:
        optimizer.load_state_dict(state["optim_dict"])
    return state


# ------------------------------------------------------------------------------------------------
# HIP-graph captured training step
# ------------------------------------------------------------------------------------------------
class GraphedStep:
    """Capture ``step_fn(x, y) -> loss`` (forward + backward + optimiser step) into one HIP graph
    for fixed-shape batches; ``__call__`` copies the batch into static buffers and replays.  Falls
    back to eager execution on CPU or when capture is disabled.

    Capture needs a few eager warm-up steps (allocator pools, lazily created optimiser state).
    When ``model`` / ``optimizer`` are given, their state is restored afterwards — parameters and
    buffers to the pre-warm-up values, optimiser state tensors to their initial zeros (step
    counts 0) — so the warm-up does not count as training.  Restoration is in place, so the
    addresses captured in the graph stay valid."""

    def __init__(self, step_fn: Callable, x_example: torch.Tensor, y_example: torch.Tensor, enabled: bool = True,
                 warmup: int = 3, model: torch.nn.Module | None = None,
                 optimizer: torch.optim.Optimizer | None = None):
        self.fn = step_fn
        self.enabled = enabled and x_example.is_cuda
        self.graph = None
        if self.enabled:
            snap = [t.detach().clone() for t in _state_tensors(model)] if model is not None else None
            self.sx = x_example.clone()
            self.sy = y_example.clone()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(warmup):
                    self.fn(self.sx, self.sy)
            torch.cuda.current_stream().wait_stream(s)
            from ..utils.hipgraph import capturing
            self.graph = torch.cuda.CUDAGraph()
            with capturing(self.graph, device=self.sx.device):
                self.sloss = self.fn(self.sx, self.sy)
            with torch.no_grad():
                if snap is not None:
                    for t, v in zip(_state_tensors(model), snap):
                        t.copy_(v)
                if optimizer is not None:
                    for st in optimizer.state.values():
                        for v in st.values():
                            if torch.is_tensor(v):
                                v.zero_()

    def __call__(self, x, y):
        if self.graph is None:
            return self.fn(x, y)
        self.sx.copy_(x, non_blocking=True)
        self.sy.copy_(y, non_blocking=True)
        self.graph.replay()
        return self.sloss


def _state_tensors(model: torch.nn.Module):
    return [p for p in model.parameters()] + [b for b in model.buffers()]
