"""Configurable feed-forward network (``FeedForwardNetwork``, P/supv/tnn.py:37-464).

Layer spec ``units:activation:batchnorm:afterAct:dropout`` per layer, comma separated
(tnn.py:100-145); losses mse/ce/lone/bce/bcel/sm/mlsm; optimisers sgd/adam/rmsprop; full-batch
(``allTrain`` :319) and mini-batch (``batchTrain`` :356-422) training with optional error tracking;
``predict`` :425; ``evaluateModel`` :452; checkpoints :262-289.

MI355X: the module and its data live on the GPU; every mini-batch step of a shuffled epoch has
the same shape, so the step (forward, loss, backward, optimiser) is captured once as a HIP graph
and replayed; with ``world > 1`` the module is wrapped in DDP (RCCL all-reduce of gradient
buckets overlapped with backward).
"""
from __future__ import annotations

from typing import Sequence

import numpy as np
import torch

from ..parallel.comm import get_comm
from ..utils.metrics import perf_metric
from .common import (GraphedStep, _cfg, create_activation, create_loss, load_checkpoint, load_data_file,
                     optimizer_from_config, pick_device, save_checkpoint, scale_data)


class FusedLinear(torch.nn.Linear):
    """``Linear`` followed by an activation, run as the K27 fused kernel on the GPU
    (``ops.mlp_ops.linear_act``).  Same parameter names as ``torch.nn.Linear``, so checkpoints keep
    the reference's ``layers.<i>.weight`` keys; the activation's slot in the Sequential holds an
    ``Identity``."""

    def __init__(self, n_in: int, n_out: int, act: str):
        super().__init__(n_in, n_out)
        self.act = act

    def forward(self, x):
        from ..ops.mlp_ops import linear_act
        return linear_act(x, self.weight, self.bias, self.act)

    def extra_repr(self) -> str:
        return super().extra_repr() + f", act={self.act}"


def parse_layer_spec(spec: str, n_in: int, fuse: bool = True) -> torch.nn.Sequential:
    layers: list[torch.nn.Module] = []
    ninp = n_in
    for ld in spec.split(","):
        parts = ld.split(":")
        if len(parts) != 5:
            raise ValueError("expecting 5 items for layer data: units:activation:batchnorm:afterAct:dropout")
        nunit, act_s, bn, after, dpr = int(parts[0]), parts[1], parts[2] == "true", parts[3] == "true", float(parts[4])
        layers.append(torch.nn.Linear(ninp, nunit))
        act = create_activation(act_s)
        if bn:
            if after:
                if act is not None:
                    layers.append(act)
                layers.append(torch.nn.BatchNorm1d(nunit))
            else:
                layers.append(torch.nn.BatchNorm1d(nunit))
                if act is not None:
                    layers.append(act)
        elif act is not None:
            from ..ops.mlp_ops import ACT_CODES
            if fuse and act_s in ACT_CODES:
                # Linear + activation -> one fused kernel; Identity keeps the module indices
                layers[-1] = FusedLinear(ninp, nunit, act_s)
                layers.append(torch.nn.Identity())
            else:
                layers.append(act)
        if dpr > 0:
            layers.append(torch.nn.Dropout(dpr))
        ninp = nunit
    return torch.nn.Sequential(*layers)


class FeedForwardNetwork(torch.nn.Module):
    def __init__(self, layer_spec: str, n_in: int, loss: str = "mse", optimizer: str = "sgd", lr: float = 1e-4,
                 batch_size: int = 10, num_iter: int = 500, device=None, conf=None, loss_reduction: str = "mean",
                 acc_metric: str | None = None, graph: bool = True, opt_kw: dict | None = None):
        super().__init__()
        self.layers = parse_layer_spec(layer_spec, n_in)
        self.device = pick_device(device)
        self.to(self.device)
        self.loss_name = loss
        self.loss_fn = create_loss(loss, loss_reduction)
        self.batch_size, self.num_iter = batch_size, num_iter
        self.acc_metric = acc_metric
        self.use_graph = graph
        cfg = dict(opt_kw or {})
        cfg.setdefault("train.optimizer", optimizer)
        cfg.setdefault("train.opt.learning.rate", lr)
        self.optimizer = optimizer_from_config(self.parameters(), conf if conf is not None else cfg,
                                               capturable=self.device.type == "cuda" and graph)
        self.conf = conf
        self.errors: list[float] = []
        self.ddp = None

    @classmethod
    def from_config(cls, conf, device=None) -> "FeedForwardNetwork":
        """Reference-style :class:`~avenir_amd.utils.config.Configuration` (P/supv/tnn.py:37-90)."""
        n_in = len(str(_cfg(conf, "train.data.feature.fields", "")).split(","))
        return cls(_cfg(conf, "train.layer.data", ""), n_in, loss=_cfg(conf, "train.lossFn", "mse"),
                   optimizer=_cfg(conf, "train.optimizer", "sgd"), lr=_cfg(conf, "train.opt.learning.rate", 1e-4),
                   batch_size=_cfg(conf, "train.batch.size", 10), num_iter=_cfg(conf, "train.num.iterations", 500),
                   device=device or _cfg(conf, "common.device", "auto"), conf=conf,
                   loss_reduction=_cfg(conf, "train.loss.reduction", "mean"),
                   acc_metric=_cfg(conf, "valid.accuracy.metric", None))

    def forward(self, x):
        return self.layers(x)

    # -- data --------------------------------------------------------------------------------------
    def prep_data(self, path, include_out: bool = True):
        conf = self.conf
        fields = [int(v) for v in str(_cfg(conf, "train.data.fields", "")).split(",")]
        feats = [int(v) for v in str(_cfg(conf, "train.data.feature.fields", "")).split(",")]
        data, feat = load_data_file(path, ",", fields, feats)
        if _cfg(conf, "common.preprocessing", None) == "scale":
            feat = scale_data(feat, _cfg(conf, "common.scaling.method", "zscale"))
        x = torch.tensor(np.asarray(feat, dtype=np.float32))
        if not include_out:
            return x
        outs = [int(v) for v in str(_cfg(conf, "train.data.out.fields", "")).split(",")]
        y = torch.tensor(np.asarray(data[:, outs], dtype=np.float32))
        return x, y

    def _target(self, y: torch.Tensor) -> torch.Tensor:
        if self.loss_name in ("ce", "nll"):
            return y.view(-1).long()
        return y.float().view(y.shape[0], -1)

    # -- training ----------------------------------------------------------------------------------
    def _step(self, x, y):
        self.optimizer.zero_grad(set_to_none=False)
        out = (self.ddp or self)(x)
        loss = self.loss_fn(out, y)
        loss.backward()
        self.optimizer.step()
        return loss.detach()

    def fit(self, x: torch.Tensor, y: torch.Tensor, num_iter: int | None = None, full_batch: bool = False,
            seed: int = 0, track_interval: int = 0) -> "FeedForwardNetwork":
        """``num_iter`` epochs of shuffled mini-batches (``batchTrain``), or full-batch steps
        (``allTrain``).  Multi-rank: each rank passes its shard; DDP keeps replicas in sync."""
        comm = get_comm()
        x = x.to(self.device).float()
        y = self._target(y.to(self.device))
        self.train()
        if comm.is_distributed and self.ddp is None:
            self.ddp = torch.nn.parallel.DistributedDataParallel(
                self, device_ids=[self.device.index] if self.device.type == "cuda" else None,
                bucket_cap_mb=64)
        n = x.shape[0]
        bs = n if full_batch else min(self.batch_size, n)
        nb = n // bs
        g = torch.Generator(device="cpu").manual_seed(seed)
        use_graph = self.use_graph and self.device.type == "cuda" and self.ddp is None
        step = None
        for ep in range(num_iter if num_iter is not None else self.num_iter):
            perm = torch.randperm(n, generator=g).to(self.device) if not full_batch else torch.arange(n, device=self.device)
            xb = x[perm[: nb * bs]].view(nb, bs, -1)
            yb = y[perm[: nb * bs]].view((nb, bs) + tuple(y.shape[1:]))
            if step is None:
                step = GraphedStep(self._step, xb[0], yb[0], enabled=use_graph, model=self,
                                   optimizer=self.optimizer)
            tot = torch.zeros((), device=self.device)
            for b in range(nb):
                tot += step(xb[b], yb[b])
            if track_interval and (ep % track_interval == 0):
                self.errors.append(float(tot) / nb)
        self.eval()
        return self

    # -- inference ---------------------------------------------------------------------------------
    @torch.no_grad()
    def predict(self, x: torch.Tensor, output: str = "raw") -> torch.Tensor:
        self.eval()
        out = self(x.to(self.device).float())
        if output == "prob" and out.shape[1] > 1:
            return torch.softmax(out, 1) if self.loss_name == "ce" else out
        if output == "binary":
            return out.argmax(1) if out.shape[1] > 1 else (out.view(-1) >= 0.5).long()
        return out

    def evaluate_model(self, x: torch.Tensor, y: torch.Tensor, metric: str | None = None) -> float:
        """Validation score (``evaluateModel``): accuracy-type metrics on class predictions,
        regression metrics (rmse / mae) on raw outputs."""
        metric = metric or self.acc_metric or ("accuracy" if self.loss_name in ("ce", "bce", "bcel") else "rmse")
        out = self.predict(x)
        y = y.to(out.device)
        if metric in ("rmse", "mse", "mae"):
            e = out.view(-1) - y.float().view(-1)
            return float({"rmse": (e * e).mean().sqrt(), "mse": (e * e).mean(), "mae": e.abs().mean()}[metric])
        if out.shape[1] > 1:
            pred = out.argmax(1)
        else:
            pred = ((torch.sigmoid(out) if self.loss_name == "bcel" else out).view(-1) >= 0.5).long()
        return float(perf_metric(metric, y.view(-1).long().cpu(), pred.cpu()))

    def save(self, path):
        save_checkpoint(path, self, self.optimizer)

    def restore(self, path, load_opt: bool = False):
        load_checkpoint(path, self, self.optimizer if load_opt else None)
        self.to(self.device)
