"""Unsupervised neural models: (denoising) autoencoder and Bernoulli RBM with imputation.

* ``AutoEncoder`` (P/unsupv/ae.py:38-275): encoder / decoder stacks from ``train.num.hidden.units``
  and activation lists, optional input noise (``train.noise.scale``), ``encode`` and per-row
  reconstruction error.
* ``RestrictedBoltzmanMachine`` (P/unsupv/rbm.py:36-158) wraps sklearn's BernoulliRBM and imputes
  missing values by Gibbs sampling; here the RBM is trained with persistent contrastive divergence
  (the same estimator as sklearn's ``BernoulliRBM``) directly on the device: every step is two
  GEMMs plus Bernoulli sampling, and imputation runs ALL rows' Gibbs chains at once with the
  observed units clamped.
"""
from __future__ import annotations

from typing import Sequence

import torch

from .common import _cfg, create_activation, create_loss, load_checkpoint, optimizer_from_config, pick_device, \
    save_checkpoint


def _stack(dims: Sequence[int], acts: Sequence[str | None], fused: bool) -> torch.nn.Sequential:
    """Linear (+ activation) layers; a Linear + activation the K27 kernel covers is ONE fused layer
    (nn/mlp.py ``FusedLinear``, an ``Identity`` keeps the activation's index, so the parameter
    names equal the ``torch.nn`` twin's)."""
    from ..ops.mlp_ops import ACT_CODES
    from .mlp import FusedLinear
    out = []
    for i in range(len(dims) - 1):
        name = acts[i] if i < len(acts) else None
        a = create_activation(name)
        if fused and a is not None and name in ACT_CODES:
            out += [FusedLinear(dims[i], dims[i + 1], name), torch.nn.Identity()]
            continue
        out.append(torch.nn.Linear(dims[i], dims[i + 1]))
        if a is not None:
            out.append(a)
    return torch.nn.Sequential(*out)


class AutoEncoder(torch.nn.Module):
    """On the GPU the layers run the fused Linear + activation kernels and one mini-batch step
    (forward, loss, backward, optimiser) is a captured HIP graph replayed per batch (the batch's
    noise is drawn outside the graph into its static input); ``fused=False`` / ``graph=False``
    give the eager ``torch.nn`` twin."""

    def __init__(self, n_in: int, hidden: Sequence[int], enc_act: Sequence[str | None], dec_act: Sequence[str | None],
                 lr: float = 1e-3, weight_decay: float = 1e-5, batch_size: int = 128, noise_scale: float = 0.0,
                 num_iter: int = 100, loss: str = "mse", optimizer: str = "adam", device=None, fused: bool = True,
                 graph: bool = True):
        super().__init__()
        dims = [n_in] + list(hidden)
        self.encoder = _stack(dims, enc_act, fused)
        self.decoder = _stack(list(reversed(dims)), dec_act, fused)
        self.use_graph = graph
        self.batch_size, self.noise, self.num_iter = batch_size, noise_scale, num_iter
        self.loss_fn = create_loss(loss)
        self.device = pick_device(device)
        self.to(self.device)
        self.optimizer = optimizer_from_config(self.parameters(), {"train.optimizer": optimizer,
                                                                   "train.opt.learning.rate": lr,
                                                                   "train.opt.weight.decay": weight_decay},
                                               capturable=self.device.type == "cuda")
        self.losses: list[float] = []

    @classmethod
    def from_config(cls, conf, device=None) -> "AutoEncoder":
        hid = [int(v) for v in str(_cfg(conf, "train.num.hidden.units", "")).split(",")]
        ea = [None if v == "none" else v for v in str(_cfg(conf, "train.encoder.activations", "")).split(",")]
        da = [None if v == "none" else v for v in str(_cfg(conf, "train.decoder.activations", "")).split(",")]
        return cls(int(_cfg(conf, "train.num.input", 1)), hid, ea, da, lr=float(_cfg(conf, "train.learning.rate", 1e-4)),
                   weight_decay=float(_cfg(conf, "train.weight.decay", 1e-5)),
                   batch_size=_cfg(conf, "train.batch.size", 128), noise_scale=float(_cfg(conf, "train.noise.scale", 0.0)),
                   num_iter=_cfg(conf, "train.num.iterations", 500), loss=_cfg(conf, "train.loss", "mse"),
                   optimizer=_cfg(conf, "train.optimizer", "adam"), device=device or _cfg(conf, "common.device", "auto"))

    def forward(self, x):
        return self.decoder(self.encoder(x))

    def _step(self, inp, target):
        self.optimizer.zero_grad(set_to_none=False)
        loss = self.loss_fn(self(inp), target)
        loss.backward()
        self.optimizer.step()
        return loss.detach()

    def fit(self, x: torch.Tensor, num_iter: int | None = None, seed: int = 0) -> "AutoEncoder":
        from .common import GraphedStep
        x = x.to(self.device).float()
        n = x.shape[0]
        bs = min(self.batch_size, n)
        nb = max(n // bs, 1)
        g = torch.Generator(device=self.device).manual_seed(seed)
        self.train()
        # the captured step is kept across fit() calls of the same batch shape (a new capture per
        # call cost more than its replays saved at one epoch per call: profiles/r6_rl_unsup.jsonl)
        key = (bs, x.shape[1], self.use_graph)
        step = self._gstep if getattr(self, "_gkey", None) == key else None
        ep_losses = []                  # on the device until the fit ends: no host sync per epoch
        for _ in range(num_iter if num_iter is not None else self.num_iter):
            perm = torch.randperm(n, device=self.device, generator=g)
            tot = torch.zeros((), device=self.device)
            for b in range(nb):
                xb = x[perm[b * bs:(b + 1) * bs]]
                inp = xb + self.noise * torch.randn(xb.shape, device=self.device, generator=g) if self.noise else xb
                if step is None:
                    step = GraphedStep(self._step, inp, xb, enabled=self.use_graph and self.device.type == "cuda",
                                       model=self, optimizer=self.optimizer)
                    self._gstep, self._gkey = step, key
                tot += step(inp, xb)
            ep_losses.append(tot / nb)
        if ep_losses:
            self.losses.extend(torch.stack(ep_losses).tolist())
        self.eval()
        return self

    @torch.no_grad()
    def encode(self, x):
        return self.encoder(x.to(self.device).float())

    @torch.no_grad()
    def reconstruction_error(self, x):
        x = x.to(self.device).float()
        return ((self(x) - x) ** 2).mean(1)

    def save(self, path):
        save_checkpoint(path, self, self.optimizer)

    def restore(self, path):
        load_checkpoint(path, self)


class RestrictedBoltzmannMachine:
    """Bernoulli-Bernoulli RBM trained by persistent contrastive divergence (PCD-1)."""

    def __init__(self, n_visible: int, n_hidden: int, lr: float = 0.1, batch_size: int = 10, num_iter: int = 10,
                 seed: int = 0, device=None):
        self.device = pick_device(device)
        self.g = torch.Generator(device=self.device).manual_seed(seed)
        self.W = 0.01 * torch.randn((n_hidden, n_visible), device=self.device, generator=self.g)
        self.bh = torch.zeros(n_hidden, device=self.device)
        self.bv = torch.zeros(n_visible, device=self.device)
        self.lr, self.batch_size, self.num_iter = lr, batch_size, num_iter
        self.pseudo_ll: list[float] = []

    @classmethod
    def from_config(cls, conf, n_visible: int, device=None):
        return cls(n_visible, int(_cfg(conf, "train.num.components", 100)), float(_cfg(conf, "train.learning.rate", 0.1)),
                   _cfg(conf, "train.batch.size", 10), _cfg(conf, "train.num.iter", 10), device=device)

    def hidden_prob(self, v):
        if v.is_cuda and v.dim() == 2:
            from ..ops.mlp_ops import linear_act
            return linear_act(v.contiguous(), self.W, self.bh, "sigmoid")   # K27 fused GEMM + sigmoid
        return torch.sigmoid(v @ self.W.T + self.bh)

    def visible_prob(self, h):
        return torch.sigmoid(h @ self.W + self.bv)

    def _bern(self, p):
        return (torch.rand(p.shape, device=p.device, generator=self.g) < p).float()

    def gibbs(self, v):
        return self._bern(self.visible_prob(self._bern(self.hidden_prob(v))))

    def _cd_step(self, v, chain, u_h, u_v, lr: float):
        """One PCD-1 update from uniforms drawn outside (device-only, capturable, in place): the
        hidden probabilities are the fused Linear + sigmoid kernel on the GPU."""
        hp = self.hidden_prob(v)
        hs = (u_h < self.hidden_prob(chain)).float()
        chain.copy_((u_v < self.visible_prob(hs)).float())
        hn = self.hidden_prob(chain)
        self.W.add_(hp.T @ v - hn.T @ chain, alpha=lr)
        self.bh.add_(hp.sum(0) - hn.sum(0), alpha=lr)
        self.bv.add_(v.sum(0) - chain.sum(0), alpha=lr)

    def fit(self, x: torch.Tensor, graph: bool = True) -> "RestrictedBoltzmannMachine":
        """PCD-1 over shuffled mini-batches.  The uniforms of a step are drawn in the eager
        order (hidden sample, then visible) into static buffers, so the graphed replay (GPU:
        the whole step is ONE HIP graph) consumes the generator exactly like the eager loop."""
        from ..utils.hipgraph import capturing
        x = x.to(self.device).float()
        n, V = x.shape
        H = self.W.shape[0]
        bs = min(self.batch_size, n)
        lr = self.lr / bs
        chain = torch.zeros((bs, V), device=self.device)
        sv = torch.zeros((bs, V), device=self.device)
        u_h = torch.empty((bs, H), device=self.device)
        u_v = torch.empty((bs, V), device=self.device)
        use_graph = graph and self.device.type == "cuda"
        cg = None
        for _ in range(self.num_iter):
            perm = torch.randperm(n, device=self.device, generator=self.g)
            for b in range(n // bs):
                sv.copy_(x[perm[b * bs:(b + 1) * bs]])
                torch.rand((bs, H), device=self.device, generator=self.g, out=u_h)
                torch.rand((bs, V), device=self.device, generator=self.g, out=u_v)
                if use_graph and cg is None:
                    # warm-up on a side stream with the state restored afterwards, then capture
                    snap = [t.clone() for t in (self.W, self.bh, self.bv, chain)]
                    side = torch.cuda.Stream(self.device)
                    side.wait_stream(torch.cuda.current_stream(self.device))
                    with torch.cuda.stream(side):
                        self._cd_step(sv, chain, u_h, u_v, lr)
                    torch.cuda.current_stream(self.device).wait_stream(side)
                    for t, s0 in zip((self.W, self.bh, self.bv, chain), snap):
                        t.copy_(s0)
                    cg = torch.cuda.CUDAGraph()
                    with capturing(cg, device=self.device):
                        self._cd_step(sv, chain, u_h, u_v, lr)
                if cg is not None:
                    cg.replay()
                else:
                    self._cd_step(sv, chain, u_h, u_v, lr)
            self.pseudo_ll.append(float(self.score_samples(x).mean()))
        return self

    def free_energy(self, v):
        return -(v @ self.bv) - torch.nn.functional.softplus(v @ self.W.T + self.bh).sum(1)

    def score_samples(self, v):
        """Stochastic pseudo-likelihood (flip one random unit per row), like sklearn's estimator."""
        v = v.to(self.device).float()
        idx = torch.randint(0, v.shape[1], (v.shape[0],), device=self.device, generator=self.g)
        vf = v.clone()
        r = torch.arange(v.shape[0], device=self.device)
        vf[r, idx] = 1 - vf[r, idx]
        return v.shape[1] * torch.nn.functional.logsigmoid(self.free_energy(vf) - self.free_energy(v))

    def save(self, path):
        """Weights and biases in the framework's container (utils/checkpoint.py; the reference
        pickles the sklearn estimator with joblib, P/unsupv/rbm.py:127-133)."""
        from ..utils import checkpoint as C
        C.save(path, {"W": self.W, "bh": self.bh, "bv": self.bv},
               {"lr": self.lr, "batch_size": self.batch_size, "num_iter": self.num_iter})

    def restore(self, path) -> "RestrictedBoltzmannMachine":
        from ..utils import checkpoint as C
        t, m = C.load(path, self.device)
        self.W, self.bh, self.bv = t["W"].float(), t["bh"].float(), t["bv"].float()
        self.lr, self.batch_size, self.num_iter = m["lr"], m["batch_size"], m["num_iter"]
        return self

    @torch.no_grad()
    def impute(self, x: torch.Tensor, missing: torch.Tensor, n_iter: int = 100, init: float | None = None):
        """Fill ``missing`` (bool mask) entries by Gibbs sampling with observed units clamped; the
        final value is the mean visible probability over the last half of the chain."""
        x = x.to(self.device).float().clone()
        m = missing.to(self.device).bool()
        x[m] = init if init is not None else 0.5
        acc = torch.zeros_like(x)
        cnt = 0
        for it in range(n_iter):
            p = self.visible_prob(self._bern(self.hidden_prob(x)))
            x = torch.where(m, self._bern(p), x)
            if it >= n_iter // 2:
                acc += p
                cnt += 1
        return torch.where(m, (acc / max(cnt, 1) >= 0.5).float(), x)
