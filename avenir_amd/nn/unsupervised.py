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


class AutoEncoder(torch.nn.Module):
    def __init__(self, n_in: int, hidden: Sequence[int], enc_act: Sequence[str | None], dec_act: Sequence[str | None],
                 lr: float = 1e-3, weight_decay: float = 1e-5, batch_size: int = 128, noise_scale: float = 0.0,
                 num_iter: int = 100, loss: str = "mse", optimizer: str = "adam", device=None):
        super().__init__()
        enc, dims = [], [n_in] + list(hidden)
        for i in range(len(hidden)):
            enc.append(torch.nn.Linear(dims[i], dims[i + 1]))
            a = create_activation(enc_act[i] if i < len(enc_act) else None)
            if a is not None:
                enc.append(a)
        dec = []
        rd = list(reversed(dims))
        for i in range(len(hidden)):
            dec.append(torch.nn.Linear(rd[i], rd[i + 1]))
            a = create_activation(dec_act[i] if i < len(dec_act) else None)
            if a is not None:
                dec.append(a)
        self.encoder, self.decoder = torch.nn.Sequential(*enc), torch.nn.Sequential(*dec)
        self.batch_size, self.noise, self.num_iter = batch_size, noise_scale, num_iter
        self.loss_fn = create_loss(loss)
        self.device = pick_device(device)
        self.to(self.device)
        self.optimizer = optimizer_from_config(self.parameters(), {"train.optimizer": optimizer,
                                                                   "train.opt.learning.rate": lr,
                                                                   "train.opt.weight.decay": weight_decay})
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

    def fit(self, x: torch.Tensor, num_iter: int | None = None, seed: int = 0) -> "AutoEncoder":
        x = x.to(self.device).float()
        n = x.shape[0]
        bs = min(self.batch_size, n)
        g = torch.Generator(device=self.device).manual_seed(seed)
        self.train()
        for _ in range(num_iter if num_iter is not None else self.num_iter):
            perm = torch.randperm(n, device=self.device, generator=g)
            tot = torch.zeros((), device=self.device)
            nb = max(n // bs, 1)
            for b in range(nb):
                xb = x[perm[b * bs:(b + 1) * bs]]
                inp = xb + self.noise * torch.randn(xb.shape, device=self.device, generator=g) if self.noise else xb
                self.optimizer.zero_grad()
                loss = self.loss_fn(self(inp), xb)
                loss.backward()
                self.optimizer.step()
                tot += loss.detach()
            self.losses.append(float(tot) / nb)
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
        return torch.sigmoid(v @ self.W.T + self.bh)

    def visible_prob(self, h):
        return torch.sigmoid(h @ self.W + self.bv)

    def _bern(self, p):
        return (torch.rand(p.shape, device=p.device, generator=self.g) < p).float()

    def gibbs(self, v):
        return self._bern(self.visible_prob(self._bern(self.hidden_prob(v))))

    def fit(self, x: torch.Tensor) -> "RestrictedBoltzmannMachine":
        x = x.to(self.device).float()
        n = x.shape[0]
        bs = min(self.batch_size, n)
        chain = torch.zeros((bs, x.shape[1]), device=self.device)
        for _ in range(self.num_iter):
            perm = torch.randperm(n, device=self.device, generator=self.g)
            for b in range(n // bs):
                v = x[perm[b * bs:(b + 1) * bs]]
                hp = self.hidden_prob(v)
                hs = self._bern(self.hidden_prob(chain))
                chain = self._bern(self.visible_prob(hs))
                hn = self.hidden_prob(chain)
                lr = self.lr / bs
                self.W += lr * (hp.T @ v - hn.T @ chain)
                self.bh += lr * (hp.sum(0) - hn.sum(0))
                self.bv += lr * (v.sum(0) - chain.sum(0))
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
