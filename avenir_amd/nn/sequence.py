"""LSTM sequence models (``LstmNetwork``, P/supv/lstm.py:42-378).

Rows hold one flattened sequence ``seq_len x input_size`` (+ optional target column); the model is
``ops.rnn.FusedLSTM`` (K27: one persistent HIP kernel launch per layer for the whole recurrence,
forward and backward; same parameter names as ``nn.LSTM``) + Linear + optional output
activation, seq-to-one (last step) or seq-to-seq.  Differences from the reference, all deliberate:
* batches are formed by ONE reshape + gather on the device instead of a per-element Python loop
  (lstm.py:187-218);
* the initial hidden state is created on the model's device (the reference makes it on the CPU,
  :267-273, which breaks GPU training);
* one checkpoint key (the reference saves under ``train.save.model`` but reads
  ``train.model.save``, :84 vs :337).
Data-parallel training (SURVEY N7 "optional DDP over RCCL"): with a multi-rank communicator every
rank fits its own row shard; the replicas start from rank 0's parameters, and each step sums the
gradients of all ranks in ONE coalesced all-reduce (RCCL over xGMI on GPUs) before clipping and the
optimiser — the global-batch gradient, so W ranks of local batch b train like one process with
batch W x b.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops.rnn import FusedLSTM
from ..parallel.comm import get_comm
from ..utils.params import bump_param_epoch
from .common import (GraphedStep, _cfg, create_activation, create_loss, load_checkpoint, optimizer_from_config, pick_device,
                     save_checkpoint, scale_data)


class LstmNetwork(torch.nn.Module):
    def __init__(self, input_size: int, hidden_size: int, output_size: int, num_layers: int = 1, seq_len: int = 1,
                 batch_size: int = 32, out_sequence: bool = False, out_activation: str | None = "sigmoid",
                 dropout: float = 0.0, loss: str = "mse", optimizer: str = "adam", lr: float = 1e-3,
                 grad_clip: float = 5.0, num_iter: int = 100, device=None, conf=None, graph: bool = True,
                 precision: str = "fp32"):
        super().__init__()
        self.input_size, self.hidden_size, self.output_size = input_size, hidden_size, output_size
        self.num_layers, self.seq_len, self.batch_size = num_layers, seq_len, batch_size
        self.out_seq, self.grad_clip, self.num_iter = out_sequence, grad_clip, num_iter
        # K27 fused LSTM (persistent HIP recurrence kernel on the GPU); nn.LSTM-compatible state dict
        # precision="fp32" (default): the reference's fp32 numerics on the fused fp32 kernels;
        # "bf16": the mixed-precision kernels; "miopen": torch.lstm
        self.lstm = FusedLSTM(input_size, hidden_size, num_layers, batch_first=True,
                              dropout=dropout if num_layers > 1 else 0.0, precision=precision)
        self.linear = torch.nn.Linear(hidden_size, output_size)
        self.out_act = create_activation(out_activation)
        self.loss_name = loss
        self.loss_fn = create_loss(loss)
        self.device = pick_device(device)
        self.to(self.device)
        cfg = conf if conf is not None else {"train.optimizer": optimizer, "train.opt.learning.rate": lr}
        self.use_graph = graph
        self.optimizer = optimizer_from_config(self.parameters(), cfg,
                                               capturable=self.device.type == "cuda" and graph)
        self.conf = conf
        self.losses: list[float] = []
        self._dp = None          # the communicator of a data-parallel fit

    @classmethod
    def from_config(cls, conf, device=None) -> "LstmNetwork":
        return cls(int(_cfg(conf, "train.input.size", 1)), int(_cfg(conf, "train.hidden.size", 10)),
                   int(_cfg(conf, "train.output.size", 1)), num_layers=_cfg(conf, "train.num.layers", 1),
                   seq_len=_cfg(conf, "train.seq.len", 1), batch_size=_cfg(conf, "train.batch.size", 32),
                   out_sequence=_cfg(conf, "train.out.sequence", True),
                   out_activation=_cfg(conf, "train.out.activation", "sigmoid"),
                   dropout=float(_cfg(conf, "train.drop.prob", 0.0)), loss=_cfg(conf, "train.loss.fn", "mse"),
                   grad_clip=float(_cfg(conf, "train.grad.clip", 5.0)),
                   num_iter=_cfg(conf, "train.num.iterations", 500),
                   device=device or _cfg(conf, "common.device", "auto"), conf=conf,
                   precision=str(_cfg(conf, "train.precision", "fp32")))

    # -- data --------------------------------------------------------------------------------------
    def to_sequences(self, rows: torch.Tensor) -> torch.Tensor:
        """[n, seq_len * input_size] -> [n, seq_len, input_size] (one view, no Python loop)."""
        return torch.as_tensor(rows).float().reshape(-1, self.seq_len, self.input_size)

    def load_data(self, path, delim: str, col_start: int, col_end: int, target_col: int = -1, scale: str | None = None):
        cols = list(range(col_start, col_end + 1)) + ([target_col] if target_col >= 0 else [])
        data = np.loadtxt(path, delimiter=delim, usecols=cols, ndmin=2)
        s = data[:, : col_end - col_start + 1]
        if scale:
            s = scale_data(s.reshape(-1, self.input_size), scale).reshape(s.shape)
        x = self.to_sequences(torch.tensor(s, dtype=torch.float32))
        if target_col < 0:
            return x
        t = torch.tensor(data[:, -1])
        return x, (t.float() if self.output_size == 1 else t.long())

    # -- model -------------------------------------------------------------------------------------
    def init_hidden(self, batch: int):
        z = torch.zeros((self.num_layers, batch, self.hidden_size), device=self.device)
        return z, z.clone()

    def forward(self, x):
        out, _ = self.lstm(x, self.init_hidden(x.shape[0]))
        if self.out_seq:
            out = self.linear(out)                     # [B, S, O]
        else:
            out = self.linear(out[:, -1])              # [B, O]
        if self.out_act is not None:
            out = self.out_act(out)
        return out

    def _target(self, y):
        if self.loss_name in ("ce", "nll"):
            return y.long().view(-1)
        return y.float().view(y.shape[0], -1) if not self.out_seq else y.float()

    def _step(self, x, tgt):
        self.optimizer.zero_grad(set_to_none=False)
        out = self(x)
        if self.out_seq and self.loss_name in ("ce", "nll"):
            out = out.reshape(-1, out.shape[-1])
        loss = self.loss_fn(out, tgt)
        loss.backward()
        if self._dp is not None:
            self._allreduce_grads(self._dp)
        if self.grad_clip:
            torch.nn.utils.clip_grad_norm_(self.parameters(), self.grad_clip, foreach=True)
        self.optimizer.step()
        return loss.detach()

    def _allreduce_grads(self, comm):
        """Average the gradients over the ranks: one flat buffer, one all-reduce."""
        grads = [p.grad for p in self.parameters() if p.grad is not None]
        flat = torch.cat([g.reshape(-1) for g in grads])
        comm.all_reduce(flat)
        flat.div_(comm.world)
        off = 0
        for g in grads:
            g.copy_(flat[off:off + g.numel()].view_as(g))
            off += g.numel()

    def fit(self, x: torch.Tensor, y: torch.Tensor, num_iter: int | None = None, seed: int = 0,
            comm=None) -> "LstmNetwork":
        """``num_iter`` epochs of shuffled fixed-size mini-batches.  On the GPU the whole step
        (fused-LSTM forward, loss, backward, clipping, optimiser) is one captured HIP graph.  With a
        multi-rank communicator (``comm`` or the process default) each rank passes its own rows:
        replicas synchronised from rank 0, gradients averaged every step, the same number of steps
        on every rank (the smallest shard's), eager steps."""
        comm = comm if comm is not None else get_comm()
        dp = comm if comm.is_distributed else None
        x = x.to(self.device).float()
        tgt = self._target(y.to(self.device))
        n = x.shape[0]
        bs = min(self.batch_size, n)
        nb = max(n // bs, 1)
        if dp is not None:
            with torch.no_grad():
                for p in self.parameters():
                    dp.broadcast(p, 0)
            bump_param_epoch()          # the packed-weight caches must not serve pre-broadcast weights
            # on the communicator's device: an RCCL group takes device tensors only
            t = torch.tensor([nb], dtype=torch.long, device=self.device)
            dp.all_reduce(t, "min")
            nb = int(t)
        g = torch.Generator().manual_seed(seed)
        self.train()
        self._dp = dp
        step = None
        # no host synchronisation inside the loop: the epoch permutations go up from pinned memory
        # without blocking, and the epoch losses stay on the device until the fit ends
        dev_losses = []
        pin = self.device.type == "cuda"
        try:
            for _ in range(num_iter if num_iter is not None else self.num_iter):
                perm = torch.randperm(n, generator=g)
                perm = (perm.pin_memory().to(self.device, non_blocking=True) if pin else perm)[: nb * bs]
                xb = x[perm].view((nb, bs) + tuple(x.shape[1:]))
                yb = tgt[perm].view((nb, bs) + tuple(tgt.shape[1:]))
                if step is None:
                    step = GraphedStep(self._step, xb[0], yb[0],
                                       enabled=self.use_graph and self.device.type == "cuda" and dp is None,
                                       model=self, optimizer=self.optimizer)
                tot = torch.zeros((), device=self.device)
                for b in range(nb):
                    tot += step(xb[b], yb[b])
                dev_losses.append(tot / nb)
            if dev_losses:
                self.losses.extend(torch.stack(dev_losses).tolist())
        finally:
            self._dp = None
        self.eval()
        return self

    @torch.no_grad()
    def predict(self, x: torch.Tensor, output: str = "raw"):
        self.eval()
        out = self(torch.as_tensor(x).to(self.device).float())
        if output == "binary":
            return out.argmax(-1) if out.shape[-1] > 1 else (out.squeeze(-1) >= 0.5).long()
        return out

    def save(self, path):
        save_checkpoint(path, self, self.optimizer)

    def restore(self, path):
        load_checkpoint(path, self)
        self.to(self.device)
