"""Principal components: batch PCA and streaming (SPIRIT-style) incremental PCA.

Reference: ``IncrementalPrincipalComponent`` (S/explore/IncrementalPrincipalComponent.scala:83-212):
per key, records in time order update each hidden unit w_i by y = w_i.x, E_i = lambda E_i + y^2,
w_i += (x - y w_i) y / E_i, x -= y w_i; the number of hidden units grows / shrinks when the
captured energy leaves [low, high] x visible energy.  State = ``PrincipalCompState``
(J/util/PrincipalCompState.java:59-212: key, dimension, #hidden, count, energies, components).
Reference bugs not reproduced: ``extendPrinComp`` indexes past the array end and the shrink branch
drops two units (``slice(0, numHiddenStates-2)``).

MI355X design: all keys advance in lockstep as a [K, H, D] batch (one time step of every key per
iteration, ragged lengths masked), so thousands of per-key PCA states update with a handful of
batched ops per step; batch PCA is a Gram GEMM (+ all-reduce across ranks) and one ``eigh``.
"""
from __future__ import annotations

from typing import Sequence

import torch

from ..parallel.comm import Comm, get_comm


class PCA:
    def __init__(self, n_components: int | None = None, comm: Comm | None = None):
        self.k, self.comm = n_components, comm

    def fit(self, X: torch.Tensor) -> "PCA":
        comm = self.comm or get_comm()
        X = torch.as_tensor(X).double()
        D = X.shape[1]
        buf = torch.cat([torch.tensor([float(X.shape[0])], dtype=torch.float64, device=X.device), X.sum(0),
                         (X.T @ X).reshape(-1)])
        if comm.is_distributed:
            buf = comm.all_reduce(buf)
        n = float(buf[0])
        mu = buf[1:1 + D] / n
        C = (buf[1 + D:].view(D, D) - n * torch.outer(mu, mu)) / (n - 1)
        ev, V = torch.linalg.eigh(C)
        o = torch.argsort(ev, descending=True)
        k = self.k or D
        self.mean_, self.explained_variance_ = mu, ev[o][:k]
        self.components_ = V[:, o][:, :k].T                            # [k, D]
        # deterministic sign: largest |loading| positive
        s = torch.sign(self.components_.gather(1, self.components_.abs().argmax(1, keepdim=True)))
        self.components_ *= s
        self.explained_variance_ratio_ = self.explained_variance_ / ev.clamp_min(0).sum()
        return self

    def transform(self, X):
        return (torch.as_tensor(X).double().to(self.mean_.device) - self.mean_) @ self.components_.T

    def inverse_transform(self, Z):
        return Z @ self.components_ + self.mean_


class PrincipalCompState:
    """Per-key streaming PCA state with the reference's delimited text form."""

    def __init__(self, key: str, dimension: int, num_hidden: int, count: int = 0, energy: Sequence[float] | None = None,
                 hidden_unit_energy: Sequence[float] | None = None, components: torch.Tensor | None = None):
        self.key, self.dimension, self.num_hidden, self.count = key, dimension, num_hidden, count
        self.visible_energy = float(energy[0]) if energy else 0.0
        self.hidden_energy = list(energy[1:]) if energy else [0.0] * num_hidden
        self.hidden_unit_energy = list(hidden_unit_energy) if hidden_unit_energy else [1.0] * num_hidden
        if components is None:
            components = torch.eye(dimension, dtype=torch.float64)[:num_hidden]
        self.components = components

    def serialize(self, delim: str = ",", precision: int = 6) -> list[str]:
        f = lambda v: f"{v:.{precision}f}"
        head = delim.join([self.key, str(self.dimension), str(self.num_hidden), str(self.count)])
        lines = [head, delim.join(f(v) for v in [self.visible_energy] + self.hidden_energy),
                 delim.join(f(v) for v in self.hidden_unit_energy)]
        lines += [delim.join(f(float(v)) for v in row) for row in self.components.tolist()]
        return lines

    @classmethod
    def load(cls, lines: Sequence[str], delim: str = ","):
        key, dim, nh, cnt = lines[0].split(delim)
        dim, nh, cnt = int(dim), int(nh), int(cnt)
        energy = [float(v) for v in lines[1].split(delim)]
        hue = [float(v) for v in lines[2].split(delim)]
        comps = torch.tensor([[float(v) for v in l.split(delim)] for l in lines[3:3 + nh]], dtype=torch.float64)
        return cls(key, dim, nh, cnt, energy, hue, comps)


class IncrementalPCA:
    """SPIRIT-style streaming PCA for many keys at once.

    ``update(streams)`` takes {key: [T_k, D] tensor (time ordered)}; states persist across calls."""

    def __init__(self, dimension: int, init_hidden: int = 1, max_hidden: int | None = None, forget: float = 0.96,
                 low_energy: float = 0.95, high_energy: float = 0.98, device="cpu"):
        self.D, self.H0 = dimension, init_hidden
        self.Hmax = max_hidden or dimension
        if not 1 <= self.Hmax <= dimension:
            raise ValueError(f"max_hidden must be in [1, dimension={dimension}], got {self.Hmax}")
        if not 1 <= init_hidden <= self.Hmax:
            raise ValueError(f"init_hidden must be in [1, max_hidden={self.Hmax}], got {init_hidden}")
        self.lam, self.lo, self.hi = forget, low_energy, high_energy
        self.device = torch.device(device)
        self.states: dict[str, PrincipalCompState] = {}

    def update(self, streams: dict[str, torch.Tensor]) -> dict[str, PrincipalCompState]:
        keys = list(streams)
        K, D, H = len(keys), self.D, self.Hmax
        dev = self.device
        # the per-key states and the padded record block are assembled on the host and moved in
        # one copy each (per-key device writes cost ~6 small copies per key: 2,048 keys took 0.4 s)
        W = torch.zeros((K, H, D), dtype=torch.float64)
        E = torch.ones((K, H), dtype=torch.float64)                       # hidden unit energy
        he = torch.zeros((K, H), dtype=torch.float64)                     # hidden energy (running mean)
        ve = torch.zeros(K, dtype=torch.float64)
        cnt = torch.zeros(K, dtype=torch.float64)
        nh = torch.full((K,), self.H0, dtype=torch.long)
        for k, key in enumerate(keys):
            st = self.states.get(key)
            if st is None:
                continue                      # fresh key: the first H0 basis vectors, unit energies
            h = st.num_hidden
            W[k, :h] = st.components.cpu()
            E[k, :h] = torch.tensor(st.hidden_unit_energy, dtype=torch.float64)
            he[k, :h] = torch.tensor(st.hidden_energy, dtype=torch.float64)
            ve[k], cnt[k], nh[k] = st.visible_energy, float(st.count), h
        fresh = torch.tensor([key not in self.states for key in keys], dtype=torch.bool)
        if bool(fresh.any()):
            W[fresh, : self.H0] = torch.eye(D, dtype=torch.float64)[: self.H0]
        seqs = [torch.as_tensor(streams[k], dtype=torch.float64) for k in keys]
        lens = torch.tensor([x.shape[0] for x in seqs], dtype=torch.long)
        T = int(lens.max()) if K else 0
        if K and all(x.device == dev for x in seqs) and dev.type == "cuda":
            X = torch.nn.utils.rnn.pad_sequence(seqs, batch_first=True)           # already on the device
        else:
            X = torch.zeros((K, T, D), dtype=torch.float64)
            for k, x in enumerate(seqs):
                X[k, : x.shape[0]] = x.cpu()
            X = X.to(dev)
        W, E, he, ve, cnt, nh, lens = (t.to(dev) for t in (W, E, he, ve, cnt, nh, lens))
        eyeD = torch.eye(D, dtype=torch.float64, device=dev)
        hidx = torch.arange(H, device=dev).view(1, -1)
        if dev.type == "cuda" and D <= 64 and H <= D and K:
            # K24 (pca.hip): one wave per key runs its whole stream in one launch
            from .. import _native
            nh32 = nh.int()
            _native.C().spirit_update(X, lens.int(), W, E, he, ve, cnt, nh32, float(self.lam), float(self.lo),
                                      float(self.hi))
            nh, T = nh32.long(), 0
        for t in range(T):
            live = (lens > t)
            x = X[:, t].clone()                                           # [K, D]
            y_all = torch.zeros((K, H), dtype=torch.float64, device=dev)
            for i in range(H):
                act = live & (nh > i)
                if not bool(act.any()):
                    break
                w = W[:, i]
                y = (w * x).sum(1)
                Ei = torch.where(act, self.lam * E[:, i] + y * y, E[:, i])
                err = x - y.view(-1, 1) * w
                w_new = w + err * (y / Ei.clamp_min(1e-300)).view(-1, 1)
                W[:, i] = torch.where(act.view(-1, 1), w_new, w)
                E[:, i] = Ei
                x = torch.where(act.view(-1, 1), x - W[:, i] * y.view(-1, 1), x)
                y_all[:, i] = torch.where(act, y, torch.zeros_like(y))
            xin = X[:, t]
            vn = (xin * xin).sum(1)
            ve = torch.where(live, (cnt * ve + vn) / (cnt + 1), ve)
            he = torch.where(live.view(-1, 1) & (hidx < nh.view(-1, 1)), (cnt.view(-1, 1) * he + y_all ** 2) /
                             (cnt.view(-1, 1) + 1), he)
            tot = (he * (hidx < nh.view(-1, 1))).sum(1)
            grow = live & (tot < self.lo * ve) & (nh < H)
            shrink = live & (tot > self.hi * ve) & (nh > 1)
            if bool(grow.any()):
                gi = grow.nonzero().view(-1)
                W[gi, nh[gi]] = eyeD[nh[gi]]                              # new unit = next basis vector
                E[gi, nh[gi]] = 1.0
                he[gi, nh[gi]] = 0.0
                nh = torch.where(grow, nh + 1, nh)
            if bool(shrink.any()):
                nh = torch.where(shrink, nh - 1, nh)
            cnt = torch.where(live, cnt + 1, cnt)
        nh_l, cnt_l, ve_l = nh.tolist(), cnt.tolist(), ve.tolist()        # one copy back per array
        he_l, E_l, W_h = he.tolist(), E.tolist(), W.cpu()
        for k, key in enumerate(keys):
            h = int(nh_l[k])
            self.states[key] = PrincipalCompState(key, D, h, int(cnt_l[k]), [float(ve_l[k])] + he_l[k][:h],
                                                  E_l[k][:h], W_h[k, :h].clone())
        return self.states
