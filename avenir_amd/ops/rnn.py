"""Fused LSTM (K27): persistent HIP recurrence kernel + library GEMMs for the parallel parts.

The reference's only GPU-addressable model is the PyTorch LSTM of ``LstmNetwork``
(P/supv/lstm.py:42-378, SURVEY.md §3.5: hidden 100, 2 layers, seq_len 5).  On MI355X the split is:

* ``x·W_ihᵀ + b_ih + b_hh`` for every timestep at once — one hipBLASLt GEMM (K = input size);
* the sequential recurrence — ONE launch of ``lstm_fwd_kernel`` (csrc/kernels/rnn.hip): each
  workgroup carries 16–64 sequences through all timesteps with W_hh resident in VGPRs as bf16
  MFMA fragments and the cell state in registers (no per-timestep launches);
* backward — ONE launch of ``lstm_bwd_kernel`` for the dz / dh / dc recurrence, then the weight
  gradients ``Σ_t dz_tᵀ h_{t-1}``, ``dzᵀ x`` and ``dx = dz·W_ih`` as GEMMs over all B·T rows.

Numerics: the recurrent product runs in bf16 with fp32 accumulation (gate math, cell state and
all outputs fp32), i.e. the usual mixed-precision LSTM; ``lstm_reference`` is the fp32 oracle.
Hidden sizes above 128 (beyond the register-resident design) use PyTorch's MIOpen LSTM on the
GPU; that is the only non-kernel path and it is selected by shape, never by a missing extension.
"""
from __future__ import annotations

import math

import torch

from .. import _native

MAX_FUSED_HIDDEN = 128


def padded_hidden(H: int) -> int:
    return 32 if H <= 32 else (64 if H <= 64 else 128)


def _pad_whh(w_hh: torch.Tensor, H: int) -> torch.Tensor:
    HP = padded_hidden(H)
    wp = torch.zeros((4, HP, HP), device=w_hh.device, dtype=torch.float32)
    wp[:, :H, :H] = w_hh.detach().float().view(4, H, H)
    return wp


def pack_whh(w_hh: torch.Tensor, H: int) -> tuple[torch.Tensor, torch.Tensor]:
    """W_hh [4H, H] -> (forward fragments [NW,4,KS,64,8], backward fragments [NW,4KS,64,8]) in bf16.

    Forward B-operand of v_mfma_f32_16x16x32_bf16 for wave w, gate g, k-step ks: lane q*16+col,
    element j holds W_hh[g*H + 16w + col, 32ks + 8q + j].  Backward (dh = dz·W_hh, k over the 4·HP
    gate rows): lane q*16+col, element j of k-step s holds W_hh[g*H + 32(s%KS) + 8q + j, 16w + col]
    with g = s // KS.
    """
    HP = padded_hidden(H)
    KS, NW = HP // 32, HP // 16
    wp = _pad_whh(w_hh, H)
    fwd = wp.view(4, NW, 16, KS, 4, 8).permute(1, 0, 3, 4, 2, 5).contiguous()
    bwd = wp.view(4, KS, 4, 8, NW, 16).permute(4, 0, 1, 2, 5, 3).contiguous().view(NW, 4 * KS, 4, 16, 8)
    return fwd.to(torch.bfloat16).contiguous(), bwd.to(torch.bfloat16).contiguous()


def lstm_cell_reference(x, h, c, w_ih, w_hh, b):
    z = x @ w_ih.t() + h @ w_hh.t() + (b if b is not None else 0.0)
    i, f, g, o = z.chunk(4, dim=-1)
    i, f, g, o = torch.sigmoid(i), torch.sigmoid(f), torch.tanh(g), torch.sigmoid(o)
    c = f * c + i * g
    return o * torch.tanh(c), c


def lstm_reference(x, w_ih, w_hh, b=None, h0=None, c0=None):
    """fp32 oracle of one LSTM layer (batch-first): returns (hseq [B,T,H], (h_T, c_T))."""
    B, T, _ = x.shape
    H = w_hh.shape[1]
    h = h0 if h0 is not None else x.new_zeros(B, H)
    c = c0 if c0 is not None else x.new_zeros(B, H)
    outs = []
    for t in range(T):
        h, c = lstm_cell_reference(x[:, t], h, c, w_ih, w_hh, b)
        outs.append(h)
    return torch.stack(outs, 1), (h, c)


class _LstmLayer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w_ih, w_hh, b, h0, c0):
        B, T, I = x.shape
        H = w_hh.shape[1]
        mod = _native.C()
        x2 = x.reshape(B * T, I)
        if b is not None:
            xw = torch.addmm(b.unsqueeze(0), x2, w_ih.t())
        else:
            xw = x2 @ w_ih.t()
        xw = xw.view(B, T, 4 * H)
        frag, frag_t = pack_whh(w_hh, H)
        need = any(ctx.needs_input_grad)
        outs = mod.lstm_forward(xw, frag, h0, c0, H, bool(need))
        hseq, cseq = outs[0], outs[1]
        if need:
            ctx.save_for_backward(x, w_ih, w_hh, hseq, cseq, outs[2], h0, c0, frag_t)
        ctx.has_b = b is not None
        return hseq, hseq[:, -1], cseq[:, -1]

    @staticmethod
    def backward(ctx, dhseq, dhn, dcn):
        x, w_ih, w_hh, hseq, cseq, gates, h0, c0, frag_t = ctx.saved_tensors
        B, T, I = x.shape
        H = w_hh.shape[1]
        if dhseq is None:
            dhseq = torch.zeros_like(hseq)
        dz, dh0, dc0 = _native.C().lstm_backward(dhseq.contiguous(), gates, cseq, c0,
                                                 None if dhn is None else dhn.contiguous(),
                                                 None if dcn is None else dcn.contiguous(), frag_t, H)
        dz2 = dz.view(B * T, 4 * H)
        dx = (dz2 @ w_ih).view(B, T, I) if ctx.needs_input_grad[0] else None
        dw_ih = dz2.t() @ x.reshape(B * T, I) if ctx.needs_input_grad[1] else None
        dw_hh = None
        if ctx.needs_input_grad[2]:
            first = h0.unsqueeze(1) if h0 is not None else hseq.new_zeros(B, 1, H)
            hprev = torch.cat([first, hseq[:, :-1]], 1).reshape(B * T, H)
            dw_hh = dz2.t() @ hprev
        db = dz2.sum(0) if ctx.has_b and ctx.needs_input_grad[3] else None
        return (dx, dw_ih, dw_hh, db, dh0 if h0 is not None else None, dc0 if c0 is not None else None)


def lstm_layer(x, w_ih, w_hh, b=None, h0=None, c0=None):
    """One batch-first LSTM layer: (hseq [B,T,H], h_T [B,H], c_T [B,H]).

    GPU tensors with H <= 128 run the fused HIP kernels (raising if the extension is missing);
    CPU tensors run the fp32 reference.
    """
    H = w_hh.shape[1]
    if x.is_cuda and H <= MAX_FUSED_HIDDEN:
        x = x.float().contiguous()
        h0 = None if h0 is None else h0.float().contiguous()
        c0 = None if c0 is None else c0.float().contiguous()
        return _LstmLayer.apply(x, w_ih, w_hh, b, h0, c0)
    hseq, (h, c) = lstm_reference(x, w_ih, w_hh, b, h0, c0)
    return hseq, h, c


class FusedLSTM(torch.nn.Module):
    """Batch-first multi-layer LSTM with ``torch.nn.LSTM``'s parameter names and init, so state
    dicts load either way.  ``forward(x, (h0, c0)) -> (out, (h_n, c_n))``."""

    def __init__(self, input_size: int, hidden_size: int, num_layers: int = 1, bias: bool = True,
                 batch_first: bool = True, dropout: float = 0.0):
        super().__init__()
        if not batch_first:
            raise ValueError("FusedLSTM is batch-first")
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.bias, self.dropout, self.batch_first = bias, float(dropout), True
        H = hidden_size
        for l in range(num_layers):
            i = input_size if l == 0 else H
            setattr(self, f"weight_ih_l{l}", torch.nn.Parameter(torch.empty(4 * H, i)))
            setattr(self, f"weight_hh_l{l}", torch.nn.Parameter(torch.empty(4 * H, H)))
            if bias:
                setattr(self, f"bias_ih_l{l}", torch.nn.Parameter(torch.empty(4 * H)))
                setattr(self, f"bias_hh_l{l}", torch.nn.Parameter(torch.empty(4 * H)))
        self.reset_parameters()

    def reset_parameters(self):
        k = 1.0 / math.sqrt(self.hidden_size)
        for p in self.parameters():
            torch.nn.init.uniform_(p, -k, k)

    def _flat_weights(self):
        ws = []
        for l in range(self.num_layers):
            ws += [getattr(self, f"weight_ih_l{l}"), getattr(self, f"weight_hh_l{l}")]
            if self.bias:
                ws += [getattr(self, f"bias_ih_l{l}"), getattr(self, f"bias_hh_l{l}")]
        return ws

    def forward(self, x, hx=None):
        H, L = self.hidden_size, self.num_layers
        if x.is_cuda and H > MAX_FUSED_HIDDEN:   # beyond the register-resident kernel: MIOpen
            if hx is None:
                z = x.new_zeros(L, x.shape[0], H)
                hx = (z, z)
            out, h, c = torch.lstm(x, hx, self._flat_weights(), self.bias, L, self.dropout, self.training,
                                   False, True)
            return out, (h, c)
        hs, cs = [], []
        out = x
        for l in range(L):
            b = None
            if self.bias:
                b = getattr(self, f"bias_ih_l{l}") + getattr(self, f"bias_hh_l{l}")
            h0 = hx[0][l] if hx is not None else None
            c0 = hx[1][l] if hx is not None else None
            out, h, c = lstm_layer(out, getattr(self, f"weight_ih_l{l}"), getattr(self, f"weight_hh_l{l}"), b, h0, c0)
            hs.append(h)
            cs.append(c)
            if self.dropout > 0 and self.training and l < L - 1:
                out = torch.nn.functional.dropout(out, self.dropout, True)
        return out, (torch.stack(hs), torch.stack(cs))
