"""Fused LSTM (K27): persistent HIP recurrence kernel + library GEMMs for the parallel parts.

The reference's only GPU-addressable model is the PyTorch LSTM of ``LstmNetwork``
(P/supv/lstm.py:42-378, SURVEY.md §3.5: hidden 100, 2 layers, seq_len 5).  On MI355X the split is:

* forward — ONE launch of ``lstm_fwd_kernel`` per layer (csrc/kernels/rnn.hip): each workgroup
  carries 16–32 sequences through all timesteps with [W_hh | W_ih] resident in VGPRs as bf16 MFMA
  fragments, the cell state in registers and the input projection fused into the recurrent
  product (no per-timestep launches, no B·T·4H projection tensor);
* backward — ONE launch of ``lstm_bwd_kernel`` for the dz / dh / dc recurrence, then ONE GEMM
  ``dzᵀ·hx`` over all B·T rows for dW_hh, dW_ih and db together (``hx`` = the forward's MFMA
  B-operand rows [h_{t-1} | x_t | 1]) and one GEMM for ``dx = dz·W_ih``.

Numerics (mixed precision): GEMM operands and the B·T·4H-sized intermediates (xw, saved gates,
gate gradients) are bf16 with fp32 accumulation; gate math, the cell state, h outputs and the
weight gradients are fp32.  ``lstm_reference`` is the fp32 oracle.
Hidden or input sizes above 128 (beyond the register-resident design) use PyTorch's MIOpen LSTM
on the GPU; that path is selected by shape, never by a missing extension.

``precision="fp32"`` (the DEFAULT, the reference's numerics: P/supv/lstm.py trains an fp32
``nn.LSTM``) runs the fp32 twin of the kernels (csrc/kernels/rnn_f32.hip): the recurrence on
v_mfma_f32_16x16x4_f32 with W_hh resident in VGPRs as f32 fragments, every stored intermediate
fp32, and the input projection x·W_ihᵀ + b of all timesteps as one fp32 GEMM ahead of it (the f32
fragments of W_hh alone take HP VGPRs) — except for inputs of <= 8 features (the reference's first
layer), whose projection runs inside the recurrence as two extra MFMA k-steps per gate; one
``lstm_pack_f32`` launch re-lays the parameters per optimizer step.  Backward: one fp32 recurrence
launch writing dz in torch gate order + ONE fp32 GEMM dzᵀ·[h_{t-1} | x | 1] (rows written by the
forward) for dW_hh, dW_ih and db together, and dx = dz·W_ih.  ``precision="bf16"`` opts into the
mixed-precision kernel above.  Both are checked against the fp32 oracle and ``nn.LSTM``
(tests/test_rnn.py).
"""
from __future__ import annotations

import math

import weakref

import torch

from .. import _native
from ..utils.params import param_epoch

MAX_FUSED_HIDDEN = 128


def padded_hidden(H: int) -> int:
    return 32 if H <= 32 else (64 if H <= 64 else 128)


def pack_weights(w_ih: torch.Tensor, w_hh: torch.Tensor, H: int) -> tuple[torch.Tensor, torch.Tensor]:
    """(W_ih [4H, I], W_hh [4H, H]) -> bf16 MFMA A-fragments (forward [NW,4,KS+IS,4,16,8], backward
    [NW,4KS,4,16,8]).

    The kernels compute transposed products (zᵀ = [W_hh | W_ih]·[h; x]ᵀ, dhᵀ = W_hhᵀ·dzᵀ), so these
    are the A-operands of v_mfma_f32_16x16x32_bf16.  Forward, wave w, gate g, k-step ks: lane
    q*16+col, element j holds Wcat[g*H + 16w + col, 32ks + 8q + j] where Wcat = [W_hh (HP cols) |
    W_ih (IP cols)].  Backward (k over the 4·HP gate rows): lane q*16+col, element j of k-step s
    holds W_hh[g*H + 32(s%KS) + 8q + j, 16w + col] with g = s // KS.  Padding is zero.
    """
    I = w_ih.shape[1]
    HP, IP = padded_hidden(H), padded_hidden(I)
    KS, NW, KT = HP // 32, HP // 16, (HP + IP) // 32
    wcat = torch.zeros((4, HP, HP + IP), device=w_hh.device, dtype=torch.float32)
    wcat[:, :H, :H] = w_hh.detach().float().view(4, H, H)
    wcat[:, :H, HP:HP + I] = w_ih.detach().float().view(4, H, I)
    fwd = wcat.view(4, NW, 16, KT, 4, 8).permute(1, 0, 3, 4, 2, 5)
    wp = wcat[:, :, :HP].contiguous()
    bwd = wp.view(4, KS, 4, 8, NW, 16).permute(4, 0, 1, 2, 5, 3).contiguous().view(NW, 4 * KS, 4, 16, 8)
    return fwd.to(torch.bfloat16).contiguous(), bwd.to(torch.bfloat16).contiguous()


def pack_weights_f32(w_hh: torch.Tensor, H: int) -> tuple[torch.Tensor, torch.Tensor]:
    """W_hh [4H, H] -> fp32 A-fragments of v_mfma_f32_16x16x4_f32 (forward [NW, 4, HP/4, 64],
    backward [NW, HP, 64]).  Forward, wave w, gate g, k-step s: lane q*16 + col holds
    W_hh[g*H + 16w + col, 4s + q].  Backward (dhᵀ = W_hhᵀ·dzᵀ, k over the 4·HP gate rows gate-major,
    k = g·HP + u): lane q*16 + col of k-step s holds W_hh[row of k = 4s + q, 16w + col].  Padding 0."""
    HP = padded_hidden(H)
    NW, KS4 = HP // 16, HP // 4
    wp = torch.zeros((4, HP, HP), device=w_hh.device, dtype=torch.float32)
    wp[:, :H, :H] = w_hh.detach().float().view(4, H, H)
    fwd = wp.view(4, NW, 16, KS4, 4).permute(1, 0, 3, 4, 2).contiguous().view(NW, 4, KS4, 64)
    bwd = wp.reshape(4 * HP, HP).view(HP, 4, NW, 16).permute(2, 0, 1, 3).contiguous().view(NW, HP, 64)
    return fwd, bwd


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


_ORDER_CACHE: dict = {}


def kernel_gate_order(H: int, device) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Kernel column order of the 4·HP gate columns: kc = 64·w + 16·g + i for unit u = 16·w + i.

    Returns (valid_kc, torch_row, inv): ``valid_kc`` are the kernel columns of real units,
    ``torch_row`` the matching row g·H + u of W_ih / W_hh / b, and ``inv[g·H + u]`` the kernel
    column of every torch row (for gathering gradients back)."""
    key = (H, str(device))
    if key not in _ORDER_CACHE:
        HP = padded_hidden(H)
        kc = torch.arange(4 * HP)
        w, g, i = kc // 64, (kc % 64) // 16, kc % 16
        u = 16 * w + i
        ok = u < H
        valid_kc = kc[ok]
        torch_row = (g * H + u)[ok]
        inv = torch.empty(4 * H, dtype=torch.long)
        inv[torch_row] = valid_kc
        _ORDER_CACHE[key] = tuple(t.to(device) for t in (valid_kc, torch_row, inv))
    return _ORDER_CACHE[key]


def to_kernel_order(w: torch.Tensor, H: int) -> torch.Tensor:
    """[4H, ...] gate-major rows (torch.nn.LSTM order) -> [4HP, ...] kernel order, padded with 0."""
    valid_kc, torch_row, _ = kernel_gate_order(H, w.device)
    out = w.new_zeros((4 * padded_hidden(H),) + tuple(w.shape[1:]))
    out[valid_kc] = w[torch_row]
    return out


class _PackCacheF32:
    """The fp32 layer's re-laid parameters (``lstm_pack_f32``: W_hh fragments, W_hhᵀ fragments,
    kernel-order W_ih and b_ih + b_hh — ONE launch), keyed on the four tensors' (storage, version)
    and the optimizer-step epoch (utils/params.py: fused optimizers do not bump versions):
    inference re-uses them across calls, training re-packs once per optimizer step.  Inside a
    HIP-graph capture the pack is recorded, so replays re-pack."""

    def __init__(self, size: int = 16):
        self.size, self.d = size, {}

    @staticmethod
    def _pack(w_ih, w_hh, b_ih, b_hh):
        c = lambda t: None if t is None else t.detach().float().contiguous()
        packed = tuple(_native.C().lstm_pack_f32(c(w_ih), c(w_hh), c(b_ih), c(b_hh)))
        # W_ih^T [I, 4H] for dx = dz W_ih on the f32-MFMA GEMM (wide inputs only)
        wt = c(w_ih).t().contiguous() if w_ih.shape[1] > 8 else None
        return packed + (wt,)

    def get(self, w_ih, w_hh, b_ih, b_hh):
        ts = (w_ih, w_hh, b_ih, b_hh)
        if torch.cuda.is_current_stream_capturing():
            return self._pack(*ts)
        key = (param_epoch(),) + tuple((t.data_ptr(), t._version, tuple(t.shape)) if t is not None else None
                                       for t in ts)
        hit = self.d.get(key)
        # the entry must belong to THESE live tensors: a freed tensor's memory (same address, shape
        # and version 0) may be re-used by a new one with different values
        if hit is not None and all((r is None and t is None) or (r is not None and r() is t)
                                   for r, t in zip(hit[0], ts)):
            return hit[1]
        if len(self.d) >= self.size:
            self.d.pop(next(iter(self.d)))
        packed = self._pack(*ts)
        self.d[key] = (tuple(None if t is None else weakref.ref(t) for t in ts), packed)
        return packed


_packs_f32 = _PackCacheF32()


class _FragCache:
    """Packed weight fragments keyed on the weights' (storage, version): inference re-uses them
    across calls, training re-packs once per optimizer step (the forward's pack serves the
    backward).  Inside a HIP-graph capture the pack is always recorded, so replays re-pack."""

    def __init__(self, size: int = 16):
        self.size, self.d = size, {}

    def get(self, w_ih: torch.Tensor, w_hh: torch.Tensor, H: int):
        if torch.cuda.is_current_stream_capturing():
            return pack_weights(w_ih, w_hh, H)
        key = (param_epoch(), w_ih.data_ptr(), w_ih._version, tuple(w_ih.shape), w_hh.data_ptr(), w_hh._version, H)
        hit = self.d.get(key)
        if hit is not None and hit[0]() is w_ih and hit[1]() is w_hh:     # the same live tensors
            return hit[2]
        if len(self.d) >= self.size:
            self.d.pop(next(iter(self.d)))
        frags = pack_weights(w_ih, w_hh, H)
        self.d[key] = (weakref.ref(w_ih), weakref.ref(w_hh), frags)
        return frags


_frags = _FragCache()


def _mm_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """bf16 x bf16 -> fp32 GEMM (hipBLASLt, fp32 accumulate and output)."""
    return torch.mm(a, b, out_dtype=torch.float32)


class _LstmLayer(torch.autograd.Function):
    """One layer: forward = ONE kernel launch (input projection fused into the recurrence); backward
    = one kernel launch + one GEMM for all weight and bias gradients (dzᵀ·hx) + one GEMM for dx.
    The B·T·4H-sized tensors (saved gates, dz) and hx are bf16; cell state, h outputs and the
    weight gradients are fp32."""

    @staticmethod
    def forward(ctx, x, w_ih, w_hh, b, h0, c0):
        B, T, I = x.shape
        H = w_hh.shape[1]
        HP = padded_hidden(H)
        frag, frag_t = _frags.get(w_ih, w_hh, H)
        bias = to_kernel_order(b.detach().float(), H) if b is not None else x.new_zeros(4 * HP)
        need = any(ctx.needs_input_grad)
        outs = _native.C().lstm_forward(x, frag, bias, h0, c0, H, bool(need))
        hseq, cseq = outs[0], outs[1]
        if need:
            w_ih_k = to_kernel_order(w_ih.detach(), H).to(torch.bfloat16)    # [4HP, I] for dx
            ctx.save_for_backward(w_ih_k, cseq, outs[2], outs[3], c0, frag_t)
        ctx.has_b, ctx.dims = b is not None, (B, T, I, H)
        return hseq, hseq[:, -1], cseq[:, -1, :H]

    @staticmethod
    def backward(ctx, dhseq, dhn, dcn):
        w_ih_k, cseq, gates, hx, c0, frag_t = ctx.saved_tensors
        B, T, I, H = ctx.dims
        HP, IP = padded_hidden(H), padded_hidden(I)
        _, _, inv = kernel_gate_order(H, cseq.device)
        if dhseq is None:
            dhseq = cseq.new_zeros(B, T, H)
        dz, dh0, dc0 = _native.C().lstm_backward(dhseq.contiguous(), gates, cseq, c0,
                                                 None if dhn is None else dhn.contiguous(),
                                                 None if dcn is None else dcn.contiguous(), frag_t, H)
        dz2 = dz.view(B * T, 4 * HP)                                 # bf16, kernel order
        dx = _mm_f32(dz2, w_ih_k).view(B, T, I) if ctx.needs_input_grad[0] else None
        dw_ih = dw_hh = db = None
        if any(ctx.needs_input_grad[1:4]):
            dwcat = _mm_f32(dz2.t(), hx.view(B * T, HP + IP)).index_select(0, inv)   # [4H, HP+IP]
            dw_hh = dwcat[:, :H].contiguous()
            dw_ih = dwcat[:, HP:HP + I].contiguous()
            if ctx.has_b:
                # hx carries a ones column at HP + I when the input is narrower than its padding
                db = dwcat[:, HP + I].contiguous() if I < IP else dz2.sum(0, dtype=torch.float32).index_select(0, inv)
        need = ctx.needs_input_grad
        return dx, dw_ih, dw_hh, db, (dh0 if need[4] else None), (dc0 if need[5] else None)


#: the fp32 layer's plain GEMMs: "mfma" = the wide-input projection and dx on the f32-MFMA tile
#: kernel of mlp.hip (linear_act_fwd: exact-f32 v_mfma_f32_32x32x2_f32, bias in the epilogue) and
#: the weight-gradient product on gemm.hip's split-K kernel (gemm_tn); "blas" = hipBLASLt for all
LSTM_GEMM = __import__("os").environ.get("AVMI_LSTM_GEMM", "mfma")


class _LstmLayerF32(torch.autograd.Function):
    """One fp32 layer.  Forward: ONE pack launch (skipped while the parameters are unchanged) + ONE
    recurrence launch — for inputs of <= 8 features the input projection runs inside it (extra MFMA
    k-steps), wider inputs get one fp32 projection GEMM (kernel gate order, biases fused) ahead of
    it.  The recurrence also writes the [h_{t-1} | x_t | 1] rows for the backward.  Backward: one
    recurrence launch writing dz in torch gate order, then ONE fp32 GEMM dzᵀ·[h_{t-1} | x | 1] for
    dW_hh, dW_ih and the bias gradient together, and dx = dz·W_ih."""

    @staticmethod
    def forward(ctx, x, w_ih, w_hh, b_ih, b_hh, h0, c0):
        B, T, I = x.shape
        H = w_hh.shape[1]
        HP = padded_hidden(H)
        frag, frag_t, w_ih_k, bias, wxfrag, w_ih_t = _packs_f32.get(w_ih, w_hh, b_ih, b_hh)
        need = any(ctx.needs_input_grad)
        if I <= 8:
            outs = _native.C().lstm_forward_f32(None, frag, h0, c0, H, bool(need), x=x, wxfrag=wxfrag, biask=bias)
        else:
            x2 = x.reshape(B * T, I)
            xw = (_native.C().linear_act_fwd(x2, w_ih_k, bias, 0) if LSTM_GEMM == "mfma"
                  else torch.addmm(bias, x2, w_ih_k.t())).view(B, T, 4 * HP)
            outs = _native.C().lstm_forward_f32(xw, frag, h0, c0, H, bool(need), x=x if need else None)
        hseq, cseq = outs[0], outs[1]
        if need:
            ctx.save_for_backward(w_ih, cseq, outs[2], outs[3], c0, frag_t, w_ih_t)
        ctx.dims = (B, T, I, H)
        return hseq, hseq[:, -1], cseq[:, -1, :H]

    @staticmethod
    def backward(ctx, dhseq, dhn, dcn):
        w_ih, cseq, gates, hx, c0, frag_t, w_ih_t = ctx.saved_tensors
        B, T, I, H = ctx.dims
        if dhseq is None:
            dhseq = cseq.new_zeros(B, T, H)
        dz, dh0, dc0 = _native.C().lstm_backward_f32(dhseq.contiguous(), gates, cseq, c0,
                                                     None if dhn is None else dhn.contiguous(),
                                                     None if dcn is None else dcn.contiguous(), frag_t, H)
        dz2 = dz.view(B * T, 4 * H)                                    # fp32, torch gate order
        need = ctx.needs_input_grad
        dx = None
        if need[0]:
            if LSTM_GEMM == "mfma" and w_ih_t is not None:
                dx = _native.C().linear_act_fwd(dz2, w_ih_t, None, 0).view(B, T, I)
            else:
                dx = (dz2 @ w_ih.detach().float()).view(B, T, I)
        dw_ih = dw_hh = db = None
        if any(need[1:5]):
            hx2 = hx.view(B * T, H + I + 1)
            dwcat = (_native.C().gemm_tn(dz2, hx2) if LSTM_GEMM == "mfma"
                     else dz2.t() @ hx2)                                 # [4H, H + I + 1]
            dw_hh = dwcat[:, :H] if need[2] else None
            dw_ih = dwcat[:, H:H + I] if need[1] else None
            db = dwcat[:, H + I] if (need[3] or need[4]) else None
        # views of one GEMM output (autograd lays each out like its parameter); the same bias
        # gradient for both biases (autograd copies it when both accumulate)
        return (dx, dw_ih, dw_hh, db if need[3] else None, db if need[4] else None,
                (dh0 if need[5] else None), (dc0 if need[6] else None))


def lstm_layer(x, w_ih, w_hh, b=None, h0=None, c0=None, precision: str = "fp32", b_hh=None):
    """One batch-first LSTM layer: (hseq [B,T,H], h_T [B,H], c_T [B,H]).  ``b`` (+ ``b_hh``, the
    torch.nn.LSTM split of the bias; added together) is the gate bias.

    GPU tensors with H <= 128 run the fused HIP kernels (raising if the extension is missing):
    ``precision="fp32"`` the fp32 recurrence (any input size: the input projection is a GEMM),
    ``"bf16"`` the mixed-precision kernel (input size <= 128 too).  CPU tensors run the fp32
    reference."""
    H = w_hh.shape[1]
    if x.is_cuda and H <= MAX_FUSED_HIDDEN and (precision == "fp32" or x.shape[-1] <= MAX_FUSED_HIDDEN):
        x = x.float().contiguous()
        h0 = None if h0 is None else h0.float().contiguous()
        c0 = None if c0 is None else c0.float().contiguous()
        if precision == "fp32":
            return _LstmLayerF32.apply(x, w_ih, w_hh, b, b_hh, h0, c0)
        if b_hh is not None:
            b = b_hh if b is None else b + b_hh
        return _LstmLayer.apply(x, w_ih, w_hh, b, h0, c0)
    if b_hh is not None:
        b = b_hh if b is None else b + b_hh
    hseq, (h, c) = lstm_reference(x, w_ih, w_hh, b, h0, c0)
    return hseq, h, c


class FusedLSTM(torch.nn.Module):
    """Batch-first multi-layer LSTM with ``torch.nn.LSTM``'s parameter names and init, so state
    dicts load either way.  ``forward(x, (h0, c0)) -> (out, (h_n, c_n))``."""

    def __init__(self, input_size: int, hidden_size: int, num_layers: int = 1, bias: bool = True,
                 batch_first: bool = True, dropout: float = 0.0, precision: str = "fp32"):
        super().__init__()
        if not batch_first:
            raise ValueError("FusedLSTM is batch-first")
        if precision not in ("bf16", "fp32", "miopen"):
            raise ValueError(f"precision must be 'fp32' (fused fp32 kernels, default), 'bf16' (fused "
                             f"mixed-precision kernel) or 'miopen' (torch.lstm), got {precision!r}")
        self.precision = precision
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
        if x.is_cuda and (H > MAX_FUSED_HIDDEN or self.precision == "miopen"
                          or (self.precision == "bf16" and self.input_size > MAX_FUSED_HIDDEN)):
            # beyond the register-resident kernels, or MIOpen requested (fp32)
            if hx is None:
                z = x.new_zeros(L, x.shape[0], H)
                hx = (z, z)
            out, h, c = torch.lstm(x, hx, self._flat_weights(), self.bias, L, self.dropout, self.training,
                                   False, True)
            return out, (h, c)
        hs, cs = [], []
        out = x
        for l in range(L):
            b_ih = getattr(self, f"bias_ih_l{l}") if self.bias else None
            b_hh = getattr(self, f"bias_hh_l{l}") if self.bias else None
            h0 = hx[0][l] if hx is not None else None
            c0 = hx[1][l] if hx is not None else None
            out, h, c = lstm_layer(out, getattr(self, f"weight_ih_l{l}"), getattr(self, f"weight_hh_l{l}"), b_ih, h0, c0,
                                   self.precision, b_hh=b_hh)
            hs.append(h)
            cs.append(c)
            if self.dropout > 0 and self.training and l < L - 1:
                out = torch.nn.functional.dropout(out, self.dropout, True)
        return out, (torch.stack(hs), torch.stack(cs))
