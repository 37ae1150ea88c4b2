"""K27 fused Linear + bias + activation (csrc/kernels/mlp.hip) as an autograd op.

``linear_act(x, W, b, act)`` = ``act(x @ W.T + b)``.  On the GPU the forward is ONE MFMA kernel with
the bias and activation applied in the accumulator epilogue (torch: addmm + a separate activation
pass over [M, N]).  The backward is one MFMA kernel forming ``dZ = dY * act'(Y)`` in its tiles and
reducing ``dW = dZ^T X`` and the bias gradient over row slices (a fixed-order slice sum after it),
then ``dX = dZ W`` on the forward MFMA kernel (layers up to 64 x 64, or up to 512 x 512 at <= 4,096
rows; the library GEMM for ``dW`` reduced all M rows inside one or two output tiles).  Wider layers: one fused ``dZ`` + bias-gradient
pass, then two hipBLASLt GEMMs.  CPU
tensors run the plain PyTorch composition (the numerics oracle of the GPU tests).

Reference: FeedForwardNetwork layer construction, P/supv/tnn.py:100-145.
"""
from __future__ import annotations

import os

import torch

from .. import _native

# layers up to this width (both N and K) take the fused weight-gradient backward (one 64 x 64 dW
# tile per row slice: the reference's networks, e.g. R/tnn_bo.properties 8-wide); wider layers re-read
# their inputs per tile there and use the fused dZ pass + hipBLASLt GEMMs instead
FUSED_BWD_MAX = int(os.environ.get("AVMI_FUSED_BWD_MAX", "64"))
# ... and at small row counts up to this width too: there the re-reads are a few hundred KB and the
# two library GEMMs cost 13-20 us each at 256 x 128 x 128 (the DQN's layers: a graphed update 334 ->
# 273 us, the autoencoder step 187 -> 160 us; profiles/r6_rl_bwd_ab.jsonl)
FUSED_BWD_SMALL_M, FUSED_BWD_SMALL_MAX = 4096, 512

ACT_CODES = {None: 0, "none": 0, "relu": 1, "sigmoid": 2, "tanh": 3, "leakyRelu": 4, "elu": 5}


def _act_torch(z: torch.Tensor, code: int) -> torch.Tensor:
    if code == 1:
        return torch.relu(z)
    if code == 2:
        return torch.sigmoid(z)
    if code == 3:
        return torch.tanh(z)
    if code == 4:
        return torch.nn.functional.leaky_relu(z, 0.01)
    if code == 5:
        return torch.nn.functional.elu(z)
    return z


class _LinearAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, b, code):
        C = _native.C()
        y = C.linear_act_fwd(x, W, b, code)
        ctx.save_for_backward(x, W, y)
        ctx.code = code
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, W, y = ctx.saved_tensors
        N, K = W.shape
        M = x.shape[0]
        if (N <= FUSED_BWD_MAX and K <= FUSED_BWD_MAX) or \
                (M <= FUSED_BWD_SMALL_M and N <= FUSED_BWD_SMALL_MAX and K <= FUSED_BWD_SMALL_MAX):
            gx, gW, db = _native.C().linear_act_backward(gy.contiguous(), y, x, W, ctx.code,
                                                         bool(ctx.needs_input_grad[0]))
            return gx, (gW if ctx.needs_input_grad[1] else None), (db if ctx.has_b else None), None
        dz, db = _native.C().linear_act_bwd(gy.contiguous(), y, ctx.code)
        gx = dz @ W if ctx.needs_input_grad[0] else None
        gW = dz.t() @ x if ctx.needs_input_grad[1] else None
        return gx, gW, (db if ctx.has_b else None), None


def linear_act(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor | None, act: str | int | None) -> torch.Tensor:
    code = act if isinstance(act, int) else ACT_CODES[act]
    if x.is_cuda and x.dtype == torch.float32 and x.dim() == 2:
        return _LinearAct.apply(x.contiguous(), W, b, code)
    return _act_torch(torch.nn.functional.linear(x, W, b), code)
