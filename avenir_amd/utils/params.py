"""A process-wide counter of optimizer steps, for caches of re-laid parameters.

The framework caches packed copies of parameters (the LSTM's MFMA weight fragments, BERT's fused
Q/K/V matrix) keyed on each tensor's storage and autograd version counter.  torch's fused
optimizers (``Adam(fused=True)`` ...) update the parameters in place WITHOUT bumping their version
counter (checked: ``p._version`` stays 1 across a fused step, a foreach step bumps it), so such a
key alone would keep serving the pre-step weights.  Every ``torch.optim`` step therefore bumps
this epoch through the global step hook, and the caches include it in their keys.
"""
from __future__ import annotations

import torch
from torch.optim.optimizer import register_optimizer_step_post_hook

_EPOCH = [0]


def _bump(optimizer, args, kwargs) -> None:
    _EPOCH[0] += 1


register_optimizer_step_post_hook(_bump)


def bump_param_epoch() -> None:
    """Invalidate every packed-parameter cache: for in-place writes that bypass autograd's
    version counter (a broadcast into ``p.data``, a ``load_state_dict`` copy)."""
    _EPOCH[0] += 1


def param_epoch() -> int:
    """Number of optimizer steps taken in this process (any optimizer, any parameters)."""
    return _EPOCH[0]
