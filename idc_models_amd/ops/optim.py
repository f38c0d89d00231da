"""Fused optimizer entry points (native HIP kernel over a flat fp32 arena)."""
from __future__ import annotations

import torch

from . import _native as nat


def rmsprop_(w: torch.Tensor, g: torch.Tensor, ms: torch.Tensor, lr: float, rho: float, eps: float,
             grad_scale: float = 1.0) -> None:
    """Keras RMSprop in place: ms = rho*ms + (1-rho)*(s*g)^2; w -= lr*s*g/(sqrt(ms)+eps)."""
    assert w.is_cuda and w.dtype == torch.float32 and w.numel() % 4 == 0
    nat.require().rmsprop(w.data_ptr(), g.data_ptr(), ms.data_ptr(), w.numel(), float(lr), float(rho),
                          float(eps), float(grad_scale), nat.stream_handle())
