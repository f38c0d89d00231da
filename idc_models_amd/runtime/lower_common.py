"""Lowering helpers shared by the model families: input staging, fused head, freeze analysis."""
from __future__ import annotations

from typing import Optional

import torch

from ..ops import _native as nat
from .builder import BF16, F32, Builder, Tensor4

RELU, RELU6 = 1, 2


class FreezeInfo:
    """Which backbone layers train, and whether gradient must flow into a layer's output.

    Keras fine-tuning freezes a PREFIX (``layers[:fine_tune_at]``), so backward stops at the
    first trainable layer (phase 1 back-propagates into the head only).
    """

    def __init__(self, base, training: bool):
        self.layers = base.layers
        self.index = {id(l): i for i, l in enumerate(self.layers)}
        flags = [training and self._has_trainable(l) for l in self.layers]
        self.prefix = [0]
        for f in flags:
            self.prefix.append(self.prefix[-1] + (1 if f else 0))
        self.flags = flags

    @staticmethod
    def _has_trainable(l) -> bool:
        return bool(l.trainable) and any(p.requires_grad for p in l.trainable_params())

    def trainable(self, layer) -> bool:
        return self.flags[self.index[id(layer)]]

    def before(self, layer) -> bool:
        """Any trainable layer strictly before ``layer``."""
        return self.prefix[self.index[id(layer)]] > 0

    def at_or_before(self, layer) -> bool:
        return self.prefix[self.index[id(layer)] + 1] > 0

    def any(self) -> bool:
        return self.prefix[-1] > 0


class HeadIO:
    def __init__(self, b: Builder, U: int):
        B = b.B
        self.U = U
        self.labels = b.alloc((B, U) if U > 1 else (B,), F32)
        self.logits = b.alloc((B, U), F32)
        self.dlogits = b.alloc((B, U), F32)
        self.loss = b.alloc((1,), F32)


def emit_input(b: Builder, H: int, W: int, C: int, input_dtype, cpad: int = 8) -> (torch.Tensor, Tensor4):
    xin = b.alloc((b.B, H, W, C), input_dtype)
    x8 = b.nhwc(b.B, H, W, cpad)
    b.emit(nat.OP_INPUT, ints=(1 if input_dtype == torch.uint8 else 0, b.B, H, W, C, cpad),
           ptrs=(xin.data_ptr(), x8.ptr))
    return xin, x8


def emit_head(b: Builder, feat: Tensor4, pro: Optional[nat.BnArgs], dense, U: int, io: HeadIO,
              training: bool):
    """[pending BN + act] -> GAP -> Dense -> loss (+ dlogits when training)."""
    a = nat.HeadArgs()
    a.x, a.ldx = feat.ptr, feat.ld
    a.N, a.HW, a.C, a.U = feat.N, feat.H * feat.W, feat.C, U
    a.pro = pro if pro is not None else nat.bn_args(mode=0, act=0)
    a.w, a.b = dense.kernel.data_ptr(), nat.ptr(dense.bias if dense.use_bias else None)
    a.labels = io.labels.data_ptr()
    a.logits = io.logits.data_ptr()
    a.feats = b.alloc((feat.N, feat.C), F32).data_ptr()
    a.dlogits = io.dlogits.data_ptr() if training else 0
    a.loss = io.loss.data_ptr()
    a.loss_scale = 1.0 / float(feat.N)
    # this rank's share of an uneven global batch enters the gradient at its seed, before the
    # all-reduce (the optimizer then scales the reduced sum by a uniform 1/N)
    a.dl_scale = a.loss_scale * b.grad_weight
    a.training = 1 if training else 0
    # per-sample losses summed in sample order by the last block (deterministic, no zero-fill op)
    a.loss_vec = b.alloc((feat.N,), F32).data_ptr()
    a.ticket = b.alloc((1,), torch.int32).data_ptr()
    b.emit(nat.OP_HEAD_FWD, a)
    io.feats_ptr = a.feats
    return a


def emit_head_bwd(b: Builder, feat: Tensor4, dense, U: int, io: HeadIO, need_dA: bool):
    a = nat.HeadBwdArgs()
    a.feats, a.dlogits, a.w = io.feats_ptr, io.dlogits.data_ptr(), dense.kernel.data_ptr()
    a.N, a.HW, a.C, a.U = feat.N, feat.H * feat.W, feat.C, U
    arena = b.arena
    train_head = dense.trainable and dense.kernel.requires_grad
    a.dw = arena.grad_of(dense.kernel).data_ptr() if train_head else b.alloc((feat.C * U,), F32).data_ptr()
    a.db = arena.grad_of(dense.bias).data_ptr() if (train_head and dense.use_bias) else 0
    dA = b.nhwc(feat.N, feat.H, feat.W, feat.C, F32) if need_dA else None
    if dA is None:
        a.dA, a.ldda = b.alloc((feat.N * feat.H * feat.W * feat.C,), F32).data_ptr(), feat.C
    else:
        a.dA, a.ldda = dA.ptr, dA.ld
    a.det = 1 if b.det else 0
    b.emit(nat.OP_HEAD_BWD, a)
    if train_head:
        b.mark_grads_ready([dense.kernel] + ([dense.bias] if dense.use_bias else []))
    return dA
