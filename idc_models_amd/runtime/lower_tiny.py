"""Tiny-CNN lowering (``secure_fed_model.py:84-98``).

Conv2D(32, 3x3, s2, relu) -> MaxPool 2x2 -> Dropout(.25) -> Flatten -> Dense(8, relu) ->
Dropout(.5) -> Dense(1): four launches forward (input staging, MFMA conv with bias+ReLU epilogue,
max-pool with argmax, fused dropout/MLP/loss head) and four backward (fused MLP head backward,
pool backward with the ReLU mask and bias gradient in its epilogue, conv weight gradient, dropout
stream advance).  Dropout masks are Philox-generated from (seed, step) in both directions, so
nothing is stored between forward and backward.
"""
from __future__ import annotations

import torch

from ..ops import _native as nat
from .builder import F32, Builder
from .lower_common import RELU, HeadIO, emit_input
from .lower_vgg import _pool_bwd_relu


def tiny_supported(net) -> bool:
    return all(l.trainable for l in net.layers)


def lower_tiny(b: Builder, net, U: int, input_dtype):
    b._no_det("the tiny-CNN MLP head")
    by_class = {}
    for l in net.layers:
        by_class.setdefault(l.keras_class, []).append(l)
    conv = by_class["Conv2D"][0]
    d1, d2 = by_class["Dense"]
    drops = by_class.get("Dropout", [])
    p0 = drops[0].rate if len(drops) > 0 else 0.0
    p1 = drops[1].rate if len(drops) > 1 else 0.0
    B, training = b.B, b.training
    H, W, Cimg = net.input_shape
    io = HeadIO(b, U)
    ar = b.arena

    b.segment = "fwd"
    xin, x8 = emit_input(b, H, W, Cimg, input_dtype)
    kh, kw = conv.kernel_size
    sh, sw = conv.strides
    Ho, Wo = (H - kh) // sh + 1, (W - kw) // sw + 1
    y = b.nhwc(B, Ho, Wo, conv.filters)
    b.conv(x8, conv, y, stride=(sh, sw), pads=(0, 0), bias=conv.bias, epi_act=RELU)
    ph, pw = Ho // 2, Wo // 2
    p = b.nhwc(B, ph, pw, conv.filters)
    am = b.alloc((B * ph * pw * conv.filters,), torch.uint8)
    b.pool(y, p, k=2, s=2, is_max=True, argmax=am)

    a = nat.Mlp2Args()
    a.x = p.ptr
    a.N, a.D0, a.D1, a.U = B, ph * pw * conv.filters, d1.units, U
    if a.D0 != d1.kernel.shape[0]:
        raise RuntimeError(f"flatten width {a.D0} != dense input {d1.kernel.shape[0]}")
    a.w1, a.b1 = d1.kernel.data_ptr(), nat.ptr(d1.bias if d1.use_bias else None)
    a.w2, a.b2 = d2.kernel.data_ptr(), nat.ptr(d2.bias if d2.use_bias else None)
    a.p0, a.p1 = float(p0), float(p1)
    a.seed = int(torch.initial_seed()) & ((1 << 64) - 1)
    step = b.alloc((4,), torch.int32)
    a.step = step.data_ptr()
    a.labels, a.logits = io.labels.data_ptr(), io.logits.data_ptr()
    a.h1 = b.alloc((B, d1.units), F32).data_ptr()
    a.loss = io.loss.data_ptr()
    a.dlogits = io.dlogits.data_ptr() if training else 0
    a.loss_scale = 1.0 / float(B)
    a.dl_scale = a.loss_scale * b.grad_weight
    a.training = 1 if training else 0
    b.memset(io.loss)
    b.emit(nat.OP_MLP_FWD, a)
    b.xin, b.io = xin, io
    if not training:
        return

    b.segment = "bwd"
    b.memset(ar.grad)
    dxp = b.nhwc(B, ph, pw, conv.filters, F32)
    a.dw1, a.db1 = ar.grad_of(d1.kernel).data_ptr(), nat.ptr(ar.grad_of(d1.bias) if d1.use_bias else None)
    a.dw2, a.db2 = ar.grad_of(d2.kernel).data_ptr(), nat.ptr(ar.grad_of(d2.bias) if d2.use_bias else None)
    a.dx = dxp.ptr
    b.emit(nat.OP_MLP_BWD, a)
    b.mark_grads_ready([d2.kernel, d1.kernel] + ([d2.bias] if d2.use_bias else []) +
                       ([d1.bias] if d1.use_bias else []))
    dy = b.nhwc(B, Ho, Wo, conv.filters)
    _pool_bwd_relu(b, dxp, dy, am, y, ar.grad_of(conv.bias) if conv.use_bias else None)
    b.wgrad(x8, conv, dy, ar.grad_of(conv.kernel), stride=(sh, sw), pads=(0, 0), cin_real=Cimg, lane=1)
    b.mark_grads_ready([conv.kernel] + ([conv.bias] if conv.use_bias else []))
    b.emit(nat.OP_MLP_STEP, ptrs=(step.data_ptr(),))  # fresh dropout masks next step
