"""VGG16 lowering (``dist_model_tf_vgg.py:119-129``, ``fed_model.py:113-123``).

Forward: 13 x [3x3 conv + bias + ReLU in the epilogue] and 5 max-pools (argmax kept for a
gather-form backward).  Backward folds every elementwise step into a GEMM epilogue:
the dgrad epilogue of conv l applies ReLU'(x_l) to dX and reduces sum(dZ) = dbias of conv l-1;
across a pool the mask is applied at pooled resolution (max-pool output > 0 iff the selected
input > 0) and the pool backward is then a plain gather.  No standalone ReLU/bias kernels.
"""
from __future__ import annotations

import torch

from ..models.layers import Conv2D, MaxPooling2D
from ..ops import _native as nat
from .builder import F32, Builder
from .lower_common import RELU, FreezeInfo, HeadIO, emit_head, emit_head_bwd, emit_input


def lower_vgg(b: Builder, net, U: int, input_dtype):
    base, dense = net.base, net.head
    B = b.B
    training = b.training
    fz = FreezeInfo(base, training)
    H, W, Cimg = base.input_shape
    io = HeadIO(b, U)
    b.segment = "fwd"
    xin, x8 = emit_input(b, H, W, Cimg, input_dtype)

    nodes = []  # forward record: (kind, layer, x, y, extra)
    cur = x8
    for l in base.layers[1:]:
        if isinstance(l, Conv2D):
            y = b.nhwc(B, cur.H, cur.W, l.filters)
            b.conv(cur, l, y, pads=(1, 1), bias=l.bias, epi_act=RELU)
            nodes.append(("conv", l, cur, y, None))
            cur = y
        elif isinstance(l, MaxPooling2D):
            Ho, Wo = cur.H // 2, cur.W // 2
            y = b.nhwc(B, Ho, Wo, cur.C)
            am = b.alloc((B * Ho * Wo * cur.C,), torch.uint8)
            b.pool(cur, y, k=2, s=2, is_max=True, argmax=am)
            nodes.append(("pool", l, cur, y, am))
            cur = y
    emit_head(b, cur, None, dense, U, io, training)
    b.xin, b.io = xin, io
    if not training:
        return

    b.segment = "bwd"
    b.memset(b.arena.grad)
    if b.det:  # the deterministic mode's private bias-gradient slots live in the stats arena
        b.memset(b.stats_arena)
    need = fz.any()
    dA = emit_head_bwd(b, cur, dense, U, io, need_dA=need)
    if not need:
        return
    ar = b.arena
    # g: gradient w.r.t. the current node's OUTPUT; `masked` says it is already dZ (pre-ReLU)
    g, masked = dA, False
    i = len(nodes) - 1
    while i >= 0:
        kind, l, x, y, am = nodes[i]
        if kind == "pool":
            if not fz.before(l):
                return
            dx = b.nhwc(x.N, x.H, x.W, x.C)
            prev_conv = nodes[i - 1][1]
            if masked:
                b.pool_bwd(g, dx, k=2, s=2, is_max=True, argmax=am)
            else:
                # mask ReLU of the producing conv + its bias gradient, in the pool-backward epilogue
                a_bias = ar.grad_of(prev_conv.bias) if fz.trainable(prev_conv) else None
                _pool_bwd_relu(b, g, dx, am, x, a_bias)
            g, masked = dx, True
        else:
            if fz.trainable(l):
                # inputs never reused; the first conv's wgrad consumes the LAST dgrad's output and
                # runs on the main lane, next to the side lane's backlog (lower_densenet stem)
                b.wgrad(x, l, g, ar.grad_of(l.kernel), pads=(1, 1), lane=0 if i == 0 else 1)
                b.mark_grads_ready([l.kernel, l.bias])
            if not fz.before(l):
                return
            dx = b.nhwc(x.N, x.H, x.W, x.C)
            # the input x of this conv is ReLU(conv_prev) (possibly pooled)
            j = i - 1
            while nodes[j][0] != "conv":
                j -= 1
            prev_conv = nodes[j][1]
            gb = ar.grad_of(prev_conv.bias) if fz.trainable(prev_conv) else None
            b.dgrad(g, l, dx, pads=(1, 1), mx=x, mbn=nat.bn_args(mode=0, act=RELU), gsum=gb)
            g, masked = dx, True
        i -= 1


def _pool_bwd_relu(b: Builder, dy, dx, argmax, x, gbias):
    a = nat.PoolBwdArgs()
    a.dy, a.lddy, a.dy_f32 = dy.ptr, dy.ld, 1 if dy.is_f32 else 0
    a.argmax = argmax.data_ptr()
    a.N, a.H, a.W, a.C = dx.N, dx.H, dx.W, dx.C
    a.k, a.s, a.pt, a.pl = 2, 2, 0, 0
    a.Ho, a.Wo = dy.H, dy.W
    a.x, a.ldx = x.ptr, x.ld
    a.bn = nat.bn_args(mode=0, act=RELU)
    a.gsum = nat.ptr(gbias)
    a.gsumx = 0
    if b.det and gbias is not None:  # one private slot per workgroup + fixed-order collapse
        a.gsum, _, a.gsum_slots, a.gsum_ld = b._det_gsum_slots(dx.C, b._rows_grid(dx.M, dx.C, 4), gbias.data_ptr())
    elif gbias is not None and b._rows_slotted(b._rows_grid(dx.M, dx.C, 4)):
        a.gsum, _, a.gsum_slots, a.gsum_ld = b.slotted_sums(dx.C, b._rows_grid(dx.M, dx.C, 4), gbias.data_ptr())
    a.dx, a.lddx = dx.ptr, dx.ld
    a.is_avg = 0
    b.emit(nat.OP_POOL_BWD, a)
