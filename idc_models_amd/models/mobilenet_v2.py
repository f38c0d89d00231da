"""MobileNetV2 (alpha=1.0, ``include_top=False``) with Keras layer names (TF<=2.2 build).

Reference use: ``keras.applications.MobileNetV2(input_shape=(50,50,3), include_top=False)``
(``dist_model_tf_mobile.py:119-121``); BN eps 1e-3 / momentum 0.999; ReLU6; stride-2 layers use
Keras ``correct_pad`` asymmetric zero padding; 155 layers incl. ``Conv1_pad``; ``fine_tune_at=100``
(``dist_model_tf_mobile.py:146``) -> ``layers[100] == 'block_11_expand_BN'``.
"""
from __future__ import annotations

from typing import List, Tuple

from .layers import (Add, BatchNormalization, Conv2D, DepthwiseConv2D, InputLayer, KModel, ReLU,
                     ZeroPadding2D, correct_pad)

# (filters, stride, expansion) for block_id 0..16
MBV2_BLOCKS = [(16, 1, 1), (24, 2, 6), (24, 1, 6), (32, 2, 6), (32, 1, 6), (32, 1, 6),
               (64, 2, 6), (64, 1, 6), (64, 1, 6), (64, 1, 6), (96, 1, 6), (96, 1, 6),
               (96, 1, 6), (160, 2, 6), (160, 1, 6), (160, 1, 6), (320, 1, 6)]

BN_EPS = 1e-3
BN_MOM = 0.999


def _make_divisible(v, divisor=8, min_value=None):
    if min_value is None:
        min_value = divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


class MobileNetV2(KModel):
    family = "mobilenetv2"

    def __init__(self, input_shape: Tuple[int, int, int] = (50, 50, 3), alpha: float = 1.0,
                 name: str = None):
        h, w, c = input_shape
        super().__init__(name or "mobilenetv2_%0.2f_%s" % (alpha, h))
        self.input_shape = tuple(input_shape)
        self.alpha = alpha
        # graph: list of (kind, payload); executed by forward()
        self.graph: List[tuple] = []
        self.add(InputLayer(input_shape, "input_1"))
        first = _make_divisible(32 * alpha, 8)
        pad = correct_pad(h, w, 3)
        self._seq(ZeroPadding2D(pad, "Conv1_pad"))
        h, w = h + sum(pad[0]), w + sum(pad[1])
        conv = Conv2D(c, first, 3, 2, "valid", False, None, "Conv1")
        self._seq(conv)
        h, w = conv.output_hw(h, w)
        self._seq(BatchNormalization(first, BN_EPS, BN_MOM, "bn_Conv1"))
        self._seq(ReLU(6.0, "Conv1_relu"))
        cin = first
        for bid, (filters, stride, t) in enumerate(MBV2_BLOCKS):
            cin, h, w = self._inverted_res_block(cin, h, w, filters, alpha, stride, t, bid)
        last = _make_divisible(1280 * alpha, 8) if alpha > 1.0 else 1280
        self._seq(Conv2D(cin, last, 1, 1, "valid", False, None, "Conv_1"))
        self._seq(BatchNormalization(last, BN_EPS, BN_MOM, "Conv_1_bn"))
        self._seq(ReLU(6.0, "out_relu"))
        self.output_channels = last
        self.output_hw = (h, w)

    def _seq(self, layer):
        self.add(layer)
        self.graph.append(("seq", layer))
        return layer

    def _inverted_res_block(self, cin, h, w, filters, alpha, stride, expansion, block_id):
        pw = _make_divisible(int(filters * alpha), 8)
        self.graph.append(("save", None))  # remember block input for the residual
        if block_id:
            prefix = f"block_{block_id}_"
            self._seq(Conv2D(cin, expansion * cin, 1, 1, "same", False, None, prefix + "expand"))
            self._seq(BatchNormalization(expansion * cin, BN_EPS, BN_MOM, prefix + "expand_BN"))
            self._seq(ReLU(6.0, prefix + "expand_relu"))
        else:
            prefix = "expanded_conv_"
        ch = expansion * cin
        if stride == 2:
            pad = correct_pad(h, w, 3)
            self._seq(ZeroPadding2D(pad, prefix + "pad"))
            h, w = h + sum(pad[0]), w + sum(pad[1])
        dw = DepthwiseConv2D(ch, 3, stride, "same" if stride == 1 else "valid", False,
                             prefix + "depthwise")
        self._seq(dw)
        h, w = dw.output_hw(h, w)
        self._seq(BatchNormalization(ch, BN_EPS, BN_MOM, prefix + "depthwise_BN"))
        self._seq(ReLU(6.0, prefix + "depthwise_relu"))
        self._seq(Conv2D(ch, pw, 1, 1, "same", False, None, prefix + "project"))
        self._seq(BatchNormalization(pw, BN_EPS, BN_MOM, prefix + "project_BN"))
        if cin == pw and stride == 1:
            add = Add(prefix + "add")
            self.add(add)
            self.graph.append(("add", add))
        else:
            self.graph.append(("drop", None))
        return pw, h, w

    def forward(self, x):
        saved = []
        for kind, layer in self.graph:
            if kind == "seq":
                x = layer(x)
            elif kind == "save":
                saved.append(x)
            elif kind == "add":
                x = layer(saved.pop(), x)
            elif kind == "drop":
                saved.pop()
        return x
