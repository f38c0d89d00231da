"""DenseNet-121/169/201 (``include_top=False``) with Keras layer names.

Reference use: ``keras.applications.densenet.DenseNet201(input_shape=(32,32,3),
include_top=False)`` (``dist_model_tf_dense.py:131-133``); the north-star benchmark uses
DenseNet-121 at 50x50x3 (BASELINE.json).  Pre-activation conv blocks (BN -> ReLU -> conv),
BN eps 1.001e-5 / momentum 0.99, growth 32, bottleneck 4*32, transitions halve channels
(SURVEY §2.4.3).  DenseNet-121 has 427 layers; ``layers[150] == 'conv4_block2_1_conv'``
(``dist_model_tf_dense.py:158``).
"""
from __future__ import annotations

from typing import List, Tuple

from .layers import (Activation, AveragePooling2D, BatchNormalization, Concatenate, Conv2D,
                     InputLayer, KModel, MaxPooling2D, ZeroPadding2D)

DENSENET_BLOCKS = {121: (6, 12, 24, 16), 169: (6, 12, 32, 32), 201: (6, 12, 48, 32)}
BN_EPS = 1.001e-5
BN_MOM = 0.99
GROWTH = 32


class DenseNet(KModel):
    family = "densenet"

    def __init__(self, depth: int = 121, input_shape: Tuple[int, int, int] = (50, 50, 3),
                 name: str = None):
        super().__init__(name or f"densenet{depth}")
        self.depth = depth
        self.blocks = DENSENET_BLOCKS[depth]
        self.input_shape = tuple(input_shape)
        h, w, c = input_shape
        self.graph: List[tuple] = []
        self.add(InputLayer(input_shape, "input_1"))
        self._seq(ZeroPadding2D(((3, 3), (3, 3)), "zero_padding2d"))
        conv = self._seq(Conv2D(c, 64, 7, 2, "valid", False, None, "conv1/conv"))
        h, w = conv.output_hw(h + 6, w + 6)
        self._seq(BatchNormalization(64, BN_EPS, BN_MOM, "conv1/bn"))
        self._seq(Activation("relu", "conv1/relu"))
        self._seq(ZeroPadding2D(((1, 1), (1, 1)), "zero_padding2d_1"))
        self._seq(MaxPooling2D(3, 2, "pool1"))
        h, w = (h + 2 - 3) // 2 + 1, (w + 2 - 3) // 2 + 1
        ch = 64
        self.stage_shapes = []
        for si, nb in enumerate(self.blocks):
            stage = si + 2
            c0 = ch
            for bi in range(1, nb + 1):
                ch = self._conv_block(ch, f"conv{stage}_block{bi}")
            self.stage_shapes.append((h, w, c0, ch))
            if si < len(self.blocks) - 1:
                name = f"pool{stage}"
                self._seq(BatchNormalization(ch, BN_EPS, BN_MOM, name + "_bn"))
                self._seq(Activation("relu", name + "_relu"))
                self._seq(Conv2D(ch, ch // 2, 1, 1, "valid", False, None, name + "_conv"))
                self._seq(AveragePooling2D(2, 2, name + "_pool"))
                ch = ch // 2
                h, w = h // 2, w // 2
        self._seq(BatchNormalization(ch, BN_EPS, BN_MOM, "bn"))
        self._seq(Activation("relu", "relu"))
        self.output_channels = ch
        self.output_hw = (h, w)

    def _seq(self, layer):
        self.add(layer)
        self.graph.append(("seq", layer))
        return layer

    def _conv_block(self, cin, name):
        self.graph.append(("save", None))
        self._seq(BatchNormalization(cin, BN_EPS, BN_MOM, name + "_0_bn"))
        self._seq(Activation("relu", name + "_0_relu"))
        self._seq(Conv2D(cin, 4 * GROWTH, 1, 1, "valid", False, None, name + "_1_conv"))
        self._seq(BatchNormalization(4 * GROWTH, BN_EPS, BN_MOM, name + "_1_bn"))
        self._seq(Activation("relu", name + "_1_relu"))
        self._seq(Conv2D(4 * GROWTH, GROWTH, 3, 1, "same", False, None, name + "_2_conv"))
        cat = Concatenate(name + "_concat")
        self.add(cat)
        self.graph.append(("concat", cat))
        return cin + GROWTH

    def forward(self, x):
        saved = []
        for kind, layer in self.graph:
            if kind == "seq":
                x = layer(x)
            elif kind == "save":
                saved.append(x)
            elif kind == "concat":
                x = layer(saved.pop(), x)
        return x


def DenseNet121(input_shape=(50, 50, 3)):
    return DenseNet(121, input_shape)


def DenseNet169(input_shape=(50, 50, 3)):
    return DenseNet(169, input_shape)


def DenseNet201(input_shape=(32, 32, 3)):
    return DenseNet(201, input_shape)
