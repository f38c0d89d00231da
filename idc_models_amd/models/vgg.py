"""VGG16 backbone (``include_top=False``) with Keras layer names.

Reference use: ``keras.applications.vgg16.VGG16(input_shape=(50,50,3), include_top=False)``
(``dist_model_tf_vgg.py:119-121``, ``fed_model.py:113-115``).  19 layers; ``layers[15]`` is
``block5_conv1`` so ``fine_tune_at=15`` trains block5 + head.
"""
from __future__ import annotations

from typing import Tuple

from .layers import Conv2D, InputLayer, KModel, MaxPooling2D

VGG16_CFG = [(64, 2), (128, 2), (256, 3), (512, 3), (512, 3)]


class VGG16(KModel):
    family = "vgg16"

    def __init__(self, input_shape: Tuple[int, int, int] = (50, 50, 3), name: str = "vgg16"):
        super().__init__(name)
        self.input_shape = tuple(input_shape)
        h, w, c = input_shape
        self.add(InputLayer(input_shape, "input_1"))
        cin = c
        for bi, (cout, n) in enumerate(VGG16_CFG, start=1):
            for ci in range(1, n + 1):
                self.add(Conv2D(cin, cout, 3, 1, "same", True, "relu", f"block{bi}_conv{ci}"))
                cin = cout
            self.add(MaxPooling2D(2, 2, f"block{bi}_pool"))
            h, w = h // 2, w // 2
        self.output_channels = cin
        self.output_hw = (h, w)

    def forward(self, x):
        for l in self.layers:
            x = l(x)
        return x
