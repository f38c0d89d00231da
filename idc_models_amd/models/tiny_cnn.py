"""The secure-FL tiny CNN (``secure_fed_model.py:84-98``).

Conv2D(32, 3x3, stride 2, relu) on 10x10x3 -> 4x4x32 -> MaxPool 2x2 -> 2x2x32 -> Dropout(.25)
-> Flatten(128) -> Dense(8, relu) -> Dropout(.5) -> Dense(1) logits.  1,937 parameters; weight
shapes match ``weights_shape`` (``secure_fed_model.py:73-78``).
"""
from __future__ import annotations

from typing import Tuple

from .layers import Conv2D, Dense, Dropout, Flatten, KModel, MaxPooling2D


class TinyCNN(KModel):
    family = "tinycnn"

    def __init__(self, input_shape: Tuple[int, int, int] = (10, 10, 3), name: str = "sequential"):
        super().__init__(name)
        self.input_shape = tuple(input_shape)
        h, w, c = input_shape
        conv = self.add(Conv2D(c, 32, 3, 2, "valid", True, "relu", "conv2d"))
        h, w = conv.output_hw(h, w)
        self.add(MaxPooling2D(2, 2, "max_pooling2d"))
        h, w = h // 2, w // 2
        self.add(Dropout(0.25, "dropout"))
        self.add(Flatten("flatten"))
        self.add(Dense(h * w * 32, 8, "relu", True, "dense"))
        self.add(Dropout(0.5, "dropout_1"))
        self.add(Dense(8, 1, None, True, "dense_1"))
        self.num_outputs = 1

    def forward(self, x):
        for l in self.layers:
            x = l(x)
        return x
