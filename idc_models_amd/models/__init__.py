"""Model zoo: Keras-faithful backbones + the reference's ``Sequential([base, GAP, Dense])`` head.

Reference head composition: ``dist_model_tf_vgg.py:123-129``, ``fed_model.py:117-123``,
``dist_model_tf_dense.py:135-141``.
"""
from __future__ import annotations

from typing import Optional, Tuple

from .densenet import DenseNet, DenseNet121, DenseNet169, DenseNet201
from .layers import (Dense, GlobalAveragePooling2D, KLayer, KModel, BatchNormalization, Conv2D,
                     DepthwiseConv2D)
from .mobilenet_v2 import MobileNetV2
from .tiny_cnn import TinyCNN
from .vgg import VGG16


class Sequential(KModel):
    """``tf.keras.Sequential([base_model, GlobalAveragePooling2D(), Dense(k)])``."""

    def __init__(self, base: KModel, num_outputs: int, name: str = "sequential"):
        super().__init__(name)
        self.add(base)
        self.add(GlobalAveragePooling2D("global_average_pooling2d"))
        self.add(Dense(base.output_channels, num_outputs, None, True, "dense"))
        self.num_outputs = num_outputs
        self.input_shape = base.input_shape

    @property
    def base(self) -> KModel:
        return self.layers[0]

    @property
    def gap(self):
        return self.layers[1]

    @property
    def head(self) -> Dense:
        return self.layers[2]

    def weight_layers(self):
        return [l for l in self.layers if l.weight_tensors()]

    def forward(self, x):
        return self.head(self.gap(self.base(x)))


BACKBONES = {
    "vgg16": lambda shape: VGG16(shape),
    "mobilenetv2": lambda shape: MobileNetV2(shape),
    "densenet121": lambda shape: DenseNet(121, shape),
    "densenet169": lambda shape: DenseNet(169, shape),
    "densenet201": lambda shape: DenseNet(201, shape),
}

DEFAULT_SHAPES = {"vgg16": (50, 50, 3), "mobilenetv2": (50, 50, 3), "densenet121": (50, 50, 3),
                  "densenet169": (50, 50, 3), "densenet201": (32, 32, 3), "tinycnn": (10, 10, 3)}


def build_backbone(arch: str, input_shape: Optional[Tuple[int, int, int]] = None) -> KModel:
    arch = arch.lower()
    return BACKBONES[arch](tuple(input_shape or DEFAULT_SHAPES[arch]))


def build_model(arch: str, input_shape: Optional[Tuple[int, int, int]] = None,
                num_outputs: int = 1, seed: Optional[int] = None) -> KModel:
    """Backbone + GAP + Dense(num_outputs) logits (or the tiny CNN, which has its own head)."""
    import torch

    if seed is not None:
        torch.manual_seed(seed)
    arch = arch.lower()
    if arch == "tinycnn":
        return TinyCNN(tuple(input_shape or DEFAULT_SHAPES[arch]))
    return Sequential(build_backbone(arch, input_shape), num_outputs)


def clone_model(model: KModel) -> KModel:
    """``tf.keras.models.clone_model``: same architecture + trainable flags, FRESH weights."""
    import copy

    m = copy.deepcopy(model)
    m.reset_parameters()
    return m


__all__ = ["VGG16", "MobileNetV2", "DenseNet", "DenseNet121", "DenseNet169", "DenseNet201",
           "TinyCNN", "Sequential", "build_model", "build_backbone", "clone_model", "KLayer",
           "KModel", "BatchNormalization", "Conv2D", "DepthwiseConv2D", "Dense"]
