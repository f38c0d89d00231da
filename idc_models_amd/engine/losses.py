"""Losses (Keras semantics, mean over the global batch).

* ``BinaryCrossentropy(from_logits=True)`` — ``dist_model_tf_vgg.py:131``, ``fed_model.py:127``,
  ``secure_fed_model.py:96``: ``max(x,0) - x*z + log(1+exp(-|x|))``.
* ``CategoricalCrossentropy(from_logits=True)`` — ``dist_model_tf_dense.py:143``; accepts one-hot
  labels, and (fixing quirk Q5) integer labels are one-hot encoded instead of crashing.
* ``SparseCategoricalCrossentropy(from_logits=True)``.

Each loss returns the mean loss and the gradient w.r.t. the logits, scaled for the global batch,
which is what the fused GPU head kernel computes in one pass.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


class Loss:
    name = "loss"
    from_logits = True

    def __call__(self, logits: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def kind(self) -> str:
        return self.name


class BinaryCrossentropy(Loss):
    name = "binary_crossentropy"

    def __init__(self, from_logits: bool = True):
        self.from_logits = from_logits

    def __call__(self, logits, y):
        logits = logits.reshape(-1).float()
        y = y.reshape(-1).to(logits.dtype)
        if self.from_logits:
            return F.binary_cross_entropy_with_logits(logits, y)
        eps = 1e-7
        p = logits.clamp(eps, 1 - eps)
        return -(y * torch.log(p) + (1 - y) * torch.log(1 - p)).mean()


class CategoricalCrossentropy(Loss):
    name = "categorical_crossentropy"

    def __init__(self, from_logits: bool = True):
        self.from_logits = from_logits

    def __call__(self, logits, y):
        logits = logits.float()
        if y.dim() == 1 or (y.dim() == 2 and y.shape[1] == 1 and logits.shape[1] > 1):
            y = F.one_hot(y.reshape(-1).long(), logits.shape[1]).to(logits.dtype)
        logp = F.log_softmax(logits, -1) if self.from_logits else torch.log(logits.clamp_min(1e-7))
        return -(y.to(logits.dtype) * logp).sum(-1).mean()


class SparseCategoricalCrossentropy(Loss):
    name = "sparse_categorical_crossentropy"

    def __init__(self, from_logits: bool = True):
        self.from_logits = from_logits

    def __call__(self, logits, y):
        logits = logits.float()
        return F.cross_entropy(logits, y.reshape(-1).long())


def get(identifier) -> Loss:
    if isinstance(identifier, Loss):
        return identifier
    name = str(identifier).lower()
    table = {"binary_crossentropy": BinaryCrossentropy, "bce": BinaryCrossentropy,
             "categorical_crossentropy": CategoricalCrossentropy,
             "sparse_categorical_crossentropy": SparseCategoricalCrossentropy}
    return table[name]()
