"""Keras-semantics layers on top of PyTorch (reference / CPU path and numerics oracle).

The reference builds every network from ``tf.keras`` layers (``dist_model_tf_vgg.py:119-129``,
``dist_model_tf_mobile.py:119``, ``dist_model_tf_dense.py:131``, ``secure_fed_model.py:84-98``).
What matters for capability parity is reproduced here exactly:

* every layer has a Keras name and sits in a flat ``layers`` list, so ``layers[:fine_tune_at]``
  freezes the same layers as Keras (``dist_model_tf_vgg.py:150-151``);
* weights are stored in Keras layouts (conv HWIO, depthwise (kh,kw,C,1), dense (in,out),
  BN gamma/beta/moving_mean/moving_variance), so ``get_weights()`` order and the HDF5 layout
  match Keras;
* a frozen BatchNormalization runs in inference mode (TF>=2.0 semantics);
* Keras default initialisers (glorot_uniform kernels, zero bias, BN gamma=1 beta=0 mean=0 var=1).

Tensors flowing between layers are NHWC (Keras ``channels_last``).  The math here is plain
PyTorch and is the fp32 reference that the MI355X kernels in ``idc_models_amd.ops`` are tested
against; the fast GPU path does not run these modules (see ``idc_models_amd.runtime``).
"""
from __future__ import annotations

import math
import re
from typing import Iterable, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


def glorot_uniform_(t: torch.Tensor, fan_in: int, fan_out: int, generator=None) -> torch.Tensor:
    limit = math.sqrt(6.0 / float(fan_in + fan_out))
    with torch.no_grad():
        t.uniform_(-limit, limit, generator=generator)
    return t


class KLayer(nn.Module):
    """Base class: a named Keras layer with a ``trainable`` flag.

    ``weight_names`` lists the Keras variable names in Keras order (trainable first as declared
    by the layer: e.g. ``kernel, bias`` or ``gamma, beta, moving_mean, moving_variance``).
    """

    keras_class = "Layer"

    def __init__(self, name: str):
        super().__init__()
        self.name = name
        self._trainable = True

    # --- trainable flag -------------------------------------------------------------------
    @property
    def trainable(self) -> bool:
        return self._trainable

    @trainable.setter
    def trainable(self, value: bool) -> None:
        self._trainable = bool(value)
        for p in self.trainable_params():
            p.requires_grad_(self._trainable)

    # --- weights --------------------------------------------------------------------------
    def weight_names(self) -> List[str]:
        return []

    def weight_tensors(self) -> List[torch.Tensor]:
        return [getattr(self, n) for n in self.weight_names()]

    def trainable_params(self) -> List[nn.Parameter]:
        return [t for t in self.weight_tensors() if isinstance(t, nn.Parameter)]

    def non_trainable_tensors(self) -> List[torch.Tensor]:
        return [t for t in self.weight_tensors() if not isinstance(t, nn.Parameter)]

    @property
    def trainable_weights(self) -> List[torch.Tensor]:
        return list(self.trainable_params()) if self._trainable else []

    @property
    def non_trainable_weights(self) -> List[torch.Tensor]:
        if self._trainable:
            return self.non_trainable_tensors()
        return self.weight_tensors()

    @property
    def weights(self) -> List[torch.Tensor]:
        return self.trainable_weights + self.non_trainable_weights

    def keras_weight_names(self) -> List[str]:
        """Names as Keras writes them into HDF5 (``layer/var:0``), in ``weights`` order."""
        by_id = {id(t): n for n, t in zip(self.weight_names(), self.weight_tensors())}
        return [f"{self.name}/{by_id[id(t)]}:0" for t in self.weights]

    def count_params(self) -> int:
        return sum(t.numel() for t in self.weight_tensors())

    def reset_parameters(self, generator=None) -> None:
        pass

    def extra_repr(self) -> str:
        return f"name={self.name!r}"


class InputLayer(KLayer):
    keras_class = "InputLayer"

    def __init__(self, shape: Tuple[int, int, int], name: str = "input_1"):
        super().__init__(name)
        self.shape = tuple(shape)

    def forward(self, x):
        return x


def _pair(v) -> Tuple[int, int]:
    return (v, v) if isinstance(v, int) else tuple(v)


def _pads_same(size: int, k: int, s: int) -> Tuple[int, int]:
    """TF 'same' padding (extra padding goes bottom/right)."""
    out = -(-size // s)
    total = max((out - 1) * s + k - size, 0)
    return total // 2, total - total // 2


class Conv2D(KLayer):
    """``keras.layers.Conv2D`` (kernel HWIO, optional bias, activation None/'relu').

    ``padding`` is ``'same'`` or ``'valid'``.  Input/output NHWC.
    """

    keras_class = "Conv2D"

    def __init__(self, in_ch: int, filters: int, kernel_size, strides=1, padding: str = "valid",
                 use_bias: bool = True, activation: Optional[str] = None, name: str = "conv"):
        super().__init__(name)
        self.in_ch, self.filters = in_ch, filters
        self.kernel_size = _pair(kernel_size)
        self.strides = _pair(strides)
        self.padding = padding
        self.use_bias = use_bias
        self.activation = activation
        kh, kw = self.kernel_size
        self.kernel = nn.Parameter(torch.empty(kh, kw, in_ch, filters))
        if use_bias:
            self.bias = nn.Parameter(torch.zeros(filters))
        self.reset_parameters()

    def weight_names(self):
        return ["kernel", "bias"] if self.use_bias else ["kernel"]

    def reset_parameters(self, generator=None):
        kh, kw = self.kernel_size
        glorot_uniform_(self.kernel, kh * kw * self.in_ch, kh * kw * self.filters, generator)
        if self.use_bias:
            with torch.no_grad():
                self.bias.zero_()

    def pads(self, h: int, w: int) -> Tuple[int, int, int, int]:
        """(top, bottom, left, right) zero padding applied before a 'valid' conv."""
        if self.padding == "valid":
            return (0, 0, 0, 0)
        kh, kw = self.kernel_size
        sh, sw = self.strides
        t, b = _pads_same(h, kh, sh)
        l, r = _pads_same(w, kw, sw)
        return (t, b, l, r)

    def output_hw(self, h: int, w: int) -> Tuple[int, int]:
        t, b, l, r = self.pads(h, w)
        kh, kw = self.kernel_size
        sh, sw = self.strides
        return ((h + t + b - kh) // sh + 1, (w + l + r - kw) // sw + 1)

    def forward(self, x):  # x: NHWC
        n, h, w, c = x.shape
        t, b, l, r = self.pads(h, w)
        xc = x.permute(0, 3, 1, 2)
        if t or b or l or r:
            xc = F.pad(xc, (l, r, t, b))
        wt = self.kernel.permute(3, 2, 0, 1)  # OIHW
        y = F.conv2d(xc, wt, self.bias if self.use_bias else None, stride=self.strides)
        if self.activation == "relu":
            y = F.relu(y)
        return y.permute(0, 2, 3, 1)


class DepthwiseConv2D(KLayer):
    """``keras.layers.DepthwiseConv2D`` (depth_multiplier 1, kernel (kh,kw,C,1))."""

    keras_class = "DepthwiseConv2D"

    def __init__(self, channels: int, kernel_size=3, strides=1, padding: str = "same",
                 use_bias: bool = False, name: str = "depthwise"):
        super().__init__(name)
        self.channels = channels
        self.kernel_size = _pair(kernel_size)
        self.strides = _pair(strides)
        self.padding = padding
        self.use_bias = use_bias
        kh, kw = self.kernel_size
        self.depthwise_kernel = nn.Parameter(torch.empty(kh, kw, channels, 1))
        if use_bias:
            self.bias = nn.Parameter(torch.zeros(channels))
        self.reset_parameters()

    def weight_names(self):
        return ["depthwise_kernel", "bias"] if self.use_bias else ["depthwise_kernel"]

    def reset_parameters(self, generator=None):
        kh, kw = self.kernel_size
        glorot_uniform_(self.depthwise_kernel, kh * kw * self.channels, kh * kw * 1, generator)

    def pads(self, h, w):
        if self.padding == "valid":
            return (0, 0, 0, 0)
        kh, kw = self.kernel_size
        sh, sw = self.strides
        t, b = _pads_same(h, kh, sh)
        l, r = _pads_same(w, kw, sw)
        return (t, b, l, r)

    def output_hw(self, h, w):
        t, b, l, r = self.pads(h, w)
        kh, kw = self.kernel_size
        sh, sw = self.strides
        return ((h + t + b - kh) // sh + 1, (w + l + r - kw) // sw + 1)

    def forward(self, x):
        n, h, w, c = x.shape
        t, b, l, r = self.pads(h, w)
        xc = x.permute(0, 3, 1, 2)
        if t or b or l or r:
            xc = F.pad(xc, (l, r, t, b))
        wt = self.depthwise_kernel.permute(2, 3, 0, 1)  # (C,1,kh,kw)
        y = F.conv2d(xc, wt, self.bias if self.use_bias else None, stride=self.strides, groups=c)
        return y.permute(0, 2, 3, 1)


class BatchNormalization(KLayer):
    """``keras.layers.BatchNormalization`` over the channel (last) axis.

    Training mode (layer trainable and model called with training=True): batch statistics,
    moving stats updated as ``moving = m*moving + (1-m)*batch`` with the Bessel-corrected
    batch variance.  Frozen layer or inference: moving statistics.
    """

    keras_class = "BatchNormalization"

    def __init__(self, channels: int, epsilon: float = 1e-3, momentum: float = 0.99,
                 name: str = "bn"):
        super().__init__(name)
        self.channels = channels
        self.epsilon = epsilon
        self.momentum = momentum
        self.gamma = nn.Parameter(torch.ones(channels))
        self.beta = nn.Parameter(torch.zeros(channels))
        self.register_buffer("moving_mean", torch.zeros(channels))
        self.register_buffer("moving_variance", torch.ones(channels))

    def weight_names(self):
        return ["gamma", "beta", "moving_mean", "moving_variance"]

    def reset_parameters(self, generator=None):
        with torch.no_grad():
            self.gamma.fill_(1.0)
            self.beta.zero_()
            self.moving_mean.zero_()
            self.moving_variance.fill_(1.0)

    def forward(self, x):
        use_batch = self.training and self._trainable
        c = x.shape[-1]
        if use_batch:
            xf = x.reshape(-1, c)
            mean = xf.mean(0)
            var = xf.var(0, unbiased=False)
            n = xf.shape[0]
            with torch.no_grad():
                unbiased = var * (n / max(n - 1, 1))
                self.moving_mean.mul_(self.momentum).add_((1 - self.momentum) * mean.detach())
                self.moving_variance.mul_(self.momentum).add_((1 - self.momentum) * unbiased.detach())
        else:
            mean, var = self.moving_mean, self.moving_variance
        inv = torch.rsqrt(var + self.epsilon)
        return (x - mean) * (inv * self.gamma) + self.beta


class Activation(KLayer):
    keras_class = "Activation"

    def __init__(self, kind: str, name: str):
        super().__init__(name)
        self.kind = kind

    def forward(self, x):
        if self.kind == "relu":
            return F.relu(x)
        if self.kind == "relu6":
            return torch.clamp(x, 0.0, 6.0)
        if self.kind == "linear":
            return x
        raise ValueError(self.kind)


class ReLU(Activation):
    """``keras.layers.ReLU(max_value)`` — ReLU6 when ``max_value == 6``."""

    keras_class = "ReLU"

    def __init__(self, max_value: Optional[float], name: str):
        super().__init__("relu6" if max_value == 6.0 else "relu", name)


class ZeroPadding2D(KLayer):
    keras_class = "ZeroPadding2D"

    def __init__(self, padding: Tuple[Tuple[int, int], Tuple[int, int]], name: str):
        super().__init__(name)
        self.padding = padding  # ((top,bottom),(left,right))

    def forward(self, x):
        (t, b), (l, r) = self.padding
        return F.pad(x, (0, 0, l, r, t, b))


class MaxPooling2D(KLayer):
    keras_class = "MaxPooling2D"

    def __init__(self, pool_size=2, strides=None, name: str = "pool"):
        super().__init__(name)
        self.pool_size = _pair(pool_size)
        self.strides = _pair(strides if strides is not None else pool_size)

    def forward(self, x):
        y = F.max_pool2d(x.permute(0, 3, 1, 2), self.pool_size, self.strides)
        return y.permute(0, 2, 3, 1)


class AveragePooling2D(KLayer):
    keras_class = "AveragePooling2D"

    def __init__(self, pool_size=2, strides=None, name: str = "pool"):
        super().__init__(name)
        self.pool_size = _pair(pool_size)
        self.strides = _pair(strides if strides is not None else pool_size)

    def forward(self, x):
        y = F.avg_pool2d(x.permute(0, 3, 1, 2), self.pool_size, self.strides)
        return y.permute(0, 2, 3, 1)


class GlobalAveragePooling2D(KLayer):
    keras_class = "GlobalAveragePooling2D"

    def __init__(self, name: str = "global_average_pooling2d"):
        super().__init__(name)

    def forward(self, x):
        return x.mean(dim=(1, 2))


class Flatten(KLayer):
    keras_class = "Flatten"

    def __init__(self, name: str = "flatten"):
        super().__init__(name)

    def forward(self, x):
        return x.reshape(x.shape[0], -1)  # NHWC flatten order == Keras channels_last


class Dropout(KLayer):
    keras_class = "Dropout"

    def __init__(self, rate: float, name: str = "dropout"):
        super().__init__(name)
        self.rate = rate

    def forward(self, x):
        return F.dropout(x, self.rate, self.training)


class Dense(KLayer):
    keras_class = "Dense"

    def __init__(self, in_features: int, units: int, activation: Optional[str] = None,
                 use_bias: bool = True, name: str = "dense"):
        super().__init__(name)
        self.in_features, self.units = in_features, units
        self.activation = activation
        self.use_bias = use_bias
        self.kernel = nn.Parameter(torch.empty(in_features, units))
        if use_bias:
            self.bias = nn.Parameter(torch.zeros(units))
        self.reset_parameters()

    def weight_names(self):
        return ["kernel", "bias"] if self.use_bias else ["kernel"]

    def reset_parameters(self, generator=None):
        glorot_uniform_(self.kernel, self.in_features, self.units, generator)
        if self.use_bias:
            with torch.no_grad():
                self.bias.zero_()

    def forward(self, x):
        y = x @ self.kernel
        if self.use_bias:
            y = y + self.bias
        if self.activation == "relu":
            y = F.relu(y)
        return y


class Add(KLayer):
    keras_class = "Add"

    def forward(self, a, b):
        return a + b


class Concatenate(KLayer):
    keras_class = "Concatenate"

    def forward(self, a, b):
        return torch.cat([a, b], dim=-1)


def correct_pad(h: int, w: int, kernel_size: int = 3) -> Tuple[Tuple[int, int], Tuple[int, int]]:
    """Keras ``correct_pad``: asymmetric padding for stride-2 'valid' convs.

    Even input -> (top,left)=k//2-1, (bottom,right)=k//2; odd input -> symmetric k//2.
    """
    c = kernel_size // 2
    adj_h, adj_w = 1 - h % 2, 1 - w % 2
    return ((c - adj_h, c), (c - adj_w, c))


class KModel(KLayer):
    """A Keras functional model: a flat ``layers`` list plus an explicit forward graph."""

    keras_class = "Model"

    def __init__(self, name: str):
        super().__init__(name)
        self._layers: List[KLayer] = []

    def add(self, layer: KLayer) -> KLayer:
        self._layers.append(layer)
        # register as a submodule under a sanitised unique attribute name
        self.add_module(f"l{len(self._layers) - 1:04d}_" + re.sub(r"[^0-9A-Za-z_]", "_", layer.name), layer)
        return layer

    @property
    def layers(self) -> List[KLayer]:
        return self._layers

    def get_layer(self, name: str) -> KLayer:
        for l in self._layers:
            if l.name == name:
                return l
        raise KeyError(name)

    @property
    def trainable(self) -> bool:
        return self._trainable

    @trainable.setter
    def trainable(self, value: bool) -> None:
        # Keras: setting a model's trainable flag sets it recursively on every layer.
        self._trainable = bool(value)
        for l in self._layers:
            l.trainable = value

    def weight_layers(self) -> List[KLayer]:
        return [l for l in self._layers if l.weight_names()]

    def weight_tensors(self):
        out = []
        for l in self._layers:
            out.extend(l.weight_tensors())
        return out

    @property
    def trainable_weights(self):
        if not self._trainable:
            return []
        out = []
        for l in self._layers:
            out.extend(l.trainable_weights)
        return out

    @property
    def non_trainable_weights(self):
        out = []
        for l in self._layers:
            out.extend(l.weight_tensors() if not self._trainable else l.non_trainable_weights)
        return out

    def keras_weight_names(self):
        # Keras nested-model HDF5 layout: every sublayer weight under the model's group, in
        # the model's ``weights`` order (trainable weights of all layers, then non-trainable).
        names = []
        by_id = {}
        for l in self._layers:
            for n, t in zip(l.weight_names(), l.weight_tensors()):
                by_id[id(t)] = f"{l.name}/{n}:0"
        for t in self.weights:
            names.append(by_id[id(t)])
        return names

    def reset_parameters(self, generator=None):
        for l in self._layers:
            l.reset_parameters(generator)

    def count_params(self):
        return sum(l.count_params() for l in self._layers)
