"""Optimizers with Keras (TF 2.1) semantics over a flat parameter arena.

* ``RMSprop`` — reference optimizer everywhere (``dist_model_tf_vgg.py:130,153``,
  ``fed_model.py:126,208``, ``secure_fed_model.py:96``): ``ms <- rho*ms + (1-rho)*g^2;
  w <- w - lr*g/(sqrt(ms)+eps)``, rho=0.9, eps=1e-7, ms0=0.  With momentum>0
  the TF ``ApplyRMSProp`` form ``mom <- m*mom + lr*g/sqrt(ms+eps); w -= mom`` is used.
* ``SGD`` — TFF's server optimizer (lr=1.0) for FedAvg.

On a GPU arena the update is ONE fused HIP kernel (``ops.optim``); on CPU the same math runs as
vectorised torch ops.  A fresh optimizer (``compile``) means fresh slot state, as in Keras.
"""
from __future__ import annotations

from typing import Optional

import torch


class Optimizer:
    name = "optimizer"

    def __init__(self, learning_rate: float):
        self.learning_rate = float(learning_rate)
        self.iterations = 0
        self._arena = None

    def bind(self, arena) -> None:
        self._arena = arena
        self._build_slots(arena)

    def _build_slots(self, arena):
        pass

    def step(self, arena=None, lr: Optional[float] = None, grad_scale: float = 1.0) -> None:
        raise NotImplementedError

    def get_config(self):
        return {"name": self.name, "learning_rate": self.learning_rate}

    # non-finite guard (SURVEY §5 failure detection): skip the whole update when any (reduced)
    # gradient is inf/nan; the fused backend does the same check on the device
    skip_nonfinite = False
    skipped = 0

    def _should_skip(self, arena) -> bool:
        if self.skip_nonfinite and not bool(torch.isfinite(arena.grad).all()):
            self.skipped += 1
            return True
        return False

    def state_tensors(self):
        return {}

    def reset_state(self) -> None:
        """Zero every slot IN PLACE (pointers captured by HIP graphs stay valid)."""
        with torch.no_grad():
            for t in self.state_tensors().values():
                if t is not None:
                    t.zero_()
        self.iterations = 0


class RMSprop(Optimizer):
    name = "RMSprop"

    def __init__(self, learning_rate: float = 0.001, rho: float = 0.9, momentum: float = 0.0,
                 epsilon: float = 1e-7, centered: bool = False, lr: Optional[float] = None):
        super().__init__(lr if lr is not None else learning_rate)  # TF2.1 accepted lr=
        self.rho = float(rho)
        self.momentum = float(momentum)
        self.epsilon = float(epsilon)
        self.centered = bool(centered)
        self.ms = self.mom = self.mg = None

    def _build_slots(self, arena):
        self.ms = torch.zeros_like(arena.data)
        self.mom = torch.zeros_like(arena.data) if self.momentum > 0 else None
        self.mg = torch.zeros_like(arena.data) if self.centered else None

    def step(self, arena=None, lr=None, grad_scale: float = 1.0):
        arena = arena or self._arena
        if self._should_skip(arena):
            return
        lr = self.learning_rate if lr is None else lr
        w, g = arena.data, arena.grad
        if w.is_cuda and self.momentum == 0 and not self.centered:
            from ..ops import optim as optim_ops
            optim_ops.rmsprop_(w, g, self.ms, lr, self.rho, self.epsilon, grad_scale)
        else:
            gs = g * grad_scale if grad_scale != 1.0 else g
            self.ms.mul_(self.rho).addcmul_(gs, gs, value=1.0 - self.rho)
            denom = self.ms
            if self.centered:
                self.mg.mul_(self.rho).add_(gs, alpha=1.0 - self.rho)
                denom = self.ms - self.mg * self.mg
            if self.momentum > 0:
                self.mom.mul_(self.momentum).add_(lr * gs / torch.sqrt(denom + self.epsilon))
                w.sub_(self.mom)
            else:
                w.sub_(lr * gs / (torch.sqrt(denom) + self.epsilon))
        self.iterations += 1

    def get_config(self):
        return {"name": self.name, "learning_rate": self.learning_rate, "rho": self.rho,
                "momentum": self.momentum, "epsilon": self.epsilon, "centered": self.centered}

    def state_tensors(self):
        out = {"ms": self.ms}
        if self.mom is not None:
            out["mom"] = self.mom
        if self.mg is not None:
            out["mg"] = self.mg
        return out


class SGD(Optimizer):
    name = "SGD"

    def __init__(self, learning_rate: float = 0.01, momentum: float = 0.0, lr=None):
        super().__init__(lr if lr is not None else learning_rate)
        self.momentum = float(momentum)
        self.buf = None

    def _build_slots(self, arena):
        self.buf = torch.zeros_like(arena.data) if self.momentum > 0 else None

    def step(self, arena=None, lr=None, grad_scale: float = 1.0):
        arena = arena or self._arena
        if self._should_skip(arena):
            return
        lr = self.learning_rate if lr is None else lr
        g = arena.grad * grad_scale if grad_scale != 1.0 else arena.grad
        if self.buf is not None:
            self.buf.mul_(self.momentum).add_(g)
            g = self.buf
        arena.data.sub_(lr * g)
        self.iterations += 1

    def state_tensors(self):
        return {"buf": self.buf} if self.buf is not None else {}


def get(identifier) -> Optimizer:
    if isinstance(identifier, Optimizer):
        return identifier
    name = str(identifier).lower()
    if name == "rmsprop":
        return RMSprop()
    if name == "sgd":
        return SGD()
    raise ValueError(f"unknown optimizer {identifier!r}")
