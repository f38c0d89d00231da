"""Flat parameter / gradient arenas.

All trainable parameters of a compiled model live in ONE contiguous fp32 buffer and their
gradients in a second one.  This is the MI355X-first layout choice from SURVEY §7.1:

* the optimizer is a single fused multi-tensor kernel over the flat buffer;
* data-parallel gradient buckets are contiguous slices of the gradient arena, so the RCCL
  all-reduce is zero-copy;
* a whole training step (which writes grads in place) is capturable in one HIP graph.

The module's ``nn.Parameter`` objects keep working: their ``.data`` and ``.grad`` are re-pointed
at views of the arenas, so ``get_weights`` / checkpoints / the eager reference path all see the
same storage.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence

import torch


@dataclass
class Slot:
    offset: int
    numel: int
    shape: torch.Size


class ParamArena:
    ALIGN = 64  # elements (256 B): keeps every tensor 16-B aligned for vector kernels

    def __init__(self, params: Sequence[torch.nn.Parameter], device=None, dtype=torch.float32):
        self.params: List[torch.nn.Parameter] = list(params)
        device = device or (self.params[0].device if self.params else torch.device("cpu"))
        self.slots: List[Slot] = []
        off = 0
        for p in self.params:
            self.slots.append(Slot(off, p.numel(), p.shape))
            off += (p.numel() + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        self.numel = max(off, self.ALIGN)
        self.data = torch.zeros(self.numel, device=device, dtype=dtype)
        self.grad = torch.zeros(self.numel, device=device, dtype=dtype)
        with torch.no_grad():
            for p, s in zip(self.params, self.slots):
                self.data[s.offset:s.offset + s.numel].copy_(p.detach().reshape(-1))
                p.data = self.data[s.offset:s.offset + s.numel].view(s.shape)
                p.grad = self.grad[s.offset:s.offset + s.numel].view(s.shape)

    def view(self, buf: torch.Tensor, i: int) -> torch.Tensor:
        s = self.slots[i]
        return buf[s.offset:s.offset + s.numel].view(s.shape)

    def grad_of(self, p) -> torch.Tensor:
        for q, s in zip(self.params, self.slots):
            if q is p:
                return self.grad[s.offset:s.offset + s.numel].view(s.shape)
        raise KeyError("parameter not in arena")

    def offset_of(self, p) -> int:
        for q, s in zip(self.params, self.slots):
            if q is p:
                return s.offset
        raise KeyError("parameter not in arena")

    def zero_grad(self):
        self.grad.zero_()

    def release(self):
        """Give every parameter its own storage again (arena is about to be dropped)."""
        with torch.no_grad():
            for p in self.params:
                p.data = p.data.clone()
                p.grad = None
