"""Timing utilities.

``Timer`` reproduces the reference's only instrumentation (five identical copies, e.g.
``dist_model_tf_vgg.py:19-32``): a context manager printing ``"{name} took {sec} seconds"``.
``StepTimer`` adds what the reference lacks: device-event timing of individual steps that
excludes warm-up and reports images/sec (synchronises only at ``stop``).
"""
from __future__ import annotations

import time
from typing import List, Optional

import torch


class Timer:
    def __init__(self, name: str, printer=print):
        self.name = name
        self.printer = printer
        self.seconds: Optional[float] = None

    def __enter__(self):
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
        self.t = time.time()
        return self

    def __exit__(self, *args, **kwargs):
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
        self.seconds = time.time() - self.t
        if self.printer is not None:
            self.printer("{} took {} seconds".format(self.name, self.seconds))


class StepTimer:
    """Per-step device timing with HIP events (falls back to wall clock on CPU)."""

    def __init__(self, device=None):
        self.cuda = device is not None and torch.device(device).type == "cuda"
        self.events: List = []
        self.walls: List[float] = []

    def mark(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.events.append(e)
        self.walls.append(time.perf_counter())

    def intervals_ms(self) -> List[float]:
        if self.cuda and len(self.events) > 1:
            self.events[-1].synchronize()
            return [a.elapsed_time(b) for a, b in zip(self.events[:-1], self.events[1:])]
        return [(b - a) * 1e3 for a, b in zip(self.walls[:-1], self.walls[1:])]
