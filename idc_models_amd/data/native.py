"""Python side of the native input pipeline (``csrc/data/loader.cpp`` -> ``_idc_data``).

Replaces the tf.data runtime the reference relies on (``list_files -> decode_png -> resize ->
cache -> shuffle(1000) -> batch -> prefetch``, ``dist_model_tf_vgg.py:34-65``):

* :func:`decode_pngs` — libpng decode + TF2 bilinear resize on C++ threads (no GIL);
* :func:`shuffle_order` — the shuffle-buffer permutation in C++;
* :class:`PrefetchIterator` — C++ worker threads gather upcoming batches into a ring of pinned host
  slots; each batch is copied to the device on a dedicated copy stream (``non_blocking``) while
  the GPU is still busy with the previous step, and the consumer's stream is ordered after the
  copy.  On a CPU-only host the slots are ordinary memory and batches are yielded as copies.

Every entry point falls back to the pure-Python implementation when the module is not built.
"""
from __future__ import annotations

import collections
import importlib
import os
import sys
from typing import Iterator, List, Optional, Tuple

import numpy as np
import torch

_MOD = None
_TRIED = False


def module():
    global _MOD, _TRIED
    if not _TRIED:
        _TRIED = True
        if os.environ.get("IDC_NATIVE_DATA", "1") != "0":
            pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
            if pkg not in sys.path:
                sys.path.insert(0, pkg)
            try:
                from ..utils.hostext import import_host_ext
                _MOD = import_host_ext("_idc_data")
            except ImportError:
                _MOD = None
    return _MOD


def available() -> bool:
    return module() is not None


def decode_pngs(files: List[str], size: int, workers: int = 8) -> Tuple[np.ndarray, List[Tuple[int, str]]]:
    """Decode ``files`` into a uint8 ``[N, size, size, 3]`` array; returns (array, failures)."""
    x = np.zeros((len(files), size, size, 3), np.uint8)
    bad = module().decode_pngs(list(files), int(size), x, int(workers))
    return x, list(bad)


def shuffle_order(index: np.ndarray, buffer: int, seed: int) -> np.ndarray:
    return module().shuffle_order(np.ascontiguousarray(index, dtype=np.int64), int(buffer),
                                  int(seed) & ((1 << 64) - 1))


class PrefetchIterator:
    """Iterate ``(x, y)`` batches of ``order`` over host arrays through the native batcher.

    ``device``: a CUDA device -> batches are returned as device tensors (pinned slot ->
    ``non_blocking`` copy on a side stream -> the consumer stream waits for it); ``None`` or CPU ->
    host tensors (copies of the slot, so the caller may keep them).
    """

    def __init__(self, x: np.ndarray, y: np.ndarray, batch: int, device=None, slots: int = 4,
                 threads: int = 2):
        self.x = np.ascontiguousarray(x)
        self.y = np.ascontiguousarray(y)
        self.batch = int(batch)
        dev = torch.device(device) if device is not None else torch.device("cpu")
        self.device = dev
        self.on_gpu = dev.type == "cuda" and torch.cuda.is_available()
        pin = self.on_gpu
        xshape = (self.batch,) + tuple(self.x.shape[1:])
        yshape = (self.batch,) + tuple(self.y.shape[1:])
        xt = torch.from_numpy(self.x[:1]).dtype
        yt = torch.from_numpy(self.y[:1]).dtype
        self.xs = [torch.empty(xshape, dtype=xt, pin_memory=pin) for _ in range(slots)]
        self.ys = [torch.empty(yshape, dtype=yt, pin_memory=pin) for _ in range(slots)]
        self.loader = module().BatchLoader(self.x, self.y, self.batch,
                                           [t.data_ptr() for t in self.xs],
                                           [t.data_ptr() for t in self.ys], int(threads))
        self.copy_stream = torch.cuda.Stream(device=dev) if self.on_gpu else None
        self.pending = collections.deque()  # (slot, event) whose H2D copy may still be running

    def _retire(self, force_all: bool = False):
        keep = max(self.loader.num_slots - 2, 0)  # keep two slots free for the workers
        while self.pending:
            slot, ev = self.pending[0]
            if ev is not None and not ev.query():
                if not force_all and len(self.pending) <= keep:
                    break
                ev.synchronize()
            self.loader.release(slot)
            self.pending.popleft()

    def epoch(self, order: np.ndarray, drop_remainder: bool = False) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        self._retire(force_all=True)
        self.loader.start_epoch(np.ascontiguousarray(order, dtype=np.int64), bool(drop_remainder))
        while True:
            self._retire()
            slot, n = self.loader.next()
            if slot < 0:
                break
            xs, ys = self.xs[slot][:n], self.ys[slot][:n]
            if self.on_gpu:
                cur = torch.cuda.current_stream(self.device)
                with torch.cuda.stream(self.copy_stream):
                    xd = xs.to(self.device, non_blocking=True)
                    yd = ys.to(self.device, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.copy_stream)
                cur.wait_stream(self.copy_stream)
                xd.record_stream(cur)
                yd.record_stream(cur)
                self.pending.append((slot, ev))
                yield xd, yd
            else:
                xb, yb = xs.clone(), ys.clone()
                self.loader.release(slot)
                yield xb, yb
        self._retire(force_all=True)

    def close(self):
        self._retire(force_all=True)
        self.loader.shutdown()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
