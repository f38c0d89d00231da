"""Keras-style callbacks: ``History``, ``ModelCheckpoint``, ``JSONLLogger``.

``ModelCheckpoint(filepath, save_weights_only=True, verbose=1)`` mirrors ``fed_model.py:103-105``
(saved every epoch; here in the Keras HDF5 layout, see ``idc_models_amd.ckpt``).
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, List


class Callback:
    model = None

    def set_model(self, model):
        self.model = model

    def on_train_begin(self, logs=None): ...
    def on_train_end(self, logs=None): ...
    def on_epoch_begin(self, epoch, logs=None): ...
    def on_epoch_end(self, epoch, logs=None): ...
    def on_train_batch_end(self, step, logs=None): ...
    def on_epoch_train_end(self, epoch, logs=None): ...  # training batches done, before validation


class History(Callback):
    """``keras.callbacks.History``: ``.history`` dict of per-epoch lists, ``.epoch`` list."""

    def __init__(self):
        self.history: Dict[str, List[float]] = {}
        self.epoch: List[int] = []

    def on_train_begin(self, logs=None):
        self.epoch = []

    def on_epoch_end(self, epoch, logs=None):
        self.epoch.append(epoch)
        for k, v in (logs or {}).items():
            self.history.setdefault(k, []).append(v)


class ModelCheckpoint(Callback):
    def __init__(self, filepath: str, save_weights_only: bool = True, verbose: int = 0,
                 rank: int = 0):
        self.filepath = filepath
        self.save_weights_only = save_weights_only
        self.verbose = verbose
        self.rank = rank

    def on_epoch_end(self, epoch, logs=None):
        if self.rank != 0:
            return
        path = self.filepath.format(epoch=epoch + 1, **(logs or {}))
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        if self.save_weights_only:
            self.model.save_weights(path)
        else:
            self.model.save_checkpoint(path)
        if self.verbose:
            print(f"\nEpoch {epoch + 1:05d}: saving model to {path}")


class ThroughputMeter(Callback):
    """Training throughput of ``fit`` (the reference times whole fits with ``Timer``,
    ``dist_model_tf_vgg.py:135-138``; this separates the training epochs from validation):
    device-synchronised wall time of each epoch's training batches and images/sec of this rank
    (``images`` counts the rows this process trained on)."""

    def __init__(self):
        self.epoch_seconds: List[float] = []
        self.epoch_images: List[int] = []
        self._t0 = 0.0
        self._n = 0

    @staticmethod
    def _sync():
        import torch
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()

    def on_epoch_begin(self, epoch, logs=None):
        self._sync()
        self._t0 = time.perf_counter()
        self._n = 0

    def on_train_batch_end(self, step, logs=None):
        self._n += int((logs or {}).get("size", 0))

    def on_epoch_train_end(self, epoch, logs=None):
        self._sync()
        self.epoch_seconds.append(time.perf_counter() - self._t0)
        self.epoch_images.append(self._n)

    def images_per_sec(self, skip_first: bool = True) -> float:
        """Images/sec of this rank over the recorded epochs (the first one, which may build and
        tune programs, excluded when there are others)."""
        k = 1 if (skip_first and len(self.epoch_seconds) > 1) else 0
        t = sum(self.epoch_seconds[k:])
        return sum(self.epoch_images[k:]) / t if t > 0 else 0.0


class JSONLLogger(Callback):
    """Rank-0 JSONL metric log (one line per epoch)."""

    def __init__(self, path: str, rank: int = 0, extra=None):
        self.path = path
        self.rank = rank
        self.extra = extra or {}

    def on_epoch_end(self, epoch, logs=None):
        if self.rank != 0:
            return
        os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
        with open(self.path, "a") as f:
            f.write(json.dumps({"ts": time.time(), "epoch": epoch, **self.extra,
                                **(logs or {})}) + "\n")


class CallbackList:
    def __init__(self, callbacks, model):
        self.callbacks = list(callbacks or [])
        for c in self.callbacks:
            c.set_model(model)

    def __getattr__(self, name):
        def call(*a, **k):
            for c in self.callbacks:
                getattr(c, name)(*a, **k)
        return call
