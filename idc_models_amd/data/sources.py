"""Dataset sources: IDC PNG directories, CIFAR-10 binaries and synthetic patches.

* IDC balanced: ``{path}/data/balanced_IDC_30k/{0,1}/*.png`` (``dist_model_tf_vgg.py:105``,
  ``fed_model.py:159-163``, ``secure_fed_model.py:217``).
* IDC Kaggle layout: ``{path}/data/IDC_regular_ps50_idx5/{patient}/{0,1}/*.png``
  (``dist_model_tf_mobile.py:105``).
* label = (parent directory name == '1') (``get_label``, ``dist_model_tf_vgg.py:34-36``); decode
  PNG to 3 channels, scale to [0,1], bilinear resize to SxS (``decode_img``, ``:37-40``; 10x10 in
  ``secure_fed_model.py:176-179``).
* CIFAR-10 (the reference uses ``tfds.load('cifar10')``, ``dist_model_tf_dense.py:120``; there is no
  network, so the standard binary release ``data_batch_{1..5}.bin``/``test_batch.bin`` is read).
* Synthetic: deterministic 50x50x3 uint8 patches whose colour statistics depend on the label,
  so models can actually learn (used by the benchmark and tests; BASELINE.json "synthetic").

Decoded images are cached as one uint8 NHWC array (``.cache()`` in the reference); PNG decode
runs in a thread pool (PIL releases the GIL).
"""
from __future__ import annotations

import glob
import os
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional, Tuple

import numpy as np

from .dataset import ArrayDataset


def _load_png(path: str, size: int) -> np.ndarray:
    from PIL import Image

    with Image.open(path) as im:
        im = im.convert("RGB")
        if im.size != (size, size):
            # TF bilinear resize (half-pixel centers, no antialias) ~ PIL BILINEAR w/o reducing
            im = im.resize((size, size), Image.BILINEAR)
        return np.asarray(im, dtype=np.uint8)


def list_idc_files(path: str, layout: str = "balanced", label: Optional[int] = None) -> List[str]:
    if layout == "balanced":
        pat = os.path.join(path, "data", "balanced_IDC_30k", "*" if label is None else str(label), "*")
    elif layout == "patient":
        pat = os.path.join(path, "data", "IDC_regular_ps50_idx5", "*",
                           "*" if label is None else str(label), "*")
    else:
        raise ValueError(layout)
    return sorted(glob.glob(pat))


def label_of(file_path: str) -> int:
    return int(os.path.basename(os.path.dirname(file_path)) == "1")


def load_files(files: List[str], size: int = 50, workers: int = 8) -> ArrayDataset:
    y = np.array([label_of(f) for f in files], np.int64)
    from . import native
    if native.available():  # libpng + resize on C++ threads (csrc/data/loader.cpp)
        x, bad = native.decode_pngs(files, size, workers)
        if bad:
            raise ValueError(f"{len(bad)} images failed to decode, first: {bad[0][1]}")
        return ArrayDataset(x, y)
    x = np.zeros((len(files), size, size, 3), np.uint8)

    def work(i):
        x[i] = _load_png(files[i], size)

    with ThreadPoolExecutor(max_workers=workers) as ex:
        list(ex.map(work, range(len(files))))
    return ArrayDataset(x, y)


def idc_dataset(path: str, layout: str = "balanced", size: int = 50, seed: int = 0,
                iid: bool = True, max_files: Optional[int] = None) -> ArrayDataset:
    """IDC patches.  ``iid=False`` reproduces ``get_data`` non-IID ordering
    (``fed_model.py:157-165``): all class-1 files, then all class-0 files (each list shuffled)."""
    rng = np.random.default_rng(seed)
    if iid:
        files = list_idc_files(path, layout)
        files = [files[i] for i in rng.permutation(len(files))]
    else:
        f1 = list_idc_files(path, layout, 1)
        f0 = list_idc_files(path, layout, 0)
        files = [f1[i] for i in rng.permutation(len(f1))] + [f0[i] for i in rng.permutation(len(f0))]
    if max_files is not None:
        files = files[:max_files]
    if not files:
        raise FileNotFoundError(f"no IDC images under {path} (layout={layout})")
    return load_files(files, size)


def cifar10_dataset(root: str, train: bool = True) -> ArrayDataset:
    names = [f"data_batch_{i}.bin" for i in range(1, 6)] if train else ["test_batch.bin"]
    xs, ys = [], []
    for n in names:
        p = os.path.join(root, n)
        raw = np.fromfile(p, dtype=np.uint8).reshape(-1, 3073)
        ys.append(raw[:, 0].astype(np.int64))
        xs.append(raw[:, 1:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1))
    return ArrayDataset(np.ascontiguousarray(np.concatenate(xs)), np.concatenate(ys))


def synthetic_dataset(n: int, shape: Tuple[int, int, int] = (50, 50, 3), num_classes: int = 2,
                      seed: int = 0, signal: float = 24.0, label_noise: float = 0.0) -> ArrayDataset:
    """Deterministic synthetic patches: noise + a label-dependent colour/texture offset.

    ``signal``: strength of the class offset (24 is trivially separable; the benchmark's
    validation set uses a weak one).  ``label_noise``: each label is re-drawn uniformly with this
    probability AFTER the images are made, so no model can exceed the noise ceiling (binary,
    re-draw probability p: a fraction p/2 ends up flipped, held-out AUC <= 1 - p/2)."""
    rng = np.random.default_rng(seed)
    h, w, c = shape
    y = rng.integers(0, num_classes, size=n).astype(np.int64)
    base = rng.normal(128.0, 40.0, size=(n, h, w, c)).astype(np.float32)
    # class-dependent channel shift and a low-frequency stripe pattern
    shift = np.linspace(-1.0, 1.0, num_classes, dtype=np.float32)[y]
    chan = np.array([1.0, -0.5, 0.25], np.float32)[:c]
    stripes = np.sin(np.arange(w, dtype=np.float32) * 0.5)[None, None, :, None]
    base += signal * shift[:, None, None, None] * chan[None, None, None, :]
    base += (signal * 0.5) * shift[:, None, None, None] * stripes
    x = np.clip(base, 0, 255).astype(np.uint8)
    if label_noise > 0:
        flip = rng.random(n) < label_noise
        y = np.where(flip, rng.integers(0, num_classes, size=n), y).astype(np.int64)
    return ArrayDataset(x, y)


def split(ds: ArrayDataset, fractions=(0.8, 0.1, 0.1)):
    """Disjoint take/skip splits (``dist_model_tf_vgg.py:108-110``, fixed quirk Q1)."""
    n = len(ds)
    sizes = [int(f * n) for f in fractions]
    sizes[-1] = n - sum(sizes[:-1])
    out, off = [], 0
    for s in sizes:
        out.append(ds.skip(off).take(s))
        off += s
    return out
