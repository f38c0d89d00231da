"""In-memory datasets with the ``tf.data`` operations the reference uses.

The reference pipeline (``dist_model_tf_vgg.py:47-65,105-113``; copies in every script) is
``list_files -> map(process_path) -> take/skip -> cache -> shuffle(1000) -> batch(32) ->
prefetch``.  The IDC / CIFAR datasets are small (30k x 50x50x3 uint8 = 225 MB), so every
dataset here is an index view over ONE uint8 NHWC array held in host memory (optionally pinned)
or already on the GPU; ``take/skip/shard/shuffle`` are index arithmetic, and batches are gathered
straight into a device-resident staging buffer.

Quirk Q1 (train/val/test overlap because ``list_files`` reshuffles each iteration before
``take/skip``) is fixed: splits are disjoint slices of a seeded permutation.
"""
from __future__ import annotations

from typing import Iterator, Optional, Tuple

import numpy as np
import torch


class ArrayDataset:
    """Images ``x`` uint8/float [N,H,W,C] (NHWC) and labels ``y`` [N] (or one-hot [N,K])."""

    def __init__(self, x, y, index: Optional[np.ndarray] = None):
        self.x = x
        self.y = y
        n = x.shape[0]
        self.index = np.arange(n, dtype=np.int64) if index is None else np.asarray(index, np.int64)

    # --- tf.data-like views ------------------------------------------------------------
    def __len__(self):
        return int(self.index.shape[0])

    @property
    def element_shape(self) -> Tuple[int, ...]:
        return tuple(self.x.shape[1:])

    def _view(self, idx):
        return ArrayDataset(self.x, self.y, idx)

    def take(self, n: int) -> "ArrayDataset":
        return self._view(self.index[:n])

    def skip(self, n: int) -> "ArrayDataset":
        return self._view(self.index[n:])

    def shard(self, num_shards: int, index: int) -> "ArrayDataset":
        """``tf.data.Dataset.shard``: elements ``index, index+num_shards, ...``
        (``secure_fed_model.py:209``)."""
        return self._view(self.index[index::num_shards])

    def concatenate(self, other: "ArrayDataset") -> "ArrayDataset":
        assert other.x is self.x, "concatenate requires a shared backing array"
        return self._view(np.concatenate([self.index, other.index]))

    def shuffle(self, seed: int = 0) -> "ArrayDataset":
        """A one-off seeded permutation (use ``batch(shuffle=True)`` for per-epoch reshuffle)."""
        rng = np.random.default_rng(seed)
        return self._view(self.index[rng.permutation(len(self.index))])

    def cache(self) -> "ArrayDataset":
        return self  # already in memory

    def labels(self) -> np.ndarray:
        y = self.y[self.index] if isinstance(self.y, np.ndarray) else self.y[torch.as_tensor(self.index)].cpu().numpy()
        return y

    def filter_label(self, label: int) -> "ArrayDataset":
        lab = self.labels()
        if lab.ndim > 1:
            lab = lab.argmax(-1)
        return self._view(self.index[lab == label])

    def batch(self, batch_size: int, shuffle: bool = True, shuffle_buffer_size: int = 1000,
              drop_remainder: bool = False, seed: int = 0, repeat: int = 1) -> "BatchedDataset":
        return BatchedDataset(self, batch_size, shuffle, shuffle_buffer_size, drop_remainder,
                              seed, repeat)

    def to_device(self, device) -> "ArrayDataset":
        """Move the backing arrays to ``device`` once (datasets are small, HBM is 288 GB)."""
        x = torch.as_tensor(self.x).to(device)
        y = torch.as_tensor(self.y).to(device)
        return ArrayDataset(x, y, self.index)


def prepare_for_training(ds: ArrayDataset, batch_size: int = 32, cache=True,
                         shuffle_buffer_size: int = 1000, seed: int = 0,
                         drop_remainder: bool = False) -> "BatchedDataset":
    """The reference helper (``dist_model_tf_vgg.py:47-65``): cache -> shuffle -> batch -> prefetch."""
    return ds.cache().batch(batch_size, True, shuffle_buffer_size, drop_remainder, seed)


def _buffer_shuffle(index: np.ndarray, buf: int, rng: np.random.Generator) -> np.ndarray:
    """Exact ``tf.data`` shuffle-buffer semantics (a window of ``buf`` elements)."""
    n = index.shape[0]
    if buf >= n:
        return index[rng.permutation(n)]
    out = np.empty_like(index)
    pool = list(index[:buf])
    j = buf
    for i in range(n):
        k = int(rng.integers(len(pool)))
        out[i] = pool[k]
        if j < n:
            pool[k] = index[j]
            j += 1
        else:
            pool[k] = pool[-1]
            pool.pop()
    return out


class BatchedDataset:
    """Iterable of ``(x, y)`` batches; reshuffles every iteration like ``tf.data``."""

    def __init__(self, ds: ArrayDataset, batch_size: int, shuffle: bool, buffer: int,
                 drop_remainder: bool, seed: int, repeat: int = 1):
        self.ds = ds
        self.batch_size = int(batch_size)
        self.shuffle = shuffle
        self.buffer = buffer
        self.drop_remainder = drop_remainder
        self.seed = seed
        self.repeat = repeat
        self._epoch = 0
        self.device = None       # prefetch_to(): batches are delivered on this device
        self._prefetcher = None
        self._prefetcher_bs = None

    def prefetch_to(self, device) -> "BatchedDataset":
        """Deliver batches as ``device`` tensors through the native pinned-memory prefetcher
        (``tf.data``'s ``prefetch(AUTOTUNE)``, ``dist_model_tf_vgg.py:63``)."""
        device = torch.device(device)
        if self.device != device:
            self.device = device
            self._prefetcher = None
        return self

    def __len__(self):
        n = len(self.ds) * self.repeat
        return n // self.batch_size if self.drop_remainder else -(-n // self.batch_size)

    @property
    def element_shape(self):
        return self.ds.element_shape

    def epoch_order(self) -> np.ndarray:
        parts = []
        for r in range(self.repeat):
            idx = self.ds.index
            if self.shuffle:
                from . import native
                if native.available():
                    key = ((self.seed * 1000003 + self._epoch) * 1000003 + r) & ((1 << 64) - 1)
                    idx = native.shuffle_order(idx, self.buffer, key)
                else:
                    rng = np.random.default_rng((self.seed, self._epoch, r))
                    idx = _buffer_shuffle(idx, self.buffer, rng)
            parts.append(idx)
        self._epoch += 1
        return np.concatenate(parts) if len(parts) > 1 else parts[0]

    def shard(self, rank: int, world: int) -> "RankShard":
        """Data-parallel view: every rank draws the SAME global batch order (same seed and
        epoch) and takes its own contiguous ``batch_size / world`` rows of each global batch in
        INDEX space, so a rank only gathers and stages its own images (no replicated global batch
        sliced after the copy).  A trailing partial global batch is dropped under data
        parallelism (static per-rank shapes; its rows would not split evenly)."""
        return RankShard(self, rank, world)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        yield from self._iter_order(self.epoch_order(), self.batch_size, self.drop_remainder)

    def _iter_order(self, order: np.ndarray, bs: int, drop_remainder: bool):
        n = order.shape[0]
        stop = n - (n % bs) if drop_remainder else n
        x, y = self.ds.x, self.ds.y
        on_dev = isinstance(x, torch.Tensor) and x.is_cuda
        if isinstance(x, np.ndarray) and isinstance(y, np.ndarray) and stop > 0:
            from . import native
            if native.available():
                if self._prefetcher is None or self._prefetcher_bs != bs:
                    self._prefetcher = native.PrefetchIterator(x, y, bs, device=self.device)
                    self._prefetcher_bs = bs
                yield from self._prefetcher.epoch(order[:stop] if drop_remainder else order,
                                                  drop_remainder)
                return
        for s in range(0, stop, bs):
            idx = order[s:s + bs]
            if on_dev:
                ti = torch.as_tensor(idx, device=x.device)
                yield x.index_select(0, ti), y.index_select(0, ti)
            else:
                xb = x[idx] if isinstance(x, np.ndarray) else x[torch.as_tensor(idx)]
                yb = y[idx] if isinstance(y, np.ndarray) else y[torch.as_tensor(idx)]
                yield torch.as_tensor(xb), torch.as_tensor(yb)


class RankShard:
    """``BatchedDataset.shard``: rank ``rank``'s rows of every global batch."""

    def __init__(self, data: BatchedDataset, rank: int, world: int):
        if data.batch_size % world:
            raise ValueError(f"global batch {data.batch_size} does not split over {world} replicas")
        self.data, self.rank, self.world = data, rank, world
        self.per = data.batch_size // world

    def __len__(self):
        return len(self.data.ds) * self.data.repeat // self.data.batch_size

    def prefetch_to(self, device):
        self.data.prefetch_to(device)
        return self

    def rank_order(self, order: np.ndarray) -> np.ndarray:
        gb = self.data.batch_size
        nb = order.shape[0] // gb
        return order[:nb * gb].reshape(nb, gb)[:, self.rank * self.per:(self.rank + 1) * self.per].reshape(-1)

    def __iter__(self):
        yield from self.data._iter_order(self.rank_order(self.data.epoch_order()), self.per, True)


def to_float_images(x: torch.Tensor) -> torch.Tensor:
    """uint8 [0,255] -> float32 [0,1] (``tf.image.convert_image_dtype``; no ImageNet
    ``preprocess_input``, quirk Q12)."""
    if x.dtype == torch.uint8:
        return x.float().mul_(1.0 / 255.0)
    return x.float()
