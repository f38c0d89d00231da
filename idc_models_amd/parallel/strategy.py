"""Distribution strategies (one process per device).

Reference: ``tf.distribute.MirroredStrategy`` (``dist_model_tf_vgg.py:115-117``,
``dist_model_tf_mobile.py:115``, ``dist_model_tf_dense.py:20-22``) and
``CentralStorageStrategy`` (``dist_model_tf_dense.py:18,24``).  TF drives N GPUs from ONE process;
on MI355X the idiomatic form is one process per GPU over RCCL:

* ``OneDeviceStrategy`` — single device (CPU plumbing config or 1 GPU).
* ``MirroredStrategy`` — rank-0 broadcast at model creation (C2), bucketed SUM all-reduce of the
  flat gradient arena overlapped with backward (C1), 1/N folded into the optimizer, every rank
  applies the same update; metrics reduced once per epoch (C3); BN moving statistics averaged at
  epoch end (C4: sync-on-read MEAN).  ``global_batch`` semantics: each batch yielded by the
  dataset is the GLOBAL batch and rank r takes rows [r*B/N, (r+1)*B/N) — the vgg/mobile
  convention; the dense script's ``256 * num_replicas`` global batch is the same thing.
* ``CentralStorageStrategy`` — variables and optimizer state are owned by rank 0: gradients are
  ``reduce``-d to rank 0, rank 0 applies RMSprop, parameters are ``broadcast`` back (C5).

On a GPU with the ``nccl`` (= RCCL) backend the strategy also owns a native RCCL communicator
(``parallel/native_comm.py``): the fused runtime then issues its bucket all-reduces from the C++
plan on the communicator's stream (no Python per bucket).  ``force_collectives=True`` (or
``IDC_FORCE_COLLECTIVES=1``) runs every collective even in a world of one rank, so the whole RCCL
path is exercised on a one-GPU machine.
"""
from __future__ import annotations

import contextlib
import os
from typing import List, Optional

import torch
import torch.distributed as dist

from . import comm
from .buckets import DEFAULT_BUCKET_BYTES, GradBucketer


class Strategy:
    def __init__(self, device=None):
        self.rank, self.world, self.local_rank = 0, 1, 0
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        device = torch.device(device)
        if device.type == "cuda" and device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self._bucketers = {}

    @property
    def num_replicas_in_sync(self) -> int:
        return self.world

    @property
    def active(self) -> bool:
        """Collectives run (more than one replica, or forced in a world of one)."""
        return False

    native_comm = None

    @property
    def is_chief(self) -> bool:
        return self.rank == 0

    def scope(self):
        from ..engine.model import strategy_scope
        return strategy_scope(self)

    # hooks used by engine.Model ------------------------------------------------------
    def broadcast_module(self, net):
        pass

    def apply_gradients(self, optimizer, arena):
        """Reduce gradients across replicas (if any) and apply the optimizer update."""
        optimizer.step(arena)

    def reduce_metrics(self, metrics):
        pass

    def sync_bn_stats(self, model):
        pass

    def distribute(self, data):
        return data

    def bucketer(self, arena):
        return None


class OneDeviceStrategy(Strategy):
    pass


_DEFAULT = None


def default_strategy() -> Strategy:
    global _DEFAULT
    if _DEFAULT is None:
        _DEFAULT = OneDeviceStrategy()
    return _DEFAULT


class MirroredStrategy(Strategy):
    def __init__(self, devices=None, bucket_bytes: int = DEFAULT_BUCKET_BYTES, backend=None,
                 device=None, force_collectives: Optional[bool] = None, native_comm: Optional[bool] = None):
        """``device`` overrides the per-rank device (e.g. several gloo ranks sharing one GPU to
        rehearse the data-parallel path on a single-GPU machine).  ``native_comm``: own an RCCL
        communicator for the fused runtime's gradient buckets (default: on for nccl on a GPU)."""
        if force_collectives is None:
            force_collectives = os.environ.get("IDC_FORCE_COLLECTIVES", "0") == "1"
        rank, world, local = comm.init_process_group(backend, force=force_collectives)
        if device is not None:
            dev = torch.device(device)
            if dev.type == "cuda":
                torch.cuda.set_device(dev)
        elif torch.cuda.is_available() and (backend in (None, "nccl")):
            torch.cuda.set_device(local)
            dev = torch.device("cuda", local)
        else:
            dev = torch.device("cpu")
        super().__init__(dev)
        self.rank, self.world, self.local_rank = rank, world, local
        self.bucket_bytes = bucket_bytes
        self.devices = devices
        self.forced = bool(force_collectives) and world == 1
        self.native_comm = None
        if native_comm is None:
            native_comm = os.environ.get("IDC_NATIVE_COMM", "1") != "0"
        if native_comm and self.active and dev.type == "cuda" and comm.backend() == "nccl":
            from .native_comm import shared_communicator
            self.native_comm = shared_communicator(rank, world, dev)

    @property
    def active(self) -> bool:
        return self.world > 1 or self.forced

    def close(self):
        """Release the native communicator and the process group (end of a run)."""
        if self.native_comm is not None:
            from .native_comm import release_shared
            release_shared(self.native_comm)
            self.native_comm = None
        comm.destroy()

    def broadcast_module(self, net):
        if not self.active:
            return
        with torch.no_grad():
            for t in net.weight_tensors():
                comm.broadcast_(t.data, 0)

    def bucketer(self, arena):
        key = id(arena)
        b = self._bucketers.get(key)
        if b is None or b.arena is not arena:
            b = GradBucketer(arena, self.bucket_bytes)
            b.install_hooks()
            self._bucketers = {key: b}
        return b

    def apply_gradients(self, optimizer, arena):
        if not self.active:
            optimizer.step(arena)
            return
        self.bucketer(arena).finish()
        optimizer.step(arena, grad_scale=1.0 / self.world)

    def reduce_metrics(self, metrics):
        if not self.active:
            return
        states, owners = [], []
        for m in metrics:
            st = m.state()
            if st:
                states.extend(st)
                owners.append((m, len(st)))
        red = comm.pack_all_reduce(states)
        i = 0
        for m, n in owners:
            m.set_state(red[i:i + n])
            i += n
        # exact AUC needs all scores: gather them (small: one float per example)
        from ..engine.metrics import AUC
        for m in metrics:
            if isinstance(m, AUC) and m.mode == "exact" and m.scores:
                s, l = m.gather_arrays()
                n = torch.tensor([s.numel()], device=self.device)
                sizes = [torch.zeros_like(n) for _ in range(self.world)]
                dist.all_gather(sizes, n)
                mx = int(max(int(x) for x in sizes))
                pad = torch.full((mx,), float("nan"), device=s.device)
                pad[:s.numel()] = s
                padl = torch.zeros(mx, device=s.device)
                padl[:l.numel()] = l
                gs = [torch.empty_like(pad) for _ in range(self.world)]
                gl = [torch.empty_like(padl) for _ in range(self.world)]
                dist.all_gather(gs, pad)
                dist.all_gather(gl, padl)
                ss = torch.cat([g[:int(k)] for g, k in zip(gs, sizes)])
                ll = torch.cat([g[:int(k)] for g, k in zip(gl, sizes)])
                m.scores, m.labels = [ss], [ll]

    def sync_bn_stats(self, model):
        if not self.active:
            return
        from ..models.layers import BatchNormalization
        if model.impl is not None:
            model.impl.sync_to_module()
        bufs = []
        for l in _all_layers(model.net):
            if isinstance(l, BatchNormalization):
                bufs += [l.moving_mean, l.moving_variance]
        if not bufs:
            return
        red = comm.pack_all_reduce(bufs)
        with torch.no_grad():
            for b, r in zip(bufs, red):
                b.copy_(r / self.world)
        if model.impl is not None:
            model.impl.sync_from_module()

    def distribute(self, data):
        if self.world == 1:
            return data
        if hasattr(data, "shard"):  # BatchedDataset: shard the index order, not the images
            return data.shard(self.rank, self.world)
        return _ShardedBatches(data, self.rank, self.world)


class CentralStorageStrategy(MirroredStrategy):
    """Params + optimizer state owned by rank 0: reduce -> update on root -> broadcast."""

    central_storage = True

    def bucketer(self, arena):
        return None

    def apply_gradients(self, optimizer, arena):
        if not self.active:
            optimizer.step(arena)
            return
        self.reduce_to_root(arena.grad)
        if self.rank == 0:
            optimizer.step(arena, grad_scale=1.0 / self.world)
        self.broadcast_from_root(arena.data)

    def reduce_to_root(self, t, stream=None):
        """SUM-reduce ``t`` to rank 0 (native RCCL on the given / current stream when owned)."""
        if self.native_comm is not None:
            self.native_comm.reduce_(t, 0, "sum", stream)
        else:
            with torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext():
                dist.reduce(t, 0, op=dist.ReduceOp.SUM)

    def broadcast_from_root(self, t, stream=None):
        if self.native_comm is not None:
            self.native_comm.broadcast_(t, 0, stream)
        else:
            with torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext():
                dist.broadcast(t, 0)


# weight of the current local batch in the global-batch mean (set by _ShardedBatches while a
# replica's slice of an unevenly split batch is being trained; read by the training steps)
current_replica_weight = [1.0]


class _ShardedBatches:
    """Fallback for arbitrary iterables of global batches: rank ``r`` takes its contiguous slice
    of every batch.  Uneven batches are split as evenly as possible (the first ``b % world``
    ranks get one extra row); a batch with fewer rows than replicas ends the epoch on every
    rank alike (every rank sees the same batch sizes, so they stay in step)."""

    def __init__(self, data, rank, world):
        self.data, self.rank, self.world = data, rank, world

    def __len__(self):
        return len(self.data)

    def __iter__(self):
        st = current_replica_weight
        for x, y in self.data:
            b = x.shape[0]
            if b < self.world:
                return
            per, extra = divmod(b, self.world)
            lo = self.rank * per + min(self.rank, extra)
            hi = lo + per + (1 if self.rank < extra else 0)
            # the global-batch mean (TF scales each replica's loss by 1 / global batch): a replica
            # holding n of the b rows weighs its local-mean gradient by n * world / b before the
            # SUM all-reduce and the optimizer's 1 / world (1 when the split is even)
            st[0] = (hi - lo) * self.world / b
            try:
                yield x[lo:hi], y[lo:hi]
            finally:
                st[0] = 1.0



def _all_layers(net):
    for l in getattr(net, "layers", []):
        yield l
        if hasattr(l, "layers") and l is not net:
            yield from _all_layers(l)
