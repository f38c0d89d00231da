"""Python face of the native RCCL communicator (``csrc/comm/communicator.cpp``).

SURVEY §5 asks for a C++ ``Communicator`` that owns the ``ncclComm_t`` and a comm stream, so the
gradient all-reduces of the data-parallel step are issued by the native plan executor (op kind
``OP_ALLREDUCE``, ordered with HIP events against the main and weight-gradient lanes) instead of
one Python ``dist.all_reduce`` call per bucket.  Reference: the NCCL all-reduce that
``tf.distribute.MirroredStrategy`` runs inside every step (``dist_model_tf_vgg.py:115``).

Bootstrap: rank 0 creates the 128-byte RCCL unique id, publishes it in the ``torch.distributed``
TCPStore, every rank reads it and joins.  A world of one needs no store.  With more than one rank
the communicator is created non-blocking (``ncclCommInitRankConfig``) and a rank whose peers do not
join within ``IDC_COMM_INIT_TIMEOUT`` seconds (default 300) raises instead of hanging; a
``CommWatchdog`` (``parallel/watchdog.py``) then aborts the communicator when RCCL reports an
asynchronous error or a step's collectives make no progress for ``IDC_COMM_TIMEOUT`` seconds
(default 300; ``IDC_COMM_WATCHDOG=0`` turns it off).
"""
from __future__ import annotations

import itertools
import os
from typing import Optional

import torch

from ..ops import _native as nat

DTYPES = {torch.float32: 0, torch.bfloat16: 1, torch.int32: 2, torch.float64: 3, torch.int64: 5,
          torch.uint8: 6}
OPS = {"sum": 0, "max": 1, "min": 2, "avg": 3}

_SEQ = itertools.count()


def _op_code(op) -> int:
    if isinstance(op, str):
        return OPS[op]
    import torch.distributed as dist
    table = {dist.ReduceOp.SUM: 0, dist.ReduceOp.MAX: 1, dist.ReduceOp.MIN: 2}
    if hasattr(dist.ReduceOp, "AVG"):
        table[dist.ReduceOp.AVG] = 3
    return table[op]


class NativeCommunicator:
    """One RCCL communicator over the ranks of the default process group (or a world of one)."""

    def __init__(self, rank: int, world: int, device, store=None, timeout_s: float = 600.0, ext=None,
                 watchdog: Optional[bool] = None, init_timeout_s: Optional[float] = None):
        """``ext``: the native module (tests pass a fake to exercise the bootstrap on the CPU).
        ``init_timeout_s``: > 0 creates the communicator non-blocking with that timeout (default:
        IDC_COMM_INIT_TIMEOUT, 300 s, for a world > 1; blocking for a world of one)."""
        ext = ext if ext is not None else nat.require()
        self.rank, self.world = int(rank), int(world)
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("NativeCommunicator needs a GPU device")
        key = f"idc_rccl_uid/{next(_SEQ)}"
        if self.world == 1:
            uid = ext.Communicator.make_unique_id()
        else:
            if store is None:
                from torch.distributed import distributed_c10d as c10d
                store = c10d._get_default_store()
            if self.rank == 0:
                uid = ext.Communicator.make_unique_id()
                store.set(key, uid)
            else:
                store.wait([key])
                uid = store.get(key)
        if init_timeout_s is not None:
            init_timeout = float(init_timeout_s)
        else:
            init_timeout = float(os.environ.get("IDC_COMM_INIT_TIMEOUT", "300")) if self.world > 1 else 0.0
        self.c = ext.Communicator(self.rank, self.world, bytes(uid), self.device.index or 0, init_timeout)
        self.watchdog = None
        if watchdog is None:
            watchdog = self.world > 1 and os.environ.get("IDC_COMM_WATCHDOG", "1") != "0"
        if watchdog:
            from .watchdog import CommWatchdog
            self.watchdog = CommWatchdog(self.c, timeout_s=float(os.environ.get("IDC_COMM_TIMEOUT", "300")),
                                         name=f"rccl rank {self.rank}/{self.world}").start()

    # ------------------------------------------------------------------ properties
    @property
    def stream_handle(self) -> int:
        return int(self.c.stream)

    @property
    def collectives(self) -> int:
        return int(self.c.collectives)

    @staticmethod
    def version() -> str:
        v = int(nat.require().rccl_version())
        return f"{v // 10000}.{(v // 100) % 100}.{v % 100}"

    # ------------------------------------------------------------------ collectives
    def _stream(self, stream) -> int:
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        return int(s.cuda_stream)

    @staticmethod
    def _check(t: torch.Tensor):
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("native collectives need contiguous device tensors")
        if t.dtype not in DTYPES:
            raise TypeError(f"unsupported dtype {t.dtype}")

    def all_reduce_(self, t: torch.Tensor, op="sum", stream: Optional[torch.cuda.Stream] = None):
        """In-place all-reduce, enqueued on ``stream`` (default: the current torch stream)."""
        self._check(t)
        self.c.all_reduce(t.data_ptr(), t.numel(), DTYPES[t.dtype], _op_code(op), self._stream(stream))
        return t

    def all_reduce_u32_(self, t: torch.Tensor, stream: Optional[torch.cuda.Stream] = None):
        """In-place SUM modulo 2^32 of a 4-byte integer tensor read as uint32 (``ncclUint32``)."""
        self._check(t)
        if t.element_size() != 4 or t.dtype.is_floating_point:
            raise TypeError("all_reduce_u32_ needs a 32-bit integer tensor")
        self.c.all_reduce(t.data_ptr(), t.numel(), 4, 0, self._stream(stream))
        return t

    def reduce_(self, t: torch.Tensor, root: int = 0, op="sum", stream=None):
        self._check(t)
        self.c.reduce(t.data_ptr(), t.numel(), DTYPES[t.dtype], _op_code(op), int(root), self._stream(stream))
        return t

    def broadcast_(self, t: torch.Tensor, root: int = 0, stream=None):
        self._check(t)
        self.c.broadcast(t.data_ptr(), t.numel(), DTYPES[t.dtype], int(root), self._stream(stream))
        return t

    def all_gather(self, t: torch.Tensor, stream=None) -> torch.Tensor:
        """Concatenation of every rank's ``t`` along a new leading dimension."""
        self._check(t)
        out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        self.c.all_gather(t.data_ptr(), out.data_ptr(), t.numel(), DTYPES[t.dtype], self._stream(stream))
        return out

    def check(self):
        """Raise if the watchdog aborted the communicator or RCCL reports an asynchronous error."""
        if self.watchdog is not None:
            self.watchdog.raise_if_failed()
        if self.c is not None:
            self.c.check_async()

    def step_issued(self):
        """After a step's collectives were enqueued: a progress mark for the watchdog, and the
        failure (if any) it detected on an earlier step raised here, on the training thread."""
        if self.watchdog is not None:
            self.watchdog.raise_if_failed()
            self.watchdog.mark()

    def close(self):
        if self.watchdog is not None:
            self.watchdog.stop()
            failed = self.watchdog.error is not None
            self.watchdog = None
            if failed:  # aborted: nothing left to destroy
                self.c = None
        if self.c is not None:
            self.c.close()
            self.c = None


# ---- one communicator per rank ------------------------------------------------------------------
# The strategy's gradient buckets, the federated sums and the secure-aggregation ring all use the
# SAME communicator of a rank (one RCCL context, one comm stream, one watchdog), created on first
# use and keyed by the default group and device.
_SHARED: dict = {}


def _group_key(world: int, device: torch.device):
    import torch.distributed as dist
    g = id(dist.group.WORLD) if dist.is_available() and dist.is_initialized() else None
    return (g, int(world), device.index or 0)


def shared_communicator(rank: int, world: int, device, **kw) -> NativeCommunicator:
    """The rank's native communicator over the default group (created on first use; a closed or
    aborted one is replaced).  ``kw`` go to the constructor when it is created."""
    dev = torch.device(device)
    key = _group_key(world, dev)
    nc = _SHARED.get(key)
    if nc is None or nc.c is None:
        nc = NativeCommunicator(rank, world, dev, **kw)
        _SHARED[key] = nc
    return nc


def release_shared(nc: Optional[NativeCommunicator]):
    """Close ``nc`` and forget it (every holder of the rank's communicator sees it closed)."""
    if nc is None:
        return
    for k, v in list(_SHARED.items()):
        if v is nc:
            del _SHARED[k]
    nc.close()
