"""Python face of the native RCCL communicator (``csrc/comm/communicator.cpp``).

SURVEY §5 asks for a C++ ``Communicator`` that owns the ``ncclComm_t`` and a comm stream, so the
gradient all-reduces of the data-parallel step are issued by the native plan executor (op kind
``OP_ALLREDUCE``, ordered with HIP events against the main and weight-gradient lanes) instead of
one Python ``dist.all_reduce`` call per bucket.  Reference: the NCCL all-reduce that
``tf.distribute.MirroredStrategy`` runs inside every step (``dist_model_tf_vgg.py:115``).

Bootstrap: rank 0 creates the 128-byte RCCL unique id, publishes it in the ``torch.distributed``
TCPStore, every rank reads it and joins (``ncclCommInitRank``).  A world of one needs no store.
"""
from __future__ import annotations

import itertools
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

    def __init__(self, rank: int, world: int, device, store=None, timeout_s: float = 600.0):
        ext = nat.require()
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
        self.c = ext.Communicator(self.rank, self.world, bytes(uid), self.device.index or 0)

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
        self.c.check_async()

    def close(self):
        if self.c is not None:
            self.c.close()
            self.c = None
