"""Grouped programs: K copies of one lowered program executed by single launches.

Client-batched federated training (SURVEY §2.3 D5 ``ClientScheduler``).  The K
clients a rank simulates share one architecture, so instead of K per-client programs of ~300 small
launches per step (240k dispatches per MobileNetV2 FedAvg round) the rank runs ONE program whose
every launch covers all K clients:

* a ``GroupRegion`` is one device slab of ``K * stride`` bytes.  The worker model, its parameter
  arena, optimizer slots and the whole lowered program (activations, statistics, tickets, split-K
  slabs, descriptor tables ...) are allocated inside copy 0 of it: every torch allocation made
  while they are built goes to a ``torch.cuda.MemPool`` whose pluggable allocator is the native
  bump allocator over copy 0 (``csrc/runtime/plan.cpp`` ``idc_region_malloc``);
* ``validate_program`` proves that every pointer in every op (argument structs, raw pointer
  operands and the device descriptor tables) lies inside copy 0;
* copy g of any buffer is then ``copy 0 + g * stride``: the kernels take a ``GroupArg`` and shift
  every pointer they dereference by ``(blockIdx.z / zn) * stride`` (``csrc/kernels/common.h``), and
  the launchers multiply their grid's z extent by K (``Plan.set_groups``);
* per-client state (weights, BN statistics, RMSprop slots, inputs, labels, losses) is addressed
  from Python as ``[K, ...]`` strided views of the slab (``view``).

Reference: TFF runs the clients of a round one after another in one process
(``fed_model.py:207-229``); the secure loop likewise (``secure_fed_model.py:224-233``).
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
from typing import List, Optional

import torch

from ..ops import _native as nat

_PAYLOAD = {
    nat.OP_CONV: nat.ConvArgs, nat.OP_WGRAD: nat.WgradArgs, nat.OP_BN_BWD_APPLY: nat.BnBwdApplyArgs,
    nat.OP_BN_BWD_REDUCE: nat.BnBwdReduceArgs, nat.OP_MAXPOOL: nat.PoolArgs, nat.OP_AVGPOOL: nat.PoolArgs,
    nat.OP_POOL_BWD: nat.PoolBwdArgs, nat.OP_HEAD_FWD: nat.HeadArgs, nat.OP_HEAD_BWD: nat.HeadBwdArgs,
    nat.OP_BN_APPLY: nat.BnArgs, nat.OP_DW_FWD: nat.DwArgs, nat.OP_DW_BWD_DATA: nat.DwArgs,
    nat.OP_DW_WGRAD: nat.DwArgs, nat.OP_MLP_FWD: nat.Mlp2Args, nat.OP_MLP_BWD: nat.Mlp2Args,
    nat.OP_DENSE_STAGE: nat.DenseStageArgs, nat.OP_MB_CHAIN: nat.MbChainArgs,
}
# descriptor-table ops: (ptr slot of the table, int slot of its length, entry type)
_TABLES = {nat.OP_BN_MOVING: (0, 0, nat.BnMovingDesc), nat.OP_STATS_SHIFT: (0, 0, nat.ShiftDesc),
           nat.OP_CAST: (0, 0, nat.CastEntry), nat.OP_WGRAD_BATCH: (0, 0, nat.WgBatchEntry),
           nat.OP_DENSE_STAGE: (0, 1, nat.DenseLayerDesc), nat.OP_MB_CHAIN: (0, 2, nat.MbPhaseDesc)}


def _struct_ptrs(obj, path=""):
    """(field path, value) of every pointer field of a ctypes struct, nested structs included."""
    for name, typ in obj._fields_:
        v = getattr(obj, name)
        if typ is C.c_void_p:
            yield path + name, int(v or 0)
        elif isinstance(v, C.Structure):
            yield from _struct_ptrs(v, path + name + ".")


def default_stride_bytes() -> int:
    return int(os.environ.get("IDC_GROUP_REGION_MB", "1024")) << 20


# Every region's MemPool (and the slab its blocks live in) stays alive for the whole process,
# interpreter shutdown included: torch requires a pool to outlive every block it handed out, and
# the model / program tensors of a grouped worker are released in arbitrary order when they are
# garbage-collected or when the interpreter tears its modules down.  The pool objects therefore
# get one extra reference that is never dropped.  Regions are created once per federated process,
# so this is a bounded, deliberate leak.
_KEEP_ALIVE: list = []


def _pin_forever(obj):
    C.pythonapi.Py_IncRef(C.py_object(obj))
    _KEEP_ALIVE.append(obj)


class GroupRegion:
    """K equally spaced copies of a program's memory (see module docstring)."""

    def __init__(self, k: int, device, stride_bytes: Optional[int] = None):
        if k < 1:
            raise ValueError("a group needs at least one copy")
        self.k = int(k)
        self.device = torch.device(device)
        self.stride = int(stride_bytes or default_stride_bytes())
        self.stride = (self.stride + 4095) // 4096 * 4096
        self.slab = torch.zeros(self.k * self.stride, dtype=torch.uint8, device=self.device)
        self.base = self.slab.data_ptr()
        self.ext = nat.require()
        self.ext.region_activate(self.base, self.stride)
        from torch.cuda.memory import CUDAPluggableAllocator
        self._alloc = CUDAPluggableAllocator(self.ext.__file__, "idc_region_malloc", "idc_region_free")
        self.pool = torch.cuda.MemPool(self._alloc.allocator())
        for o in (self.pool, self._alloc, self.slab):
            _pin_forever(o)

    # ------------------------------------------------------------------ allocation
    @contextlib.contextmanager
    def allocating(self):
        """Every torch allocation on this thread inside the block lands in copy 0."""
        self.ext.region_activate(self.base, self.stride)
        with torch.cuda.use_mem_pool(self.pool):
            yield self

    @property
    def used(self) -> int:
        return int(self.ext.region_used(self.base))

    def contains(self, ptr: int, nbytes: int = 1) -> bool:
        return self.base <= ptr and ptr + nbytes <= self.base + self.stride

    def replicate(self, stream: Optional[torch.cuda.Stream] = None):
        """Copies 1..K-1 become byte copies of copy 0 (its used part), ordered on ``stream``."""
        n = self.used
        if self.k == 1 or n == 0:
            return
        src = self.slab[:n]
        ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
        with ctx:
            if stream is not None:
                stream.wait_stream(torch.cuda.current_stream(self.device))
            dst = self.slab.as_strided((self.k - 1, n), (self.stride, 1), self.stride)
            dst.copy_(src.unsqueeze(0).expand(self.k - 1, n))

    def view(self, t: torch.Tensor) -> torch.Tensor:
        """``[K, *t.shape]`` view of the K copies of the copy-0 tensor ``t``."""
        off = t.data_ptr() - self.base
        es = t.element_size()
        if not self.contains(t.data_ptr(), t.numel() * es) or off % es or self.stride % es:
            raise ValueError("tensor is not inside copy 0 of the group region")
        flat = self.slab.view(t.dtype)
        return flat.as_strided((self.k,) + tuple(t.shape), (self.stride // es,) + tuple(t.stride()), off // es)

    # ------------------------------------------------------------------ validation
    def validate_program(self, prog) -> int:
        """Raise unless every pointer of ``prog``'s plan points into copy 0.  Returns the number
        of pointers checked."""
        plan = prog.plan
        bad: List[str] = []
        n = 0

        def chk(where, p):
            nonlocal n
            if p:
                n += 1
                if not self.contains(p):
                    bad.append(f"{where}=0x{p:x}")

        for i in range(plan.size()):
            kind = plan.kind(i)
            if kind == nat.OP_ALLREDUCE:
                raise RuntimeError("a grouped program cannot hold collectives")
            desc = plan.describe(i)
            cls = _PAYLOAD.get(kind)
            if cls is not None:
                obj = cls.from_buffer_copy(plan.payload(i))
                for name, p in _struct_ptrs(obj):
                    chk(f"op{i}:{desc}.{name}", p)
            for slot in range(8):
                chk(f"op{i}:{desc}.p[{slot}]", plan.get_ptr(i, slot))
            tab = _TABLES.get(kind)
            if tab is not None:
                pslot, islot, etype = tab
                ptr, cnt = plan.get_ptr(i, pslot), plan.get_int(i, islot)
                if ptr and cnt > 0:
                    raw = torch.empty(cnt * C.sizeof(etype), dtype=torch.uint8)
                    src = self.slab[ptr - self.base: ptr - self.base + raw.numel()]
                    raw.copy_(src)
                    arr = (etype * cnt).from_buffer_copy(bytes(raw.numpy()))
                    for j, e in enumerate(arr):
                        for name, p in _struct_ptrs(e):
                            chk(f"op{i}:{desc}[{j}].{name}", p)
        if prog._cast_all_plan is not None:
            cp = prog._cast_all_plan
            for slot in range(2):
                chk(f"cast_all.p[{slot}]", cp.get_ptr(0, slot))
        if bad:
            raise RuntimeError(f"grouped program has {len(bad)} pointer(s) outside its region copy 0: "
                               + ", ".join(bad[:12]))
        return n

    def close(self):
        """Stop allocating into this region (its memory stays reserved, see _KEEP_ALIVE)."""
        self.ext.region_forget(self.base)
