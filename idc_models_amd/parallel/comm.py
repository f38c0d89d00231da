"""Process-group bootstrap and collective helpers (RCCL over xGMI on MI355X, gloo on CPU).

One process per GPU (``torchrun --nproc-per-node N`` or ``launch.spawn``); the ``nccl`` backend of
``torch.distributed`` *is* RCCL on ROCm.  Rendezvous is ``env://`` (TCPStore on MASTER_ADDR,
which must be 127.0.0.1 on this pool).  ``HSA_ENABLE_IPC_MODE_LEGACY=0`` is required for RCCL's
dmabuf IPC and is set here if the caller did not.
"""
from __future__ import annotations

import datetime
import os
from typing import List, Optional

import torch
import torch.distributed as dist


def env_world() -> tuple:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0"))))


_FORCED = False  # collectives run even in a world of one (tests / benches of the comm path)


def init_process_group(backend: Optional[str] = None, timeout_s: int = 600, force: bool = False) -> tuple:
    """Initialise the default group from the environment; returns (rank, world, local_rank).

    ``force``: create the group (and run every collective helper below for real) even when the
    world has one rank, so the RCCL path can be exercised on a one-GPU machine."""
    global _FORCED
    rank, world, local = env_world()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if force and world == 1:
        _FORCED = True
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29512")
        os.environ.setdefault("RANK", str(rank))  # a forced world of one has no launcher env
        os.environ.setdefault("WORLD_SIZE", str(world))
        os.environ.setdefault("LOCAL_RANK", str(local))
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return rank, world, local


def is_dist() -> bool:
    """True when collectives must run: a process group of more than one rank, or a forced one."""
    return dist.is_available() and dist.is_initialized() and (dist.get_world_size() > 1 or _FORCED)


def backend() -> Optional[str]:
    return dist.get_backend() if dist.is_available() and dist.is_initialized() else None


def destroy():
    global _FORCED
    destroy_native_ring()
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _FORCED = False


def world_size() -> int:
    return dist.get_world_size() if is_dist() else 1


def rank() -> int:
    return dist.get_rank() if is_dist() else 0


def barrier():
    if is_dist():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_reduce_(t: torch.Tensor, op=dist.ReduceOp.SUM, async_op=False):
    if not is_dist():
        return None
    return dist.all_reduce(t, op=op, async_op=async_op)


def broadcast_(t: torch.Tensor, src: int = 0):
    if is_dist():
        dist.broadcast(t, src)


def all_reduce_max(value: float, device) -> float:
    t = torch.tensor([value], dtype=torch.float64, device=device)
    all_reduce_(t, dist.ReduceOp.MAX)
    return float(t.item())


def _native_ring(device):
    """The rank's native RCCL communicator (``native_comm.shared_communicator``: the one the
    strategy's gradient buckets use, with its init timeout and watchdog), or None when the group is
    not RCCL or native collectives are off (IDC_NATIVE_COMM=0)."""
    if backend() != "nccl" or os.environ.get("IDC_NATIVE_COMM", "1") == "0":
        return None
    from .native_comm import shared_communicator
    return shared_communicator(dist.get_rank(), dist.get_world_size(), device)


def ring_sum_u32_(t: torch.Tensor) -> torch.Tensor:
    """In-place SUM over the ranks modulo 2^32 of an int32 tensor that holds uint32 bit patterns
    (the masked fixed-point vectors of secure aggregation, fed/secagg.py).  On RCCL: ONE native
    ``ncclUint32`` all-reduce (unsigned wrap is defined; a signed int32 sum that wraps is not) on
    the communicator's own stream behind a watchdog progress mark, and the caller's stream is
    released only when it completed -- a dead peer raises ``CommFailure`` after the watchdog
    timeout instead of hanging the secure round; on gloo (or with native collectives off): an
    exact int64 sum of the unsigned values, reduced mod 2^32."""
    if not is_dist():
        return t
    if t.dtype != torch.int32:
        raise TypeError("ring_sum_u32_: int32 bit patterns expected")
    nc = _native_ring(t.device) if t.is_cuda else None
    if nc is not None:
        nc.check()
        cur = torch.cuda.current_stream(t.device)
        cs = torch.cuda.ExternalStream(nc.stream_handle, device=t.device)
        cs.wait_stream(cur)
        nc.all_reduce_u32_(t, stream=cs)
        nc.step_issued()
        done = torch.cuda.Event()
        done.record(cs)
        if nc.watchdog is not None:
            from .watchdog import wait_with_watchdog
            wait_with_watchdog(nc.watchdog, done.query)
        cur.wait_event(done)
        return t
    wide = t.to(torch.int64) & 0xFFFFFFFF
    dist.all_reduce(wide)  # < world * 2^32: exact in int64
    wide &= 0xFFFFFFFF
    t.copy_(torch.where(wide >= (1 << 31), wide - (1 << 32), wide).to(torch.int32))
    return t


def destroy_native_ring():
    """Close the rank's shared native communicator (end of the process group)."""
    from .native_comm import _SHARED, release_shared
    for nc in list(_SHARED.values()):
        release_shared(nc)


def all_reduce_packed_(tensors: List[torch.Tensor], op=dist.ReduceOp.SUM) -> List[torch.Tensor]:
    """In-place SUM over the ranks of many tensors: ONE packed all-reduce per dtype, each in its
    own dtype (float64 accumulators are never rounded through float32)."""
    if not is_dist() or not tensors:
        return tensors
    groups = {}
    for t in tensors:
        groups.setdefault(t.dtype, []).append(t)
    for dt, ts in groups.items():
        flat = torch.cat([t.reshape(-1) for t in ts])
        all_reduce_(flat, op)
        off = 0
        for t in ts:
            t.copy_(flat[off:off + t.numel()].view(t.shape))
            off += t.numel()
    return tensors


def pack_all_reduce(tensors: List[torch.Tensor], op=dist.ReduceOp.SUM) -> List[torch.Tensor]:
    """One packed all-reduce for many small tensors (metric accumulators, BN statistics)."""
    if not is_dist() or not tensors:
        return tensors
    flat = torch.cat([t.reshape(-1).double() for t in tensors])
    dist.all_reduce(flat, op=op)
    out, off = [], 0
    for t in tensors:
        n = t.numel()
        out.append(flat[off:off + n].view(t.shape).to(t.dtype))
        off += n
    return out
