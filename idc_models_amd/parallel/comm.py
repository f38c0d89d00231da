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
