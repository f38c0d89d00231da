"""Single-node multi-process launcher (one process per MI355X, or N gloo ranks on the CPU).

The reference drives all GPUs from one TF process (``MirroredStrategy``); here every GPU gets its
own process and RCCL connects them.  ``torchrun --nproc-per-node N --master-addr 127.0.0.1`` is the
production launcher; :func:`spawn` is the in-Python equivalent used by tests and notebooks: it
picks a free TCP port on 127.0.0.1, sets RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* per child, starts the
children with the ``spawn`` method (never fork after HIP initialisation) and re-raises the first
child failure in the parent.
"""
from __future__ import annotations

import os
import socket
import traceback
from typing import Any, Callable, Sequence

import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _child(rank: int, fn: Callable, world: int, port: int, backend: str, args: Sequence, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    try:
        from . import comm
        comm.init_process_group(backend)
        out = fn(rank, world, *args)
        q.put((rank, "ok", out))
    except BaseException:  # report, then fail the child
        q.put((rank, "err", traceback.format_exc()))
        raise
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def spawn(fn: Callable, world_size: int, args: Sequence = (), backend: str = "gloo",
          timeout_s: float = 600.0) -> list:
    """Run ``fn(rank, world, *args)`` in ``world_size`` processes; return per-rank results.

    ``fn`` must be importable (module level) and its return value picklable.
    """
    port = free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_child, args=(r, fn, world_size, port, backend, tuple(args), q))
             for r in range(world_size)]
    for p in procs:
        p.start()
    results: dict = {}
    err = None
    try:
        for _ in range(world_size):
            rank, status, payload = q.get(timeout=timeout_s)
            if status == "err":
                err = f"rank {rank} failed:\n{payload}"
                break
            results[rank] = payload
    finally:
        for p in procs:
            p.join(timeout=5 if err else timeout_s)
            if p.is_alive():
                p.terminate()
                p.join()
    if err:
        raise RuntimeError(err)
    return [results[r] for r in range(world_size)]
