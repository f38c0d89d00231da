"""roctx host ranges for rocprofv3 timelines (SURVEY.md §5 "Tracing / profiling").

The reference's only instrumentation is the wall-clock ``Timer`` (``dist_model_tf_vgg.py:19-32``,
kept as :class:`idc_models_amd.utils.timer.Timer`).  Here the training step additionally pushes
named roctx ranges — ``step``, ``seg:fwd``, ``seg:bwd``, ``seg:opt``, ``allreduce:bucket<i>`` — so
``rocprofv3 --marker-trace --kernel-trace`` shows which kernels and collectives belong to which
phase.  Ranges are host-side and cost ~1 us each, so they are OFF unless ``IDC_ROCTX=1``; with
the switch off :func:`range` is a no-op context manager and nothing is loaded.

    IDC_ROCTX=1 rocprofv3 --marker-trace --kernel-trace -d out -- python bench.py --steps 5
"""
import contextlib
import ctypes
import os
from typing import Optional

_LIBS = ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4", "libroctx64.so")
_lib: Optional[ctypes.CDLL] = None
_tried = False


def enabled() -> bool:
    return os.environ.get("IDC_ROCTX", "0") == "1"


def _load() -> Optional[ctypes.CDLL]:
    global _lib, _tried
    if _tried:
        return _lib
    _tried = True
    for name in _LIBS:
        for path in (name, os.path.join("/opt/rocm/lib", name)):
            try:
                lib = ctypes.CDLL(path)
            except OSError:
                continue
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.argtypes = []
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            lib.roctxMarkA.restype = None
            _lib = lib
            return _lib
    return None


def push(name: str) -> None:
    lib = _load() if enabled() else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())


def pop() -> None:
    lib = _load() if enabled() else None
    if lib is not None:
        lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _load() if enabled() else None
    if lib is not None:
        lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    """``with trace.range("seg:bwd"): ...`` — a roctx range when IDC_ROCTX=1, else nothing."""
    if not enabled():
        yield
        return
    push(name)
    try:
        yield
    finally:
        pop()
