"""Loader for the native MI355X extension + ctypes mirrors of its argument structs.

The kernels take plain C structs (``csrc/kernels/*.h``).  Python fills the identical layout with
``ctypes`` and hands the raw bytes to the C++ plan (``csrc/runtime/plan.cpp``); sizes and a few
field offsets are verified against ``sizeof/offsetof`` reported by the extension at import time,
so a layout drift fails loudly instead of corrupting a launch.

On a machine with a GPU the extension MUST load (there is no silent eager fallback for the fused
runtime); on a CPU-only machine ``available()`` is False and only the reference path runs.
"""
from __future__ import annotations

import ctypes as C
import importlib
import os

import torch

_ext = None
_err = None

vp = C.c_void_p
ci = C.c_int
cf = C.c_float
cll = C.c_longlong


class BnArgs(C.Structure):
    _fields_ = [("stats", vp), ("gamma", vp), ("beta", vp), ("mmean", vp), ("mvar", vp),
                ("inv_count", cf), ("eps", cf), ("mode", ci), ("act", ci), ("C", ci), ("slots", ci),
                ("shift", vp)]


class BwdAff(C.Structure):
    """csrc/kernels/common.h BwdAff: a BatchNorm backward applied by the consumer while staging."""
    _fields_ = [("x", vp), ("ldx", ci), ("bn", BnArgs), ("gsum", vp), ("gsumx", vp),
                ("gsum_slots", ci), ("gsum_ld", ci), ("inv_n", cf), ("unit_alpha", ci), ("mode", ci),
                ("fold_C", ci), ("fgsum", vp), ("fgsumx", vp), ("fold_sum", vp), ("fold_sumx", vp)]


class ConvArgs(C.Structure):
    _fields_ = [("x", vp), ("N", ci), ("H", ci), ("W", ci), ("Cin", ci), ("ldx", ci),
                ("Ho", ci), ("Wo", ci), ("Cout", ci), ("y", vp), ("ldy", ci),
                ("w", vp), ("KH", ci), ("KW", ci), ("SH", ci), ("SW", ci), ("PT", ci), ("PL", ci),
                ("pro", BnArgs), ("epi_mode", ci), ("bias", vp), ("epi_act", ci), ("out_mode", ci),
                ("stats_out", vp), ("stats_ld", ci), ("stats_off", ci),
                ("mx", vp), ("ldmx", ci), ("mbn", BnArgs), ("gsum", vp), ("gsumx", vp),
                ("slab", vp), ("tickets", vp), ("slab_floats", cll), ("tickets_n", ci),
                ("ksplit", ci), ("stats_slots", ci), ("gsum_slots", ci), ("gsum_ld", ci),
                ("bpro", BwdAff), ("bepi", BwdAff), ("aout", vp), ("ldaout", ci), ("stats_shift", vp)]


class WgradArgs(C.Structure):
    _fields_ = [("x", vp), ("N", ci), ("H", ci), ("W", ci), ("Cin", ci), ("ldx", ci),
                ("g", vp), ("ldg", ci), ("Ho", ci), ("Wo", ci), ("Cout", ci),
                ("KH", ci), ("KW", ci), ("SH", ci), ("SW", ci), ("PT", ci), ("PL", ci),
                ("pro", BnArgs), ("dw", vp), ("scale", cf), ("cin_real", ci), ("pix_per_split", ci),
                ("gpro", BwdAff), ("part", vp), ("part_floats", cll)]


class BnBwdApplyArgs(C.Structure):
    _fields_ = [("dz", vp), ("lddz", ci), ("x", vp), ("ldx", ci), ("bn", BnArgs),
                ("gsum", vp), ("gsumx", vp), ("inv_n", cf), ("dst", vp), ("lddst", ci),
                ("dst_f32", ci), ("accumulate", ci), ("M", ci), ("C", ci), ("gsum_slots", ci),
                ("gsum_ld", ci), ("fold_sum", vp), ("fold_sumx", vp)]


class BnBwdReduceArgs(C.Structure):
    _fields_ = [("dy", vp), ("lddy", ci), ("dy_f32", ci), ("x", vp), ("ldx", ci), ("bn", BnArgs),
                ("dz", vp), ("lddz", ci), ("gsum", vp), ("gsumx", vp), ("M", ci), ("C", ci),
                ("gsum_slots", ci), ("gsum_ld", ci), ("dz_f32", ci)]


class PoolArgs(C.Structure):
    _fields_ = [("x", vp), ("ldx", ci), ("N", ci), ("H", ci), ("W", ci), ("C", ci),
                ("pro", BnArgs), ("k", ci), ("s", ci), ("pt", ci), ("pl", ci), ("Ho", ci),
                ("Wo", ci), ("y", vp), ("ldy", ci), ("argmax", vp), ("stats", vp),
                ("stats_ld", ci), ("stats_off", ci), ("stats_slots", ci), ("stats_shift", vp)]


class PoolBwdArgs(C.Structure):
    _fields_ = [("dy", vp), ("lddy", ci), ("dy_f32", ci), ("argmax", vp), ("N", ci), ("H", ci),
                ("W", ci), ("C", ci), ("k", ci), ("s", ci), ("pt", ci), ("pl", ci), ("Ho", ci),
                ("Wo", ci), ("x", vp), ("ldx", ci), ("bn", BnArgs), ("dx", vp), ("lddx", ci),
                ("gsum", vp), ("gsumx", vp), ("is_avg", ci), ("gsum_slots", ci), ("gsum_ld", ci),
                ("dyaff", BwdAff), ("dx_f32", ci)]


class BnMovingDesc(C.Structure):
    _fields_ = [("stats", vp), ("C", ci), ("inv_count", cf), ("unbias", cf), ("mmean", vp),
                ("mvar", vp), ("momentum", cf), ("ld", ci), ("slots", ci), ("shift", vp)]


class ShiftDesc(C.Structure):
    _fields_ = [("stats", vp), ("shift", vp), ("ld", ci), ("slots", ci), ("inv_count", cf), ("pad", ci)]


class HeadArgs(C.Structure):
    _fields_ = [("x", vp), ("ldx", ci), ("N", ci), ("HW", ci), ("C", ci), ("U", ci),
                ("pro", BnArgs), ("w", vp), ("b", vp), ("labels", vp), ("logits", vp),
                ("feats", vp), ("dlogits", vp), ("loss", vp), ("loss_scale", cf), ("training", ci),
                ("loss_vec", vp), ("ticket", vp), ("dl_scale", cf)]


class HeadBwdArgs(C.Structure):
    _fields_ = [("feats", vp), ("dlogits", vp), ("w", vp), ("N", ci), ("HW", ci), ("C", ci),
                ("U", ci), ("dw", vp), ("db", vp), ("dA", vp), ("ldda", ci), ("det", ci)]


class CastEntry(C.Structure):
    _fields_ = [("src", vp), ("fwd", vp), ("dgrad", vp), ("KH", ci), ("KW", ci), ("Cin", ci),
                ("Cout", ci), ("Cpad", ci), ("dw", ci), ("begin", cll)]


class DwArgs(C.Structure):
    _fields_ = [("x", vp), ("ldx", ci), ("N", ci), ("H", ci), ("W", ci), ("C", ci),
                ("pro", BnArgs), ("w", vp), ("KH", ci), ("KW", ci), ("S", ci), ("PT", ci),
                ("PL", ci), ("Ho", ci), ("Wo", ci), ("y", vp), ("ldy", ci), ("stats", vp),
                ("stats_ld", ci), ("dy", vp), ("lddy", ci), ("dx", vp), ("lddx", ci),
                ("gsum", vp), ("gsumx", vp), ("dw", vp), ("ws", vp), ("stats_slots", ci),
                ("gsum_slots", ci), ("gsum_ld", ci), ("dyaff", BwdAff), ("stats_shift", vp)]


class Mlp2Args(C.Structure):
    _fields_ = [("x", vp), ("N", ci), ("D0", ci), ("D1", ci), ("U", ci), ("w1", vp), ("b1", vp),
                ("w2", vp), ("b2", vp), ("p0", cf), ("p1", cf), ("seed", C.c_uint64), ("step", vp),
                ("labels", vp), ("logits", vp), ("h1", vp), ("loss", vp), ("dlogits", vp),
                ("loss_scale", cf), ("training", ci), ("dw1", vp), ("db1", vp), ("dw2", vp),
                ("db2", vp), ("dx", vp), ("dl_scale", cf)]


class WgBatchEntry(C.Structure):
    """One member of a batched weight-gradient launch (conv_wgrad.h)."""
    _fields_ = [("a", WgradArgs), ("gx", ci), ("gy", ci), ("gz", ci), ("ipw", ci)]


class DenseLayerDesc(C.Structure):
    """One dense layer of a persistent dense-stage launch (dense_stage.h)."""
    _fields_ = [("w1", vp), ("w2", vp), ("g1", vp), ("b1", vp), ("g2", vp), ("b2", vp), ("t", vp),
                ("tstats", vp), ("tshift", vp), ("eps1", cf), ("eps2", cf), ("cin", ci), ("pad_", ci),
                ("mm1", vp), ("mv1", vp), ("mm2", vp), ("mv2", vp)]


class DenseStageArgs(C.Structure):
    _fields_ = [("buf", vp), ("sstats", vp), ("sshift", vp), ("layers", vp), ("sync", vp), ("err", vp),
                ("scratch", vp), ("stamps", vp),
                ("N", ci), ("H", ci), ("W", ci), ("ld", ci), ("nlayers", ci), ("k2", ci),
                ("act1", ci), ("act2", ci), ("inv_count", cf), ("max_polls", C.c_uint), ("lookahead", ci),
                ("infer", ci), ("stepflag", vp), ("hostflag", vp), ("partials", vp), ("ksplit", ci),
                ("rows", ci), ("rows_ipg", ci)]


class DenseBwdLayerDesc(C.Structure):
    """One dense layer of a persistent dense-stage backward launch (dense_stage.h)."""
    _fields_ = [(n, vp) for n in ("w1d", "w2d", "g1", "b1", "g2", "b2", "t", "tstats", "tshift", "dO16", "dt",
                                  "dbeta1", "dgamma1", "dbeta2", "dgamma2", "r1", "r2")] + \
               [("eps1", cf), ("eps2", cf), ("cin", ci), ("pad_", ci)]


class DenseBwdPhase(C.Structure):
    _fields_ = [("first", ci), ("kind", ci), ("layer", ci), ("tiles", ci)]


class DenseBwdArgs(C.Structure):
    _fields_ = [(n, vp) for n in ("buf", "sstats", "sshift", "dbuf", "dnew", "dx16", "z2")] + \
               [("pend", BwdAff)] + \
               [(n, vp) for n in ("layers", "phases", "sync", "btot", "err", "stamps")] + \
               [(n, ci) for n in ("N", "H", "W", "ld", "c0", "nlayers", "k2", "act", "nphases", "ntickets")] + \
               [("inv_count", cf), ("max_polls", C.c_uint), ("stepflag", vp), ("hostflag", vp),
                ("rows", ci), ("rows_ipg", ci), ("rpart", vp), ("rpart_floats", C.c_longlong)]


class MbPhaseDesc(C.Structure):
    """One phase of a persistent MobileNetV2 block-chain launch (csrc/kernels/mb_chain.h)."""
    _fields_ = [(n, ci) for n in ("kind", "first", "tiles", "dep", "pro", "act_in", "tab_in", "tab_out",
                                  "N", "H", "W", "Ho", "Wo", "S", "PT", "PL", "Cin", "Cout", "tm", "tn",
                                  "slots", "bn_mode", "ldx", "ldy")] + \
               [(n, vp) for n in ("x", "res", "aout", "w16", "w32", "y", "stats", "shift", "slotbuf",
                                  "gamma", "beta", "mmean", "mvar")] + \
               [("eps", cf), ("inv_count", cf), ("pre", BnArgs)]


class MbChainArgs(C.Structure):
    _fields_ = [(n, vp) for n in ("phases", "sync", "tabs", "err", "stepflag", "hostflag", "stamps")] + \
               [("nphases", ci), ("ntickets", ci), ("max_polls", C.c_uint), ("pad_", ci)]


MB_TAB, MB_PW, MB_DW = 1, 2, 3


class MbInferArgs(C.Structure):
    """One MobileNetV2 block in inference mode, one launch (csrc/kernels/mb_infer.h)."""
    _fields_ = [("x", vp), ("ldx", ci), ("ldres", ci), ("xbn", BnArgs), ("res", vp), ("we", vp), ("ebn", BnArgs),
                ("wd", vp), ("dbn", BnArgs), ("wp", vp), ("pbn", BnArgs), ("y", vp), ("ldy", ci)] + \
               [(n, ci) for n in ("N", "H", "W", "Cin", "Cexp", "Cout", "Ho", "Wo", "S", "PT", "PL",
                                  "residual", "ipg", "cs")] + \
               [("slab", vp), ("tickets", vp)]


class DenseInferArgs(C.Structure):
    """A whole dense block in inference mode, one launch (csrc/kernels/dense_stage.h)."""
    _fields_ = [("buf", vp), ("ld", ci)] + [(n, ci) for n in ("N", "H", "W", "c0", "L", "ipg", "act")] + \
               [("layers", vp)]


def mb_infer_default_cs(cexp: int, groups: int, expand: bool = True) -> int:
    """Expanded channels per workgroup of an mb_infer launch (csrc/kernels/mb_infer.h): enough
    slices per image group that the launch has >= 256 workgroups, in multiples of 32."""
    full = -(-cexp // 32) * 32
    if not expand:
        return full
    want = max(1, -(-256 // max(groups, 1)))
    return min(full, max(32, -(-(-(-cexp // want)) // 32) * 32))

_STRUCTS = {"BnArgs": BnArgs, "BwdAff": BwdAff, "ConvArgs": ConvArgs, "WgradArgs": WgradArgs,
            "WgBatchEntry": WgBatchEntry,
            "BnBwdApplyArgs": BnBwdApplyArgs, "BnBwdReduceArgs": BnBwdReduceArgs,
            "PoolArgs": PoolArgs, "PoolBwdArgs": PoolBwdArgs, "BnMovingDesc": BnMovingDesc,
            "HeadArgs": HeadArgs, "HeadBwdArgs": HeadBwdArgs, "CastEntry": CastEntry,
            "DwArgs": DwArgs, "Mlp2Args": Mlp2Args, "ShiftDesc": ShiftDesc,
            "DenseStageArgs": DenseStageArgs, "DenseLayerDesc": DenseLayerDesc,
            "DenseBwdArgs": DenseBwdArgs, "DenseBwdLayerDesc": DenseBwdLayerDesc, "DenseBwdPhase": DenseBwdPhase,
            "MbPhaseDesc": MbPhaseDesc, "MbChainArgs": MbChainArgs, "MbInferArgs": MbInferArgs,
            "DenseInferArgs": DenseInferArgs}

# op kinds (csrc/runtime/plan.cpp)
OP_CONV, OP_WGRAD, OP_BN_BWD_APPLY, OP_BN_BWD_REDUCE, OP_MAXPOOL, OP_AVGPOOL, OP_POOL_BWD = range(7)
OP_BN_MOVING, OP_HEAD_FWD, OP_HEAD_BWD, OP_RMSPROP, OP_CAST, OP_INPUT, OP_MEMSET = range(7, 14)
OP_BN_STATS, OP_BN_APPLY, OP_DW_FWD, OP_DW_BWD_DATA, OP_DW_WGRAD, OP_COPY, OP_FINITE_CHECK = range(14, 21)
OP_MLP_FWD, OP_MLP_BWD, OP_MLP_STEP, OP_COLLAPSE, OP_STATS_SHIFT, OP_ALLREDUCE, OP_WGRAD_BATCH = range(21, 28)
OP_DENSE_STAGE = 28
OP_DENSE_STAGE_BWD = 29
OP_MB_CHAIN = 30
OP_MB_INFER = 31
OP_DENSE_INFER = 32

ACT = {None: 0, "none": 0, "linear": 0, "relu": 1, "relu6": 2}
OUT_BF16, OUT_F32, OUT_F32_ACC = 0, 1, 2


def _verify(ext):
    if ext.OP_ALLREDUCE != OP_ALLREDUCE:
        raise RuntimeError("native op-kind table drifted (OP_ALLREDUCE)")
    if ext.OP_DENSE_STAGE != OP_DENSE_STAGE or ext.OP_MB_CHAIN != OP_MB_CHAIN or ext.OP_MB_INFER != OP_MB_INFER \
            or ext.OP_DENSE_INFER != OP_DENSE_INFER:
        raise RuntimeError("native op-kind table drifted (OP_DENSE_STAGE / OP_MB_CHAIN)")
    sizes = ext.struct_sizes()
    for name, cls in _STRUCTS.items():
        if C.sizeof(cls) != sizes[name]:
            raise RuntimeError(f"native struct {name}: ctypes {C.sizeof(cls)} != C++ {sizes[name]}")
    checks = {"ConvArgs.mbn": ConvArgs.mbn.offset, "ConvArgs.gsumx": ConvArgs.gsumx.offset,
              "ConvArgs.ksplit": ConvArgs.ksplit.offset,
              "WgradArgs.pix_per_split": WgradArgs.pix_per_split.offset,
              "HeadArgs.training": HeadArgs.training.offset,
              "PoolBwdArgs.is_avg": PoolBwdArgs.is_avg.offset,
              "ConvArgs.gsum_ld": ConvArgs.gsum_ld.offset, "BnArgs.slots": BnArgs.slots.offset,
              "DwArgs.gsum_ld": DwArgs.gsum_ld.offset, "ConvArgs.bepi": ConvArgs.bepi.offset,
              "WgradArgs.gpro": WgradArgs.gpro.offset, "PoolBwdArgs.dx_f32": PoolBwdArgs.dx_f32.offset,
              "BwdAff.fold_sumx": BwdAff.fold_sumx.offset, "ConvArgs.aout": ConvArgs.aout.offset,
              "WgradArgs.part_floats": WgradArgs.part_floats.offset, "HeadBwdArgs.det": HeadBwdArgs.det.offset,
              "DwArgs.dyaff": DwArgs.dyaff.offset, "BnArgs.shift": BnArgs.shift.offset,
              "ConvArgs.stats_shift": ConvArgs.stats_shift.offset,
              "PoolArgs.stats_shift": PoolArgs.stats_shift.offset,
              "DwArgs.stats_shift": DwArgs.stats_shift.offset,
              "BnMovingDesc.shift": BnMovingDesc.shift.offset, "MbPhaseDesc.pre": MbPhaseDesc.pre.offset}
    for k, v in checks.items():
        if sizes[k] != v:
            raise RuntimeError(f"native struct field {k}: ctypes offset {v} != C++ {sizes[k]}")


def load(build_if_missing: bool = True):
    """Import the extension (building it first if the .so is absent and hipcc exists)."""
    global _ext, _err
    if _ext is not None:
        return _ext
    try:
        _ext = importlib.import_module("idc_models_amd._idc_native")
    except ImportError as e:  # pragma: no cover - exercised on fresh checkouts
        _err = e
        if build_if_missing and os.path.exists("/opt/rocm/bin/hipcc"):
            import sys
            root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
            sys.path.insert(0, root)
            from tools.build_native import build
            build(verbose=False)
            _ext = importlib.import_module("idc_models_amd._idc_native")
        else:
            raise
    _verify(_ext)
    return _ext


def available() -> bool:
    try:
        load(build_if_missing=False)
        return True
    except Exception:
        return False


def require():
    """The GPU path must run native code: raise loudly if it cannot."""
    try:
        return load()
    except Exception as e:
        raise RuntimeError("idc_models_amd native extension (gfx950 HIP kernels) is not available; "
                           "run `python tools/build_native.py`") from e


def ptr(t) -> int:
    if t is None:
        return 0
    if isinstance(t, int):
        return t
    return t.data_ptr()


def stream_handle(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def raw(struct) -> bytes:
    return C.string_at(C.addressof(struct), C.sizeof(struct))


def bn_args(stats=None, gamma=None, beta=None, mmean=None, mvar=None, count=1, eps=1e-3,
            mode=0, act=0, C_=0, slots=1, shift=None) -> BnArgs:
    b = BnArgs()
    b.stats, b.gamma, b.beta = ptr(stats), ptr(gamma), ptr(beta)
    b.shift = ptr(shift)
    b.mmean, b.mvar = ptr(mmean), ptr(mvar)
    b.inv_count = 1.0 / float(max(count, 1))
    b.eps = float(eps)
    b.mode = int(mode)
    b.act = int(act)
    b.C = int(C_)
    b.slots = int(slots)
    return b
