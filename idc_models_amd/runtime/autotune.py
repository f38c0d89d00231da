"""Plan-build-time autotuning of conv tile shapes and wgrad split factors.

The conv GEMMs of these CNNs are skinny and irregular (N = 32..512, K = 27..4608, M = 256..640k;
SURVEY §2.4), so no single tile wins: each conv / wgrad op of a freshly built plan is timed on
its real shape with every applicable tile (or split factor) and the fastest is written back into
the op before the plan is captured into a HIP graph.  Results are cached per shape signature for
the process (and optionally persisted as JSON via IDC_TUNE_CACHE).

Side effects of the trial launches only touch buffers that every step re-initialises (the
statistics arena and the gradient arena are memset at the start of their segments; activations
are overwritten), so tuning is safe before the first real step.
"""
from __future__ import annotations

import json
import os
import threading
from typing import Dict, Tuple

import torch

from ..ops import _native as nat

_CACHE: Dict[Tuple, int] = {}
_LOADED = False
# one tuning at a time per process (concurrent federated clients build their programs on worker
# threads): trial timings taken beside another plan's trials would be picked under contention, and
# the cache dict must not change size while it is being serialised
_LOCK = threading.RLock()


def _load_cache():
    global _LOADED
    if _LOADED:
        return
    _LOADED = True
    p = os.environ.get("IDC_TUNE_CACHE")
    if p and os.path.exists(p):
        try:
            with open(p) as f:
                entries = json.load(f)
            for k, v in entries.items():
                _CACHE[tuple(json.loads(k))] = v
        except (OSError, ValueError) as e:  # a torn or foreign file: retune rather than fail
            print(f"[autotune] ignoring unreadable tune cache {p}: {e}")


def _save_cache():
    """Persist the cache (IDC_TUNE_CACHE): rank 0 only, written to a temporary file and renamed
    into place so concurrent readers never see a partial file."""
    p = os.environ.get("IDC_TUNE_CACHE")
    if not p or int(os.environ.get("RANK", "0")) != 0:
        return
    tmp = f"{p}.tmp{os.getpid()}"
    with _LOCK:
        snap = dict(_CACHE)
    with open(tmp, "w") as f:
        json.dump({json.dumps(list(k)): v for k, v in snap.items()}, f)
    os.replace(tmp, p)


def _time_op(plan, i, stream, reps=4) -> float:
    sh = stream.cuda_stream
    plan.run(i, i + 1, sh)  # warm-up
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        e0.record()
        for _ in range(reps):
            plan.run(i, i + 1, sh)
        e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def _conv_candidates(ext, M: int, cout: int, payload: bytes = None, a_f32: int = 0):
    ntile = ext.num_tiles()
    cap = 32 if cout <= 32 else (64 if cout <= 64 else 128)
    out = []
    no32 = os.environ.get("IDC_NO_TILE32", "0") == "1"
    for t in range(ntile):
        bm, bn = ext.tile_bm(t), ext.tile_bn(t)
        if bm < 64 and no32:
            continue
        if bn > cap:
            continue
        if bm > 64 and M <= 2 * 64:
            continue
        out.append(t)
    # the image-resident 3x3 kernel (conv_img.hip: DenseNet's 128 -> 32 / 32 -> 128 convs on small
    # maps), one workgroup per image
    if payload is not None and os.environ.get("IDC_CONV_IMG", "1") != "0" and hasattr(ext, "img_ok") \
            and ext.img_ok(payload, a_f32):
        out.append(ext.TILE_IMG)
    # the image-resident stem conv (conv_stem.hip: 8-channel staged images)
    if payload is not None and os.environ.get("IDC_CONV_STEM", "1") != "0" and hasattr(ext, "stem_ok") \
            and ext.stem_ok(payload, a_f32):
        out.append(ext.TILE_STEM)
    # 256 x {128, 256} global_load_lds tiles for plain wide layers (conv_big.hip), when they
    # still make >= 128 workgroups
    if payload is not None and os.environ.get("IDC_CONV_BIG", "1") != "0" and ext.big_ok(payload, a_f32):
        # (BIG64: 4 waves of 64 x 64, the 64-channel layers -- VGG16's 50x50 dgrads)
        for t, bn in ((ext.TILE_BIG64, 64), (ext.TILE_BIG128, 128), (ext.TILE_BIG128D, 128), (ext.TILE_BIG256, 256)):
            if cout >= bn and -(-M // 256) * -(-cout // bn) >= 8:
                out.append(t)
    return out


def _tile_shape(ext, t: int):
    """(BM, BN, BK) of conv tile ``t``; None for a tile id outside the tables."""
    if t == ext.TILE_BIG64:
        return 256, 64, 64
    if t in (ext.TILE_BIG128, ext.TILE_BIG128D):
        return 256, 128, 64
    if t == ext.TILE_BIG256:
        return 256, 256, 64
    if t >= ext.num_tiles():
        return None
    return ext.tile_bm(t), ext.tile_bn(t), ext.tile_bk(t)


def _splits_for(ext, a, t: int, M: int, slab_floats: int):
    """Feasible split-K factors for conv tile ``t``: the partial slabs must fit the workspace, each
    slice must keep >= 2 K-steps, and only grids that leave the GPU under-filled are split."""
    shape = _tile_shape(ext, t)
    if shape is None or t == ext.TILE_BIG64:  # (BIG64 split-K: no exactness test, not offered)
        return []
    bm, bn, bk = shape
    tiles = -(-M // bm) * -(-a.Cout // bn)
    if tiles >= int(os.environ.get("IDC_SPLITK_MAX_TILES", "256")):
        return []
    K = a.KH * a.KW * a.Cin
    nk = -(-K // bk)
    if bm == 256:  # conv_big.hip: one workgroup per CU, so the split grid must fit 256 CUs
        return [s for s in (2, 3, 4, 6, 8) if tiles * s <= 256 and tiles * s * bm * bn <= slab_floats
                and nk >= 4 * s]
    return [s for s in (2, 4, 8) if tiles * s * bm * bn <= slab_floats and nk >= 2 * s]


def _autotune_plan_unlocked(plan, stream, verbose: bool = False, reset_tickets=None, slab_floats: int = 0) -> int:
    """Tune every conv / wgrad op of ``plan`` in place: tile shape, then the split-K factor of the
    best few tiles (ops whose payload carries a split-K workspace).  Returns the number tuned."""
    _load_cache()
    ext = nat.load()
    n = 0
    for i in range(plan.size()):
        kind = plan.kind(i)
        if kind == nat.OP_CONV:
            a = nat.ConvArgs.from_buffer_copy(plan.payload(i))
            f32 = plan.get_int(i, 1)
            M = a.N * a.Ho * a.Wo
            pro = 2 if a.bpro.mode != 0 else int(a.pro.mode != 0 or a.pro.act != 0)
            key = ("conv", M, a.Cout, a.Cin, a.KH, a.KW, a.SH, a.PT, a.ldx, f32, pro, a.epi_mode,
                   a.out_mode, int(bool(a.bias)), a.H, a.W)
            best = _CACHE.get(key)
            if best is None:
                times = {}
                plan.set_int(i, 2, 1)
                for t in _conv_candidates(ext, M, a.Cout, plan.payload(i), f32) or [ext.pick_tile(M, a.Cout)]:
                    plan.set_int(i, 0, t)
                    times[(t, 1)] = _time_op(plan, i, stream)
                if a.slab and a.tickets and reset_tickets is not None and \
                        os.environ.get("IDC_SPLITK", "1") != "0":
                    top = sorted((v, t) for (t, s), v in times.items() if _tile_shape(ext, t))[:3]
                    # the 256-row tiles are under-filled exactly where split-K pays: always try them
                    top += [(v, t) for (t, s), v in times.items()
                            if _tile_shape(ext, t) and _tile_shape(ext, t)[0] == 256 and (v, t) not in top]
                    for _, t in top:
                        for s in _splits_for(ext, a, t, M, slab_floats):
                            plan.set_int(i, 0, t)
                            plan.set_int(i, 2, s)
                            reset_tickets()
                            times[(t, s)] = _time_op(plan, i, stream)
                best = min(times, key=times.get)
                _CACHE[key] = best
                if verbose:
                    print("tune conv", key, {f"{k[0]}/{k[1]}": round(v * 1e3, 1) for k, v in times.items()},
                          "->", best)
            if isinstance(best, list):  # JSON round trip
                best = tuple(best)
            if not isinstance(best, tuple):
                best = (best, 1)
            plan.set_int(i, 0, best[0])
            plan.set_int(i, 2, best[1] if (a.slab and a.tickets) else 1)
            n += 1
        elif kind == nat.OP_WGRAD:
            a = nat.WgradArgs.from_buffer_copy(plan.payload(i))
            f32 = plan.get_int(i, 1)
            s0 = max(plan.get_int(i, 0), 1)
            M = a.N * a.Ho * a.Wo
            key = ("wgrad2", M, a.Cout, a.Cin, a.KH, a.KW, a.SH, f32, int(a.pro.mode != 0 or a.pro.act != 0),
                   int(a.gpro.mode != 0))
            best = _CACHE.get(key)
            if best is None:
                cands = sorted({max(1, s0 // 4), max(1, s0 // 2), s0, s0 * 2, s0 * 4})
                cands = [s for s in cands if (M + s - 1) // s >= 32] or [1]
                times = {}
                plan.set_int(i, 2, 0)
                for s in cands:
                    plan.set_int(i, 0, s)
                    times[(0, s)] = _time_op(plan, i, stream)
                # the large-tile LDS-DMA kernels (wgrad_big.hip) where they apply
                if hasattr(ext, "wgrad_big_ok") and os.environ.get("IDC_WG_TILES", "1") != "0":
                    K = a.KH * a.KW * a.Cin
                    for v in range(1, ext.wgrad_num_variants()):
                        if not ext.wgrad_big_ok(plan.payload(i), f32, v):
                            continue
                        sp = ext.wgrad_big_pick_splits(M, K, a.Cout, v)
                        for s in sorted({max(1, sp // 2), sp, sp * 2}):
                            plan.set_int(i, 0, s)
                            plan.set_int(i, 2, v)
                            times[(v, s)] = _time_op(plan, i, stream)
                    plan.set_int(i, 2, 0)
                # the isolated optimum: biasing wgrad splits either way (fewest / most slices
                # within 10-50% of it) measured 1-23% slower steps on DenseNet-121 and VGG16
                best = min(times, key=times.get)
                _CACHE[key] = best
                if verbose:
                    print("tune wgrad", key, {f"{k[0]}/{k[1]}": round(v * 1e3, 1) for k, v in times.items()},
                          "->", best)
            if isinstance(best, list):  # JSON round trip
                best = tuple(best)
            if not isinstance(best, tuple):  # caches written before the large-tile variants
                best = (0, best)
            plan.set_int(i, 0, best[1])
            plan.set_int(i, 2, best[0])
            n += 1
    _save_cache()
    torch.cuda.synchronize()
    return n


def autotune_plan(plan, stream, *args, **kwargs):
    """Tune every conv / wgrad op of ``plan`` (serialised per process, see ``_LOCK``)."""
    with _LOCK:
        return _autotune_plan_unlocked(plan, stream, *args, **kwargs)
