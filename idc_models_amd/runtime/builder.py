"""Program builder: lowers a model into a static launch plan over preallocated device arenas.

Design (MI355X-first):

* shapes are static per (batch, training) — every buffer is allocated once, every kernel argument
  struct is built once, and the whole step is replayed as HIP graphs by the native ``Plan``;
* activations are NHWC bf16; "pending BN" — tensors are stored RAW (pre-BN) together with their
  per-channel [sum|sumsq] batch statistics produced in the producer's epilogue, and every consumer
  applies its own BN affine + activation while staging its operand (no BN/ReLU kernels);
* all batch statistics of a step live in ONE stats arena (one memset per step), all gradients in
  the flat fp32 gradient arena (one memset per step), all BN moving-average updates are ONE launch;
* bf16 weight copies in kernel layouts (forward ``[Cout][KH][KW][Cin]``, flipped dgrad
  ``[Cin][KH][KW][Cout]``) are produced from the fp32 Keras-layout masters by ONE cast launch
  after each optimizer step.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch

from ..ops import _native as nat

BF16 = torch.bfloat16
F32 = torch.float32


@dataclass
class Tensor4:
    """A (possibly channel-sliced) NHWC tensor view: base tensor + channel offset + pixel stride."""
    t: torch.Tensor
    N: int
    H: int
    W: int
    C: int          # channels of this view
    ld: int         # pixel stride (elements)
    coff: int = 0   # channel offset into base

    @property
    def ptr(self) -> int:
        return self.t.data_ptr() + self.coff * self.t.element_size()

    @property
    def M(self) -> int:
        return self.N * self.H * self.W

    @property
    def is_f32(self) -> bool:
        return self.t.dtype == F32

    def slice(self, c0: int, c: int) -> "Tensor4":
        return Tensor4(self.t, self.N, self.H, self.W, c, self.ld, self.coff + c0)


def stat_slots_for(rows: int) -> int:
    """Statistics slot copies for a reduction over ``rows`` rows (csrc/kernels/common.h,
    "Statistics slots"): global float atomics serialise per address at ~24 ns each, so producers
    with many row blocks spread their per-channel adds over copies that consumers sum.  About
    one copy per 4096 rows, at most IDC_STAT_SLOTS_CAP (default 4) copies: the consumers' batched
    table loads take <= 4 copies (common.h "Batched table inputs")."""
    cap = max(1, min(16, int(os.environ.get("IDC_STAT_SLOTS_CAP", "4"))))
    s = 1
    while s < cap and s * 4096 < rows:
        s *= 2
    return s


@dataclass
class Stats:
    """[sum | sumsq] statistics of a tensor: row length ``ld`` channels, ``count`` samples,
    ``slots`` copies of the [sum | sumsq] pair (stride 2*ld) that consumers add up."""
    t: torch.Tensor   # view into the stats arena, 2*ld*slots floats
    ld: int
    count: int
    slots: int = 1
    # per-channel shift K (persistent across steps, NOT in the zeroed arena): the producers
    # accumulate y - K, and K advances to the batch mean after every backward (common.h
    # "Shifted statistics")
    shift: Optional[torch.Tensor] = None

    def shift_ptr(self, off: int = 0) -> int:
        return self.shift.data_ptr() + 4 * off if self.shift is not None else 0

    @property
    def ptr(self):
        return self.t.data_ptr()


class BNRef:
    """A Keras BatchNormalization layer resolved for one program."""

    def __init__(self, layer, builder: "Builder", stats: Optional[Stats], act: int):
        self.layer = layer
        self.training = builder.training and layer.trainable
        self.mode = 1 if self.training else 2
        self.stats = stats
        self.act = act
        self.C = layer.channels
        self.b = builder
        arena = builder.arena
        self.gamma = layer.gamma
        self.beta = layer.beta
        self.trainable = builder.training and layer.trainable and layer.gamma.requires_grad
        self.dgamma = arena.grad_of(layer.gamma) if self.trainable else None
        self.dbeta = arena.grad_of(layer.beta) if self.trainable else None

    def args(self) -> nat.BnArgs:
        st = self.stats
        return nat.bn_args(stats=st.t if (st is not None and self.mode == 1) else None,
                           gamma=self.gamma, beta=self.beta,
                           mmean=self.layer.moving_mean, mvar=self.layer.moving_variance,
                           count=st.count if st is not None else 1, eps=self.layer.epsilon,
                           mode=self.mode, act=self.act, C_=st.ld if st is not None else self.C,
                           slots=st.slots if (st is not None and self.mode == 1) else 1,
                           shift=st.shift if (st is not None and self.mode == 1) else None)


def act_only(act: int) -> nat.BnArgs:
    return nat.bn_args(mode=0, act=act)


IDENT = None

# Persistent dense-stage launches switched off for the rest of the process (a launch gave up on a
# wait: see disable_persistent); checked by dense_stage_ok / dense_stage_bwd_ok
_PERSISTENT_OFF: List[str] = []


def disable_persistent(reason: str):
    """Build no more persistent dense-stage launches in this process (programs built from now on
    run the per-layer kernels).  Called by the runtime when a launch timed out (runtime/program.py
    FusedStep.check_persistent, fed/fedavg.py client batching)."""
    if not _PERSISTENT_OFF:
        import warnings
        warnings.warn(f"persistent dense-stage launches disabled: {reason}", RuntimeWarning, stacklevel=2)
    _PERSISTENT_OFF.append(reason)


def persistent_disabled() -> bool:
    return bool(_PERSISTENT_OFF)


def rows_bwd_enabled() -> bool:
    """The row-resident dense-stage backward (dense_rows_bwd.hip; IDC_DS_ROWS_BWD)."""
    return os.environ.get("IDC_DS_ROWS_BWD", "0") == "1"


_HOST_FLAGS = {"base": 0, "next": 0}
_HOST_FLAG_SLOTS = 4096


def _host_flag_slot() -> int:
    """Address of a fresh zeroed int in ONE process-lifetime slab of mapped pinned host memory
    (allocated once, never freed while kernels that hold slots may still be captured in graphs;
    a program whose slots run out shares the last one: the flag is only a trigger)."""
    if not _HOST_FLAGS["base"]:
        _HOST_FLAGS["base"] = int(nat.load().host_alloc(4 * _HOST_FLAG_SLOTS))
    i = min(_HOST_FLAGS["next"], _HOST_FLAG_SLOTS - 1)
    _HOST_FLAGS["next"] += 1
    return _HOST_FLAGS["base"] + 4 * i


class PersistentLaunchError(RuntimeError):
    """A persistent dense-stage launch gave up on a wait (IDC_DS_ON_FAIL=raise); the step it
    belonged to skipped its weight update."""


class Builder:
    def __init__(self, net, arena, device, batch: int, training: bool):
        self.net = net
        self.arena = arena
        self.device = device
        self.B = batch
        self.training = training
        self.ops: List[tuple] = []  # (segment, kind, payload bytes, ints, floats, longs, ptrs, lane)
        self.keep: List[torch.Tensor] = []  # keep allocations alive
        self._stats_chunks: List[Tuple[int, int]] = []
        self._stats_size = 0
        self.stats_arena: Optional[torch.Tensor] = None
        self.cast_all: List[nat.CastEntry] = []
        self.cast_trainable: List[nat.CastEntry] = []
        self.moving: List[nat.BnMovingDesc] = []
        self.conv_weights: Dict[int, dict] = {}
        self.segment = "fwd"
        self.side_lane = os.environ.get("IDC_SIDE_LANE", "1") != "0"
        self.guard = os.environ.get("IDC_GUARD") == "1"
        # statistics slots (stat_slots_for, default on; IDC_STAT_SLOTS=0: one copy everywhere).
        # Every workgroup of a large-map producer adds its per-channel sums into the same few
        # addresses, and float atomics on one address serialise at the memory side (a 676-tile
        # stage-1 concat-gradient dgrad: 28.3 us with one copy, 17.0 us with 4, conv phase micro,
        # round 5).  At most 4 copies (IDC_STAT_SLOTS_CAP): consumers then keep the one-round-trip
        # batched table loads (common.h "Batched table inputs").  bench.py A/B on one box, round 5:
        # DenseNet-121 3.53-3.55 ms/step with 4 copies vs 3.64-3.67 with one (2 copies 3.64-3.66,
        # 8 copies 3.65); MobileNetV2 2.26 vs 2.32; VGG16 2.40 either way.
        self.stat_slots_on = os.environ.get("IDC_STAT_SLOTS", "1") == "1"
        self.pending_sums: List["BNRef"] = []  # BatchNorms whose gradient slot copies await a fold
        # IDC_DETERMINISTIC=1: every float reduction has a fixed order (see _det_* below); the
        # same program on the same inputs then produces the same bits run after run
        self.det = os.environ.get("IDC_DETERMINISTIC", "0") == "1"
        self._post: List[tuple] = []  # collapse ops queued to follow the next emitted op
        self._wslab: Dict[int, torch.Tensor] = {}  # det wgrad partial slabs, one per lane
        self.guards: List[tuple] = []
        self.splitk_slab: Optional[torch.Tensor] = None
        self.tickets: List[torch.Tensor] = []
        self.bwd_marks: List[Tuple[int, int]] = []  # (op index, lowest arena param index ready)
        # stats arena is allocated lazily with a generous capacity; views are handed out in order
        # (the deterministic mode's per-workgroup private slots need ~10-40x more)
        # (only the used prefix is cleared each step, so the capacity itself costs nothing per step;
        # the persistent dense-stage launches keep their statistics slots here too)
        self._stats_cap = (1 << 25) if self.det else (1 << 23)
        self.stats_arena = torch.zeros(self._stats_cap, dtype=F32, device=device)
        self.all_stats: List[Stats] = []
        # shifted statistics (IDC_STATS_SHIFT=0: plain E[y^2] - E[y]^2, for comparisons)
        self.shift_stats = os.environ.get("IDC_STATS_SHIFT", "1") != "0"
        # batched weight gradients (conv_wgrad.h WgBatchEntry): side-lane wgrads a lowering marks
        # ``batch=True`` are collected and launched as ONE kernel per kernel shape at the next
        # flush_wgrad_batch (DenseNet: the end of a late stage's dense layers)
        self._wg_batch: List[tuple] = []
        self._wg_batch_marks: list = []
        # fail-safe of the persistent launches (csrc/kernels/persist.h note_fail): a per-step guard
        # word in the stats arena (zeroed by every training step's arena memset) that a give-up ORs
        # 2 into and the optimizer's skip test reads, and a pinned host word the runtime polls
        self.step_flag: Optional[torch.Tensor] = None
        self.host_flag: int = 0
        # another program may run concurrently on this device (concurrent federated clients): the
        # forward launch's lookahead queue order, which needs more than one phase of its own
        # workgroups resident, is not used
        self.shared_device = False
        # this rank's weight in an uneven split of a global batch (n_local * world / global): the
        # loss head's gradient seed carries it, so each rank's local gradient is weighted BEFORE
        # the all-reduce sum (lower_common.emit_head dl_scale)
        self.grad_weight = 1.0
        # persistent (work-queue) launches allowed: FusedProgram clears it for training programs
        # whose update cannot honour the step guard word (a host optimizer) or whose replicas would
        # not agree on it (data parallelism without the native communicator's guard all-reduce)
        self.persist_ok = True

    # ------------------------------------------------------------------ allocation
    def alloc(self, shape, dtype=BF16) -> torch.Tensor:
        if self.guard:
            return self._alloc_guarded(shape, dtype)
        t = torch.zeros(shape, dtype=dtype, device=self.device)
        self.keep.append(t)
        return t

    GUARD = 1 << 14  # elements on each side (IDC_GUARD=1 debugging aid)

    def _alloc_guarded(self, shape, dtype) -> torch.Tensor:
        """Buffer flanked by NaN guards: out-of-bounds reads poison results, out-of-bounds
        writes are found by ``guards_intact`` (see tools/guard_check.py)."""
        n = 1
        for d in (shape if isinstance(shape, (tuple, list)) else (shape,)):
            n *= int(d)
        g = self.GUARD
        base = torch.empty(n + 2 * g, dtype=dtype, device=self.device)
        fill = float("nan") if dtype.is_floating_point else 0
        base.fill_(fill)
        base[g:g + n].zero_()
        self.keep.append(base)
        self.guards.append((base, g, n))
        return base[g:g + n].view(shape)

    def nhwc(self, N, H, W, C, dtype=BF16) -> Tensor4:
        return Tensor4(self.alloc((N, H, W, C), dtype), N, H, W, C, C)

    def _stats_floats(self, n: int) -> torch.Tensor:
        """A view of ``n`` floats of the stats arena (zeroed at the start of every step)."""
        n = (n + 3) // 4 * 4
        if self._stats_size + n > self._stats_cap:
            raise RuntimeError("stats arena capacity exceeded")
        v = self.stats_arena[self._stats_size:self._stats_size + n]
        self._stats_size += n
        return v

    def stats(self, ld: int, count: int, slotted: bool = False, single: bool = False) -> Stats:
        """``slotted``: this producer spreads its adds over slot copies even when IDC_STAT_SLOTS
        is off (producers with ~1k workgroups per channel, e.g. the depthwise convs).  ``single``:
        one copy regardless (read by a persistent launch)."""
        slots = stat_slots_for(count) if ((self.stat_slots_on or slotted) and not self.det and not single) else 1
        st = Stats(self._stats_floats(2 * ld * slots), ld, count, slots,
                   self.alloc((ld,), F32) if self.shift_stats else None)
        self.all_stats.append(st)
        return st

    def emit_stats_shift(self):
        """After the last consumer of this step's statistics: every shifted statistics array's K
        becomes its batch mean (the next step's producers accumulate around it).  Issued as the
        LAST side-lane op: side-lane weight gradients read the statistics (and K) in their
        prologues, and the final side batch is forked after every main-lane op (plan.cpp issue),
        so it runs after the consumers of both lanes."""
        descs = [st for st in self.all_stats if st.shift is not None]
        if not descs:
            return
        arr = (nat.ShiftDesc * len(descs))()
        for d, st in zip(arr, descs):
            d.stats, d.shift, d.ld, d.slots = st.ptr, st.shift.data_ptr(), st.ld, st.slots
            d.inv_count = 1.0 / float(max(st.count, 1))
        host = torch.frombuffer(bytearray(C.string_at(C.addressof(arr), C.sizeof(arr))), dtype=torch.uint8)
        dev = host.to(self.device)
        self.keep.append(dev)
        self.emit(nat.OP_STATS_SHIFT, ints=(len(descs), max(st.ld for st in descs)), ptrs=(dev.data_ptr(),),
                  lane=1 if self.side_lane else 0)

    def grad_sums(self, bn: Optional["BNRef"], rows: int, grid: int = 0, slotted: bool = False):
        """(gsum, gsumx, slots, ld) for the producer of a BatchNorm backward's reductions
        (sum dZ -> d beta, sum dZ*xhat -> d gamma).  With several row blocks the producer adds
        into slot copies in the stats arena and ``finish_grad_sums`` folds them into the gradient
        arena on the side lane; consumers (bn_bwd_apply) read the copies directly."""
        if bn is None or bn.dbeta is None:
            return 0, 0, 1, 0
        if getattr(bn, "gsums", None) is not None:
            raise RuntimeError(f"{bn.layer.name}: a second BatchNorm-backward reduction producer")
        if self.det:
            # the producer's workgroup w adds only into its private slot w; a fixed-order collapse
            # into d beta / d gamma follows it; consumers read the collapsed sums
            bn.gsums = (bn.dbeta.data_ptr(), bn.dgamma.data_ptr(), 1, 0)
            return self._det_gsum_slots(bn.C, max(int(grid), 1), bn.dbeta.data_ptr(), bn.dgamma.data_ptr())
        S = stat_slots_for(rows) if (self.stat_slots_on or slotted) else 1
        if S == 1:
            bn.gsums = (bn.dbeta.data_ptr(), bn.dgamma.data_ptr(), 1, 0)
        else:
            v = self._stats_floats(2 * S * bn.C)
            bn.gsums = (v.data_ptr(), v.data_ptr() + 4 * S * bn.C, S, bn.C)
        return bn.gsums

    def finish_grad_sums(self, bn: Optional["BNRef"]):
        """After the producer op: slot copies still have to be folded into d beta / d gamma.
        The BatchNorm's bn_bwd_apply does it for free (its block 0 already sums the copies);
        ``mark_grads_ready`` and ``flush_grad_sums`` emit a collapse op for any BatchNorm whose
        apply never comes (freeze boundaries) or comes after its gradients are declared final."""
        if bn is None or getattr(bn, "gsums", None) is None:
            return
        if bn.gsums[2] > 1:
            self.pending_sums.append(bn)

    def _collapse(self, bn: "BNRef"):
        g, gx, S, ld = bn.gsums
        self.emit(nat.OP_COLLAPSE, ints=(S, ld, bn.C), ptrs=(g, bn.dbeta.data_ptr(), gx, bn.dgamma.data_ptr()))

    def flush_grad_sums(self, params=None):
        """Collapse pending slot copies (of the BatchNorms owning ``params``, or all)."""
        keep = []
        for bn in self.pending_sums:
            if params is None or any(bn.gamma is q or bn.beta is q for q in params):
                self._collapse(bn)
            else:
                keep.append(bn)
        self.pending_sums = keep

    # ------------------------------------------------------------------ op emission
    def emit(self, kind, payload=None, ints=(), floats=(), longs=(), ptrs=(), lane=0):
        """Append one op.  ``lane=1`` puts it on the plan's side stream (see plan.cpp): only for
        ops whose inputs no later main-lane op of the segment overwrites (weight gradients)."""
        raw = nat.raw(payload) if payload is not None else b""
        self.ops.append((self.segment, kind, raw, list(ints), list(floats), list(longs),
                         [int(p) for p in ptrs], lane if self.side_lane else 0))
        post, self._post = self._post, []
        for k2, i2, p2 in post:  # deterministic-mode collapses of this op's private slots
            self.ops.append((self.segment, k2, b"", list(i2), [], [], [int(q) for q in p2],
                             lane if self.side_lane else 0))

    # ------------------------------------------------------------------ deterministic mode
    def _det_gsum_slots(self, C: int, S: int, dst: int, dst2: int = 0):
        """A private [S][C] pair of slot arrays (gsum, gsumx layout: stride C) for one producer
        whose workgroup w adds only into slot w (single adder per address: exact on the zeroed
        stats arena), and the fixed-order collapse into dst/dst2 queued behind it.
        Returns (gsum, gsumx, slots, ld) for the kernel arguments."""
        raw = self._stats_floats(2 * S * C)
        r1 = raw.data_ptr()
        r2 = r1 + 4 * S * C if dst2 else 0
        self._post.append((nat.OP_COLLAPSE, (S, C, C), (r1, dst, r2, dst2)))
        return r1, r2, S, C

    @staticmethod
    def _rows_slotted(row_blocks: int) -> bool:
        # opt-in: measured neutral on VGG16 bs 256 (2.431 vs 2.402 ms/step, round 5): the block-1
        # data gradient's 2x over its forward is not the bias-gradient atomics
        return os.environ.get("IDC_GSUM_SLOTS", "0") == "1" and row_blocks >= 1024

    def slotted_sums(self, C: int, row_blocks: int, dst: int):
        """A [S][C] slot array in the stats arena for a producer with many row blocks that adds
        per-channel sums (a bias gradient) into ``dst``: block b adds into copy b % S, and a
        collapse op queued right behind the producer adds the copies into ``dst`` (IDC_GSUM_SLOTS=1).
        Returns (gsum, 0, S, ld) for the kernel arguments."""
        S = max(2, min(16, row_blocks // 64))  # (<= MAX_STAT_SLOTS: the pool backward checks it)
        v = self._stats_floats(S * C)
        self._post.append((nat.OP_COLLAPSE, (S, C, C), (v.data_ptr(), dst, 0, 0)))
        return v.data_ptr(), 0, S, C

    def _det_stats_slots(self, C: int, S: int, final: "Stats", off: int):
        """Forward statistics form: private [S][2][C] slots, collapsed into ``final`` at channel
        offset ``off``.  Returns (stats_out, stats_ld, stats_off, stats_slots)."""
        raw = self._stats_floats(2 * S * C).data_ptr()
        fin = final.ptr + 4 * off
        self._post.append((nat.OP_COLLAPSE, (S, 2 * C, C), (raw, fin, raw + 4 * C, fin + 4 * final.ld)))
        return raw, C, 0, S

    @staticmethod
    def _conv_row_tiles(M: int) -> int:
        return -(-M // 32)  # the most row tiles any conv tile shape (BM >= 32) produces

    def _rows_grid(self, M: int, C: int, per: int) -> int:
        return int(nat.load().rows_grid(int(M), int(C), int(per)))

    def _pool_grid(self, M: int, C: int, per: int) -> int:
        """Grid of the pool kernels (nn_kernels.hip pool_grid_div, IDC_POOL_GRID_DIV)."""
        ext = nat.load()
        f = getattr(ext, "pool_rows_grid", None)
        return int(f(int(M), int(C), int(per)) if f is not None else ext.rows_grid(int(M), int(C), int(per)))

    def mark_grads_ready(self, params):
        """Backward has finished producing the grads of ``params`` (for DP bucket overlap).
        While batched weight gradients are pending, the mark waits for their launch."""
        if self._wg_batch:
            self._wg_batch_marks.extend(params)
            return
        self.flush_grad_sums(params)
        idx = [i for i, p in enumerate(self.arena.params) if any(p is q for q in params)]
        if idx:
            self.bwd_marks.append((len(self.ops), min(idx)))

    # ------------------------------------------------------------------ weights
    def conv_weight(self, layer, cin_pad: Optional[int] = None, need_dgrad: bool = False,
                    center: bool = False):
        """bf16 kernel-layout copies of a Conv2D kernel (cast from the fp32 Keras master).
        ``center``: only the centre tap of a 3x3 kernel (a 'same' 3x3 conv on a 1x1 image is a 1x1
        conv with W[1,1] — the other 8 taps only ever multiply zero padding)."""
        key = (id(layer), center)
        ent = self.conv_weights.get(key)
        kh, kw = (1, 1) if center else layer.kernel_size
        cin, cout = layer.in_ch, layer.filters
        cpad = cin_pad or cin
        if ent is None:
            fwd = self.alloc((cout * kh * kw * cpad,), BF16)
            ent = {"fwd": fwd, "dgrad": None, "cpad": cpad, "layer": layer, "center": center}
            self.conv_weights[key] = ent
        if need_dgrad and ent["dgrad"] is None:
            ent["dgrad"] = self.alloc((cin * kh * kw * cout,), BF16)
        return ent

    @staticmethod
    def is_center_only(layer, H: int, W: int, stride, pads) -> bool:
        return (tuple(layer.kernel_size) == (3, 3) and H == 1 and W == 1 and tuple(stride) == (1, 1)
                and tuple(pads) == (1, 1))

    def finalize_casts(self):
        trainable_ids = {id(p) for p in self.arena.params}
        entries_all, entries_tr = [], []
        for ent in self.conv_weights.values():
            layer = ent["layer"]
            kh, kw = layer.kernel_size
            e = nat.CastEntry()
            e.src = layer.kernel.data_ptr()
            if ent["center"]:  # HWIO[1][1] is a contiguous (Cin, Cout) block = a 1x1 HWIO kernel
                e.src += (kw + 1) * layer.in_ch * layer.filters * layer.kernel.element_size()
                kh, kw = 1, 1
            e.fwd = ent["fwd"].data_ptr()
            e.dgrad = ent["dgrad"].data_ptr() if ent["dgrad"] is not None else 0
            e.KH, e.KW, e.Cin, e.Cout, e.Cpad, e.dw = kh, kw, layer.in_ch, layer.filters, ent["cpad"], 0
            entries_all.append(e)
            if id(layer.kernel) in trainable_ids:
                entries_tr.append(e)
        (self.cast_all_dev, self.cast_all_map, self.cast_all_total,
         self.cast_all_n) = self._upload_cast(entries_all)
        (self.cast_tr_dev, self.cast_tr_map, self.cast_tr_total,
         self.cast_tr_n) = self._upload_cast(entries_tr)

    def _upload_cast(self, entries):
        """Device CastEntry array + tile -> entry map for the tiled cast kernel (64x64 tiles of
        each kernel's [KH*KW*Cin, Cout] matrix; ``begin`` = the entry's first tile)."""
        if not entries:
            return None, None, 0, 0
        total = 0
        owner = []
        for i, e in enumerate(entries):
            e = entries[i]
            e.begin = total
            n = -(-(e.KH * e.KW * e.Cin) // 64) * -(-e.Cout // 64)
            owner += [i] * n
            total += n
        arr = (nat.CastEntry * len(entries))(*entries)
        host = torch.frombuffer(bytearray(C.string_at(C.addressof(arr), C.sizeof(arr))),
                                dtype=torch.uint8)
        dev = host.to(self.device)
        tmap = torch.tensor(owner, dtype=torch.int32).to(self.device)
        self.keep += [dev, tmap]
        return dev, tmap, total, len(entries)

    def finalize_moving(self):
        if not self.moving:
            self.moving_dev = None
            return
        arr = (nat.BnMovingDesc * len(self.moving))(*self.moving)
        host = torch.frombuffer(bytearray(C.string_at(C.addressof(arr), C.sizeof(arr))),
                                dtype=torch.uint8)
        self.moving_dev = host.to(self.device)
        self.keep.append(self.moving_dev)
        self.moving_maxc = max(d.C for d in self.moving)

    def add_moving(self, bn: BNRef):
        if bn.mode != 1:
            return
        st = bn.stats
        d = nat.BnMovingDesc()
        d.stats = st.ptr
        d.C = bn.C
        d.ld = st.ld
        d.slots = st.slots
        d.inv_count = 1.0 / st.count
        d.unbias = st.count / max(st.count - 1, 1)
        d.mmean = bn.layer.moving_mean.data_ptr()
        d.mvar = bn.layer.moving_variance.data_ptr()
        d.momentum = bn.layer.momentum
        d.shift = st.shift_ptr()
        self.moving.append(d)

    # ------------------------------------------------------------------ kernels
    def bwd_aff(self, bn: "BNRef", x: Tensor4, c0: int = 0, unit_alpha: bool = False,
                fold: bool = False) -> nat.BwdAff:
        """The pending backward of BatchNorm ``bn`` for its channels [c0, c0 + x.C), applied by a
        consumer while it stages its operand (common.h BwdAff): v' = A*v + B*x + C, with ``x`` the
        BatchNorm's raw forward input at the consumer's positions (a view whose channel 0 is BN
        channel c0).  ``unit_alpha``: the operand already holds A*dZ (DenseNet concat gradient).
        ``fold``: this consumer (a main-lane kernel that runs after the reductions are complete)
        also folds the statistics-slot copies of the reductions into d beta / d gamma."""
        a = nat.BwdAff()
        a.x, a.ldx = x.ptr, x.ld
        bna = bn.args()
        off = 4 * c0

        def sh(v):
            return (v or 0) + off if v else 0

        bna.stats, bna.gamma, bna.beta = sh(bna.stats), sh(bna.gamma), sh(bna.beta)
        bna.mmean, bna.mvar, bna.shift = sh(bna.mmean), sh(bna.mvar), sh(bna.shift)
        a.bn = bna
        if bn.mode == 1:
            if getattr(bn, "gsums", None) is None:
                raise RuntimeError(f"{bn.layer.name}: backward affine before its reductions")
            g, gx, S, ld = bn.gsums
            a.gsum, a.gsumx, a.gsum_slots, a.gsum_ld = g + off, gx + off, S, ld
            a.inv_n = 1.0 / float(bn.stats.count)
            if fold and bn in self.pending_sums:
                a.fold_C, a.fgsum, a.fgsumx = bn.C, g, gx
                a.fold_sum, a.fold_sumx = bn.dbeta.data_ptr(), bn.dgamma.data_ptr()
                self.pending_sums.remove(bn)
        else:
            a.inv_n = 1.0
        a.unit_alpha = 1 if unit_alpha else 0
        a.mode = 1
        return a

    def fwd_aff(self, bn: "BNRef", p: Tensor4, res: Optional[Tensor4] = None) -> nat.BwdAff:
        """A BatchNorm FORWARD (+ residual ``res``) applied by a consumer while it stages its
        operand ``p`` (common.h BwdAff mode 2): v' = sc*p + sh [+ res].  With ``aout`` the consumer
        also stores v' -- the materialised block output -- from its first column tiles."""
        a = nat.BwdAff()
        r = res if res is not None else p
        if r.C != p.C or r.M != p.M or r.is_f32 or p.is_f32:
            raise RuntimeError("forward affine needs bf16 operand and residual of one shape")
        a.x, a.ldx = r.ptr, r.ld
        a.bn = bn.args()
        a.inv_n = 1.0
        a.unit_alpha = 1 if res is not None else 0
        a.mode = 2
        return a

    def conv(self, x: Tensor4, layer, y: Tensor4, *, stride=(1, 1), pads=(0, 0), pro=None,
             bias=None, epi_act=0, out_mode=nat.OUT_BF16, stats: Optional[Stats] = None,
             stats_off=0, w=None, cin_override=None, tile=-1, bpro: Optional[nat.BwdAff] = None,
             aout: Optional[Tensor4] = None):
        """Forward conv (or, with ``w`` given, a generic conv such as a dgrad).  ``bpro`` +
        ``aout``: the staged operand is also stored (bf16, shaped like ``x``)."""
        a = nat.ConvArgs()
        a.x = x.ptr
        a.N, a.H, a.W = x.N, x.H, x.W
        a.Cin = cin_override or x.C
        a.ldx = x.ld
        a.Ho, a.Wo, a.Cout = y.H, y.W, y.C
        a.y, a.ldy = y.ptr, y.ld
        kh, kw = layer.kernel_size if layer is not None else w["k"]
        center = w is None and self.is_center_only(layer, x.H, x.W, stride, pads)
        if center:
            kh, kw, pads = 1, 1, (0, 0)
        a.KH, a.KW = kh, kw
        a.SH, a.SW = stride
        a.PT, a.PL = pads
        if w is None:
            ent = self.conv_weight(layer, cin_pad=a.Cin, center=center)
            a.w = ent["fwd"].data_ptr()
        else:
            a.w = w["ptr"]
        a.pro = pro if pro is not None else act_only(0)
        a.epi_mode = 0
        a.bias = nat.ptr(bias)
        a.epi_act = epi_act
        a.out_mode = out_mode
        M = x.N * y.H * y.W
        if stats is not None:
            a.stats_out, a.stats_ld, a.stats_off = stats.ptr, stats.ld, stats_off
            a.stats_slots = stats.slots
            a.stats_shift = stats.shift_ptr(stats_off)
            if self.det:
                a.stats_out, a.stats_ld, a.stats_off, a.stats_slots = self._det_stats_slots(
                    y.C, self._conv_row_tiles(M), stats, stats_off)
        a.mbn = act_only(0)
        if bpro is not None:
            a.bpro = bpro
            if aout is not None:
                if aout.C != x.C or aout.M != x.M or aout.is_f32 or (kh, kw) != (1, 1):
                    raise RuntimeError("operand side output must be bf16, shaped like x, of a 1x1 conv")
                a.aout, a.ldaout = aout.ptr, aout.ld
        elif aout is not None:
            raise RuntimeError("operand side output needs an operand affine")
        if tile < 0:
            tile = self._default_tile(a, M, y.C)
        self._splitk(a, M, y.C)
        self.emit(nat.OP_CONV, a, ints=(tile, 1 if x.is_f32 else 0, 1))

    # split-K workspace (conv_igemm.h): one fp32 partial-tile slab shared by every main-lane conv
    # (they run one after another on the plan stream) and one ticket array per op
    SLAB_FLOATS = 16 << 20  # 64 MB: room for 256x256 big-tile partials (conv_big.hip)

    def _splitk(self, a, M: int, cout: int):
        if self.splitk_slab is None:
            self.splitk_slab = self.alloc((self.SLAB_FLOATS,), F32)
        tiles = -(-M // 32) * -(-cout // 32)  # the smallest tile shape (32 x 32) has the most tiles
        t = self.alloc((tiles,), torch.int32)
        self.tickets.append(t)
        a.slab, a.tickets, a.ksplit = self.splitk_slab.data_ptr(), t.data_ptr(), 1
        a.slab_floats, a.tickets_n = self.SLAB_FLOATS, tiles

    def reset_tickets(self):
        for t in self.tickets:
            t.zero_()

    def _default_tile(self, a, M: int, cout: int) -> int:
        return nat.load().pick_tile(M, cout)

    def dgrad(self, dy: Tensor4, layer, dx: Tensor4, *, pads=(0, 0), mx: Optional[Tensor4] = None,
              mbn: Optional[nat.BnArgs] = None, gsum=None, gsumx=None, gbn: Optional["BNRef"] = None,
              out_mode=nat.OUT_BF16, bpro: Optional[nat.BwdAff] = None,
              bepi: Optional[nat.BwdAff] = None, aout: Optional[Tensor4] = None, slotted: bool = False):
        """Stride-1 data gradient: conv of dy with the flipped kernel; optional BN-backward
        epilogue through the BN+act that produced the forward input ``mx`` whose reductions go
        to ``gbn``'s gradient sums (or to explicit ``gsum``/``gsumx`` arrays).

        ``bpro``: dy is staged through a pending BatchNorm backward (common.h BwdAff).
        ``bepi`` (with ``mx``; ``dx`` fp32): epilogue mode 2 — instead of storing dZ, accumulate
        gamma*rstd*dZ plus ``bepi``'s pending B*x + C into the fp32 buffer ``dx`` (DenseNet).
        ``aout`` (with ``bpro``): also store the staged dy (bf16) for a side-lane weight gradient."""
        kh, kw = layer.kernel_size
        center = self.is_center_only(layer, dx.H, dx.W, (1, 1), pads)
        if center:
            kh, kw, pads = 1, 1, (0, 0)
        ent = self.conv_weight(layer, need_dgrad=True, center=center)
        a = nat.ConvArgs()
        a.x = dy.ptr
        a.N, a.H, a.W, a.Cin, a.ldx = dy.N, dy.H, dy.W, dy.C, dy.ld
        a.Ho, a.Wo, a.Cout = dx.H, dx.W, dx.C
        a.y, a.ldy = dx.ptr, dx.ld
        a.w = ent["dgrad"].data_ptr()
        a.KH, a.KW, a.SH, a.SW = kh, kw, 1, 1
        a.PT, a.PL = kh - 1 - pads[0], kw - 1 - pads[1]
        a.pro = act_only(0)
        a.mbn = act_only(0)
        if bpro is not None:
            a.bpro = bpro
            if aout is not None:
                if aout.C != dy.C or aout.M != dy.M or aout.is_f32:
                    raise RuntimeError("operand side output must be a bf16 tensor shaped like dy")
                a.aout, a.ldaout = aout.ptr, aout.ld
        elif aout is not None:
            raise RuntimeError("operand side output needs a backward-affine prologue")
        if bepi is not None:
            if mx is None or not dx.is_f32:
                raise RuntimeError("epilogue mode 2 needs mx and an fp32 destination")
            a.bepi = bepi
        if mx is not None:
            a.epi_mode = 2 if bepi is not None else 1
            a.mx, a.ldmx = mx.ptr, mx.ld
            a.mbn = mbn
            if bepi is None and dx.is_f32:
                # epilogue 1 into fp32: dL/dy (accumulated for OUT_F32_ACC) stored unmasked-rounded
                # and reduced against mx -- a BatchNorm OUTPUT's gradient (block outputs with a
                # residual); an activation mask on an accumulated sum would be meaningless
                if out_mode not in (nat.OUT_F32, nat.OUT_F32_ACC) or (out_mode == nat.OUT_F32_ACC and mbn.act):
                    raise RuntimeError("fp32 epilogue-1 dgrad needs OUT_F32 / OUT_F32_ACC without activation")
                a.out_mode = out_mode
            if gbn is not None:
                a.gsum, a.gsumx, a.gsum_slots, a.gsum_ld = self.grad_sums(gbn, dx.M, self._conv_row_tiles(dx.M),
                                                                          slotted=slotted)
            elif self.det and (gsum is not None or gsumx is not None):
                a.gsum, a.gsumx, a.gsum_slots, a.gsum_ld = self._det_gsum_slots(
                    dx.C, self._conv_row_tiles(dx.M), nat.ptr(gsum) if gsum is not None else nat.ptr(gsumx),
                    nat.ptr(gsumx) if (gsum is not None and gsumx is not None) else 0)
                if gsum is None:
                    a.gsum, a.gsumx = 0, a.gsum
            elif gsum is not None and gsumx is None and self._rows_slotted(self._conv_row_tiles(dx.M)):
                a.gsum, _, a.gsum_slots, a.gsum_ld = self.slotted_sums(dx.C, self._conv_row_tiles(dx.M),
                                                                       nat.ptr(gsum))
            else:
                a.gsum, a.gsumx = nat.ptr(gsum), nat.ptr(gsumx)
        else:
            a.epi_mode = 0
            a.out_mode = out_mode
        tile = self._default_tile(a, dx.M, dx.C)
        self._splitk(a, dx.M, dx.C)
        self.emit(nat.OP_CONV, a, ints=(tile, 1 if dy.is_f32 else 0, 1))
        self.finish_grad_sums(gbn)

    def wgrad(self, x: Tensor4, layer, g: Tensor4, dw: torch.Tensor, *, stride=(1, 1), pads=(0, 0),
              pro=None, cin_real=0, splits=-1, lane=0, gpro: Optional[nat.BwdAff] = None, batch=False):
        kh, kw = layer.kernel_size
        if self.is_center_only(layer, x.H, x.W, stride, pads):
            # only the centre tap sees data: its gradient is the 1x1 wgrad; the other taps keep
            # the zero the gradient arena was cleared to
            if dw.numel() != kh * kw * layer.in_ch * layer.filters:
                raise RuntimeError(f"wgrad target of {layer.name} has {dw.numel()} elements")
            dw = dw.view(kh, kw, layer.in_ch, layer.filters)[1, 1]
            kh, kw, pads = 1, 1, (0, 0)
        a = nat.WgradArgs()
        a.x = x.ptr
        a.N, a.H, a.W, a.Cin, a.ldx = x.N, x.H, x.W, x.C, x.ld
        a.g, a.ldg = g.ptr, g.ld
        a.Ho, a.Wo, a.Cout = g.H, g.W, g.C
        a.KH, a.KW = kh, kw
        a.SH, a.SW = stride
        a.PT, a.PL = pads
        a.pro = pro if pro is not None else act_only(0)
        if gpro is not None:
            a.gpro = gpro
        a.dw = dw.data_ptr()
        a.scale = 1.0
        if not cin_real and x.C != layer.in_ch:
            cin_real = layer.in_ch  # channel-padded staged input (first conv): Keras rows only
        if dw.numel() != kh * kw * layer.in_ch * layer.filters:
            raise RuntimeError(f"wgrad target of {layer.name} has {dw.numel()} elements")
        if not dw.is_contiguous():
            raise RuntimeError(f"wgrad target of {layer.name} is not contiguous")
        a.cin_real = cin_real
        if splits < 0:
            splits = nat.load().pick_splits(g.M, kh * kw * x.C, g.C)
        if batch and not self.det and lane == 1 and self.side_lane:
            if nat.load().wgrad_batch_sig(nat.raw(a), 1 if g.is_f32 else 0, 0) >= 0:
                self._wg_batch.append((a, splits))
                return
        if self.det:
            # per-slice partials + a fixed-order reduce instead of float atomics (plan.cpp OP_WGRAD);
            # one slab per lane, reused by that lane's wgrads (a lane runs them one after another)
            ln = lane if self.side_lane else 0
            need = int(nat.load().effective_splits(nat.raw(a), splits)) * dw.numel()
            slab = self._wslab.get(ln)
            if slab is None or slab.numel() < need:
                slab = self.alloc((max(need, 2 * (slab.numel() if slab is not None else 0)),), F32)
                self._wslab[ln] = slab
            a.part, a.part_floats = slab.data_ptr(), slab.numel()
        elif nat.load().wgrad_stem_ok(nat.raw(a), 1 if g.is_f32 else 0):
            # the image-resident stem weight gradient (wgrad_stem.hip) stores one partial dW per
            # workgroup into its own slab, summed in order right after (plan.cpp OP_WGRAD): float
            # atomics from its ~500-1000 workgroups onto the same few thousand addresses serialise
            need = int(nat.load().effective_splits(nat.raw(a), splits)) * dw.numel()
            slab = self.alloc((need,), F32)
            a.part, a.part_floats = slab.data_ptr(), slab.numel()
        self.emit(nat.OP_WGRAD, a, ints=(splits, 1 if g.is_f32 else 0), lane=lane)

    def has_wgrad_batch(self) -> bool:
        return bool(self._wg_batch)

    def flush_wgrad_batch(self):
        """Launch the collected weight gradients: one OP_WGRAD_BATCH per kernel shape (members in
        collection order, at most WG_BATCH_MAX each) on the side lane, then the gradient-ready
        marks that waited for them."""
        if not self._wg_batch:
            return
        ext = nat.load()
        members, self._wg_batch = self._wg_batch, []
        groups: Dict[int, list] = {}
        for a, splits in members:
            groups.setdefault(int(ext.wgrad_batch_sig(nat.raw(a), 0, 0)), []).append((a, splits))
        for sig, mem in groups.items():
            for i in range(0, len(mem), int(ext.WG_BATCH_MAX)):
                chunk = mem[i:i + int(ext.WG_BATCH_MAX)]
                tab, begins, total, smem, sig2 = ext.wgrad_batch_pack([nat.raw(a) for a, _ in chunk],
                                                                       [int(s) for _, s in chunk])
                tdev = torch.frombuffer(bytearray(tab), dtype=torch.uint8).to(self.device)
                bdev = torch.tensor(begins, dtype=torch.int32).to(self.device)
                self.keep += [tdev, bdev]
                self.emit(nat.OP_WGRAD_BATCH, ints=(len(chunk), int(total), int(sig2)), longs=(int(smem),),
                          ptrs=(tdev.data_ptr(), bdev.data_ptr()), lane=1)
        marks, self._wg_batch_marks = self._wg_batch_marks, []
        if marks:
            self.mark_grads_ready(marks)

    # ------------------------------------------------------------------ persistent dense stage
    def _fail_words(self, a):
        """Point a persistent launch's give-up sinks at this program's step guard (training
        programs: the optimizer skips a step whose launch gave up) and its pinned host flag."""
        if self.training:
            if self.step_flag is None:
                self.step_flag = self._stats_floats(4).view(torch.int32)
            a.stepflag = self.step_flag.data_ptr()
        if getattr(self, "grouped", False):
            return  # a grouped program's pointers all lie in its region (the trainer reads dense_err)
        if not self.host_flag and torch.cuda.is_available():  # (CPU-only lowering tests: none)
            self.host_flag = _host_flag_slot()
        a.hostflag = self.host_flag

    def dense_stage_ok(self, sbuf: Optional[Stats], layers, H: int, W: int) -> bool:
        """Whether the dense layers of one stage can run as ONE persistent launch
        (csrc/kernels/dense_stage.hip): training-mode BatchNorms on single-copy statistics,
        1x1 inputs of <= DS_MAX_CIN (2,048) channels in multiples of 32 (DenseNet-121/169/201),
        128-channel bottlenecks, 32 new channels per layer, maps whose 3x3 windows fit the
        launch's staging rows, and no fixed-order (deterministic) reductions."""
        if os.environ.get("IDC_DENSE_STAGE", "1") == "0" or self.det or persistent_disabled() \
                or not self.persist_ok:
            return False
        infer = all(lay["bn1"].mode == 2 and lay["bn2"].mode == 2 for lay in layers)
        if infer:
            # inference-mode BatchNorms (evaluation programs, a frozen base): moving statistics,
            # nothing produced but the stage buffer and t (IDC_DENSE_STAGE_INFER=0: per layer)
            if os.environ.get("IDC_DENSE_STAGE_INFER", "1") == "0":
                return False
        else:
            # a training program: every slice's statistics are produced; a frozen layer (fine-tuning
            # cut inside the stage) normalises with its moving statistics (per-layer mode bits)
            if not self.training or sbuf is None or sbuf.slots != 1:
                return False
        ext = nat.load()
        for lay in layers:
            if not infer and (lay["bn1"].mode not in (1, 2) or lay["bn2"].mode not in (1, 2)
                              or lay["stt"] is None or lay["stt"].slots != 1):
                return False
            if lay["cin"] % 32 or lay["cin"] > int(ext.DS_MAX_CIN) or lay["cv1"].filters != 128 \
                    or lay["cv2"].filters != 32:
                return False
            if tuple(lay["cv2"].kernel_size) != (3, 3) or tuple(lay["cv1"].kernel_size) != (1, 1):
                return False
        return bool(ext.dense_stage_shape_ok(self.B, H, W, max(lay["cin"] for lay in layers)))

    def _dense_layer_table(self, layers, center: bool, infer: bool) -> torch.Tensor:
        """Device table of DenseLayerDesc (dense_stage.h) for a stage's dense layers."""
        arr = (nat.DenseLayerDesc * len(layers))()
        for d, lay in zip(arr, layers):
            cin, bn1, bn2 = lay["cin"], lay["bn1"], lay["bn2"]
            d.w1 = self.conv_weight(lay["cv1"], cin_pad=cin)["fwd"].data_ptr()
            d.w2 = self.conv_weight(lay["cv2"], cin_pad=128, center=center)["fwd"].data_ptr()
            d.g1, d.b1 = bn1.gamma.data_ptr(), bn1.beta.data_ptr()
            d.g2, d.b2 = bn2.gamma.data_ptr(), bn2.beta.data_ptr()
            if lay.get("stt") is not None:
                d.tstats, d.tshift = lay["stt"].ptr, lay["stt"].shift_ptr()
            d.t = lay["t"].ptr if lay.get("t") is not None else 0
            d.eps1, d.eps2 = bn1.layer.epsilon, bn2.layer.epsilon
            d.cin = cin
            d.mm1, d.mv1 = bn1.layer.moving_mean.data_ptr(), bn1.layer.moving_variance.data_ptr()
            d.mm2, d.mv2 = bn2.layer.moving_mean.data_ptr(), bn2.layer.moving_variance.data_ptr()
            d.pad_ = 0 if infer else (1 if bn1.mode == 2 else 0) | (2 if bn2.mode == 2 else 0)
        host = torch.frombuffer(bytearray(C.string_at(C.addressof(arr), C.sizeof(arr))), dtype=torch.uint8)
        tab = host.to(self.device)
        self.keep.append(tab)
        return tab

    def dense_infer(self, buf: Tensor4, layers, act: int) -> bool:
        """A whole dense block in inference mode as ONE launch (dense_infer.hip): every layer's
        BatchNorms on moving statistics, nothing downstream needing the stage's statistics.  Writes
        the new channels into ``buf``; no t buffers, no statistics.  False (nothing emitted) outside
        the kernel's shapes, in grouped programs or with IDC_DENSE_INFER=0."""
        if os.environ.get("IDC_DENSE_INFER", "1") != "1" or getattr(self, "grouped", False):
            return False
        if any(lay["bn1"].mode != 2 or lay["bn2"].mode != 2 for lay in layers):
            return False
        if any(tuple(lay["cv2"].kernel_size) != (3, 3) or tuple(lay["cv1"].kernel_size) != (1, 1)
               or lay["cv1"].filters != 128 or lay["cv2"].filters != 32 for lay in layers):
            return False
        center = self.is_center_only(layers[0]["cv2"], buf.H, buf.W, (1, 1), (1, 1))
        if center != (buf.H == 1 and buf.W == 1):  # (the kernel takes the centre slice on 1x1 maps)
            return False
        ext = nat.load()
        a = nat.DenseInferArgs()
        a.buf, a.ld = buf.ptr, buf.ld
        a.N, a.H, a.W, a.c0, a.L, a.act = buf.N, buf.H, buf.W, layers[0]["cin"], len(layers), layers[0]["bn1"].act
        if any(lay["cin"] != a.c0 + 32 * i for i, lay in enumerate(layers)):
            return False
        # one image per workgroup: with the layer's weight fragments held in registers the
        # re-read is cheap and twice the workgroups wins (measured 0.973-0.980 ms frozen step
        # at ipg 1 vs 1.012-1.014 at ipg 2 on the 6x6 stage); maps of fewer than
        # IDC_DENSE_INFER_ROWS pixels group images up to that many rows (1x1 maps: 16 images);
        # IDC_DENSE_INFER_IPG overrides
        rows = int(os.environ.get("IDC_DENSE_INFER_ROWS", "16"))
        want = int(os.environ.get("IDC_DENSE_INFER_IPG", "0")) or max(1, rows // (buf.H * buf.W))
        for ipg in sorted({want, 1}, reverse=True):
            a.ipg = ipg
            a.layers = 1  # (placeholder: the size query checks shapes only)
            if int(ext.dense_infer_smem(nat.raw(a))) >= 0:
                a.layers = self._dense_layer_table(layers, center, True).data_ptr()
                self.emit(nat.OP_DENSE_INFER, a)
                return True
        return False

    def dense_img_candidate(self, rows: int, H: int, W: int) -> bool:
        """Before a stage's statistics are allocated: whether it may take the per-image training
        launch (dense_img_ok), so its statistics get the single copy that launch reads."""
        return (self.training and os.environ.get("IDC_DENSE_IMG", "0") == "1" and H * W > 1
                and rows > int(os.environ.get("IDC_DENSE_STAGE_MAXM", "2304"))
                and not getattr(self, "grouped", False) and not self.shared_device and not self.det)

    def dense_img_ok(self, buf: Tensor4, sbuf: Optional[Stats], layers) -> bool:
        """Whether a TRAINING stage whose images the row-resident launch cannot hold (13x13 / 6x6
        at 50x50) can run as ONE per-image launch (dense_infer.hip dense_img_fwd, DenseStageArgs
        rows 2): the persistent-launch conditions of dense_stage_ok, 3x3 maps of more than one
        pixel, a stage buffer exactly c0 + 32 L wide, the grid co-resident (no grouped / shared-
        device programs) and the LDS fit.  IDC_DENSE_IMG=0: per-layer convs."""
        if os.environ.get("IDC_DENSE_IMG", "0") != "1" or getattr(self, "grouped", False) or self.shared_device:
            return False
        if any(lay["bn1"].mode == 2 and lay["bn2"].mode == 2 for lay in layers) or not self.training:
            return False
        if buf.H * buf.W <= 1 or buf.ld != layers[0]["cin"] + 32 * len(layers):
            return False
        if not self.dense_stage_ok(sbuf, layers, 1, 1):  # (1 x 1: skip the work-queue staging check)
            return False
        a = nat.DenseStageArgs()
        a.buf, a.ld, a.N, a.H, a.W, a.nlayers, a.k2 = buf.ptr, buf.ld, buf.N, buf.H, buf.W, len(layers), 3
        a.act1 = a.act2 = layers[0]["bn1"].act
        return bool(nat.load().dense_img_ok(nat.raw(a)))

    def dense_stage(self, buf: Tensor4, sbuf: Stats, layers, act: int, img: bool = False):
        """Emit ONE persistent launch for the dense layers ``layers`` of a stage (dicts with cin,
        bn1, cv1, bn2, cv2, t, stt as in lower_densenet): same buffers, statistics and weights as
        the per-layer convs, so everything downstream (backward included) is unchanged.  ``img``:
        the per-image training launch (dense_img_ok)."""
        H, W = buf.H, buf.W
        center = self.is_center_only(layers[0]["cv2"], H, W, (1, 1), (1, 1))
        infer = all(lay["bn1"].mode == 2 and lay["bn2"].mode == 2 for lay in layers)
        tab = self._dense_layer_table(layers, center, infer)
        if getattr(self, "dense_err", None) is None:
            # count of dense-stage launches of this program that gave up on a wait (FusedProgram
            # checks it under IDC_VALIDATE; tests read it)
            self.dense_err = self.alloc((4,), torch.int32)
        ext = nat.load()
        # counters and the in-launch statistics slots live in the stats arena: zeroed every step
        # (a program without a stats-arena reset -- evaluation -- zeroes its counters itself)
        M = buf.N * H * W
        # ticket, sharded phase counters, fail flag, per-tile split-K helper counters
        sync = self._stats_floats(int(ext.dense_stage_sync_words(M, len(layers))))
        if not self.training:
            self.memset(sync)
        # split K of the 1x1 phases' older-channel accumulation (dense_stage.hip): enough items
        # per phase to occupy the launch's grid (stage 4 at bs 256: 16 tiles x 8); not in grouped
        # programs (their K copies share the grid)
        grid = int(os.environ.get("IDC_DS_GRID", "256"))
        ksplit = 1 if getattr(self, "grouped", False) else int(ext.dense_stage_default_ksplit(M, grid))
        pfl = int(ext.dense_stage_partial_floats(M, ksplit))
        partials = self.alloc((pfl,), F32) if pfl else None
        scratch = self._stats_floats(int(ext.DS_SCRATCH_PER_LAYER) * len(layers)) if not infer else None
        a = nat.DenseStageArgs()
        a.buf = buf.ptr
        if sbuf is not None and not infer:
            a.sstats, a.sshift = sbuf.ptr, sbuf.shift_ptr()
        a.infer = 1 if infer else 0
        a.layers, a.sync, a.err = tab.data_ptr(), sync.data_ptr(), self.dense_err.data_ptr()
        a.scratch = scratch.data_ptr() if scratch is not None else 0
        a.N, a.H, a.W, a.ld, a.nlayers, a.k2 = buf.N, H, W, buf.ld, len(layers), 1 if center else 3
        a.act1 = a.act2 = act
        a.inv_count = 1.0 / float(buf.N * H * W)
        a.max_polls = int(os.environ.get("IDC_DS_MAX_POLLS", "0"))
        a.lookahead = -1 if self.shared_device else 0
        a.ksplit = ksplit
        a.partials = partials.data_ptr() if partials is not None else 0
        # row-resident form (dense_rows.hip: whole images per workgroup, only BatchNorm statistics
        # cross workgroups) where its geometry fits; not beside other launches of its kind
        # (grouped programs, concurrent federated clients: its workgroups must be co-resident)
        # Round 6, bench.py A/B (DenseNet-121 bs 256, 3 rounds on one box): stage 3 (M = 2,304) row-
        # resident 3.449-3.465 vs 3.468-3.476 ms/step work-queue (stamps: 382 vs 410 us); stage 4 (M =
        # 256, 16 workgroups) is faster on the work queue (181 vs 208 us), hence IDC_DS_ROWS_MINM
        a.rows = 1 if (os.environ.get("IDC_DS_ROWS", "1") == "1" and not getattr(self, "grouped", False)
                       and not self.shared_device
                       and M >= int(os.environ.get("IDC_DS_ROWS_MINM", "1024"))) else 0
        if img:
            a.rows = 2
        self._fail_words(a)
        if not img and os.environ.get("IDC_DS_STAMPS", "0") == "1":
            # per-work-item s_memrealtime stamps (tools/dense_stamps.py reads them after a step);
            # row-resident launches: one row per (layer, workgroup)
            rows_geo = tuple(ext.dense_rows_geometry(buf.N, H, W, buf.ld, max(lay["cin"] for lay in layers))) \
                if a.rows else (False, 0, 0, 0)
            n_items = len(layers) * rows_geo[3] if rows_geo[0] else int(ext.dense_stage_tasks(nat.raw(a)))
            stamps = self.alloc((8 * n_items,), torch.int64)
            a.stamps = stamps.data_ptr()
            self.dense_stamps = getattr(self, "dense_stamps", []) + [
                (stamps, len(layers), M, ksplit, rows_geo[3] if rows_geo[0] else 0)]
        self.emit(nat.OP_DENSE_STAGE, a, ints=(grid, len(layers)), ptrs=(tab.data_ptr(),))

    def dense_stage_bwd_ok(self, buf: Tensor4, layers, pend: "BNRef") -> bool:
        """Whether a stage's dense-layer backward can run as ONE persistent launch
        (csrc/kernels/dense_stage_bwd.hip): every layer and BatchNorm trainable in batch mode, the
        stage's consumer BatchNorm in batch mode with single-copy reductions, shapes within the
        launch's limits, no fixed-order (deterministic) reductions."""
        # Default on for the smallest maps only (lower_densenet: IDC_DENSE_STAGE_BWD_MAXM=256, stage
        # 4 at bs 256): there its one launch beats 32 latency-bound per-layer dgrads (3.94 vs 4.00-4.02
        # ms/step); on stage 3 as well its gather tiles wait on agent-coherent loads of ~3 us each
        # under load (761 + 234 us against ~720 us per-layer: 4.12 ms/step, round 4, see
        # tools/dense_stamps.py).  Not in grouped (client-batched) programs.
        if os.environ.get("IDC_DENSE_STAGE_BWD", "1") != "1" or not self.training or self.det or \
                persistent_disabled() or not self.persist_ok:
            return False
        if getattr(self, "grouped", False):
            return False
        if pend.mode != 1 or getattr(pend, "gsums", None) is None or pend.gsums[2] != 1 or pend.stats.slots != 1:
            return False
        ext = nat.load()
        c0 = layers[0]["cin"]
        if c0 % 32 or c0 <= 32 or c0 // 32 > int(ext.DSB_MAX_CG) or buf.ld % 8:
            return False
        for lay in layers:
            for bn in (lay["bn1"], lay["bn2"]):
                if bn.mode != 1 or bn.dbeta is None or bn.stats.slots != 1:
                    return False
            if lay["cin"] > int(ext.DS_MAX_CIN) or lay["cv1"].filters != 128 or lay["cv2"].filters != 32:
                return False
        return bool(ext.dense_stage_shape_ok(buf.N, buf.H, buf.W, max(lay["cin"] for lay in layers)))

    def dense_stage_bwd(self, buf: Tensor4, sbuf: Stats, layers, pend: "BNRef", dbuf: Tensor4, act: int):
        """Emit ONE persistent launch for the data gradients of a stage's dense layers (dicts as in
        lower_densenet, each with its wgrad operand buffers ``dO16`` / ``dt`` allocated).  ``dbuf``
        holds A*dZ of the stage's consumer BatchNorm ``pend`` on entry.  Returns the bf16 final
        gradient of the stage input channels [0, c0) (the transition's / stem's operand)."""
        ext = nat.load()
        N, H, W = buf.N, buf.H, buf.W
        M = N * H * W
        L = len(layers)
        c0 = layers[0]["cin"]
        center = self.is_center_only(layers[0]["cv2"], H, W, (1, 1), (1, 1))
        S = int(ext.DS_SLOTS)
        nmt = -(-M // 32)
        arr = (nat.DenseBwdLayerDesc * L)()
        for d, lay in zip(arr, layers):
            cin, bn1, bn2 = lay["cin"], lay["bn1"], lay["bn2"]
            d.w1d = self.conv_weight(lay["cv1"], cin_pad=cin, need_dgrad=True)["dgrad"].data_ptr()
            d.w2d = self.conv_weight(lay["cv2"], cin_pad=128, need_dgrad=True, center=center)["dgrad"].data_ptr()
            d.g1, d.b1 = bn1.gamma.data_ptr(), bn1.beta.data_ptr()
            d.g2, d.b2 = bn2.gamma.data_ptr(), bn2.beta.data_ptr()
            d.t, d.tstats, d.tshift = lay["t"].ptr, lay["stt"].ptr, lay["stt"].shift_ptr()
            d.dO16, d.dt = lay["dO16"].ptr, lay["dt"].ptr
            d.dbeta1, d.dgamma1 = bn1.dbeta.data_ptr(), bn1.dgamma.data_ptr()
            d.dbeta2, d.dgamma2 = bn2.dbeta.data_ptr(), bn2.dgamma.data_ptr()
            d.r1 = self._stats_floats(S * 2 * cin).data_ptr()
            d.r2 = self._stats_floats(S * 256).data_ptr()
            d.eps1, d.eps2 = bn1.layer.epsilon, bn2.layer.epsilon
            d.cin = cin
        # work queue: for l = L-1 .. 0: P_l, QN_l, G_{l-2}, GIN (l == 1); FIN1; FIN2
        from ..ops.functional import dense_bwd_queue
        ph = dense_bwd_queue(L, nmt, c0, int(ext.DSB_KG))
        parr = (nat.DenseBwdPhase * len(ph))(*[nat.DenseBwdPhase(*p) for p in ph])
        ntickets = ph[-1][0] + ph[-1][3]
        blob = C.string_at(C.addressof(arr), C.sizeof(arr)) + C.string_at(C.addressof(parr), C.sizeof(parr))
        tab = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(self.device)
        self.keep.append(tab)
        if getattr(self, "dense_err", None) is None:
            self.dense_err = self.alloc((4,), torch.int32)
        sync = self._stats_floats(int(ext.dsb_sync_words(L)))
        btot = self._stats_floats(2 * buf.ld)
        dnew = self.alloc((2 * M * 32,), F32)
        z2 = self.alloc((M * 128,), BF16)
        dx16 = self.nhwc(N, H, W, c0)
        a = nat.DenseBwdArgs()
        a.buf, a.sstats, a.sshift = buf.ptr, sbuf.ptr, sbuf.shift_ptr()
        a.dbuf, a.dnew, a.dx16, a.z2 = dbuf.ptr, dnew.data_ptr(), dx16.ptr, z2.data_ptr()
        a.pend = self.bwd_aff(pend, buf, unit_alpha=True)
        a.layers = tab.data_ptr()
        a.phases = tab.data_ptr() + C.sizeof(arr)
        a.sync, a.btot, a.err = sync.data_ptr(), btot.data_ptr(), self.dense_err.data_ptr()
        a.N, a.H, a.W, a.ld, a.c0, a.nlayers = N, H, W, buf.ld, c0, L
        a.k2, a.act, a.nphases, a.ntickets = 1 if center else 3, act, len(ph), ntickets
        a.inv_count = 1.0 / float(M)
        a.max_polls = int(os.environ.get("IDC_DS_MAX_POLLS", "0"))
        # row-resident form (dense_rows_bwd.hip) where its geometry fits (not beside other launches
        # of its kind: its workgroups must be co-resident)
        a.rows = 1 if (rows_bwd_enabled() and not getattr(self, "grouped", False) and not self.shared_device) else 0
        if a.rows:
            ok, _ipg, g = ext.dense_rows_bwd_geometry(N, H, W, buf.ld, L)
            if ok:
                n = int(ext.dense_rows_bwd_part_floats(c0, L, g))
                a.rpart, a.rpart_floats = self.alloc((n,), F32).data_ptr(), n
        self._fail_words(a)
        if os.environ.get("IDC_DS_STAMPS", "0") == "1" and a.rows:
            ok, ipg, g = ext.dense_rows_bwd_geometry(N, H, W, buf.ld, L)
            if ok:
                stamps = self.alloc((8 * L * g,), torch.int64)
                a.stamps = stamps.data_ptr()
                self.dense_bwd_stamps = getattr(self, "dense_bwd_stamps", []) + [(stamps, None, M, g, L)]
        elif os.environ.get("IDC_DS_STAMPS", "0") == "1":
            stamps = self.alloc((8 * ntickets,), torch.int64)
            a.stamps = stamps.data_ptr()
            self.dense_bwd_stamps = getattr(self, "dense_bwd_stamps", []) + [(stamps, ph, M)]
        grid = int(os.environ.get("IDC_DS_GRID", "256"))
        self.emit(nat.OP_DENSE_STAGE_BWD, a, ints=(grid, L), ptrs=(tab.data_ptr(),))
        return dx16

    def bn_bwd_apply(self, dz: Tensor4, x: Tensor4, bn: BNRef, dst: Tensor4, accumulate: bool):
        a = nat.BnBwdApplyArgs()
        a.dz, a.lddz = dz.ptr, dz.ld
        a.x, a.ldx = x.ptr, x.ld
        a.bn = bn.args()
        if bn.mode == 1:
            if getattr(bn, "gsums", None) is None:
                raise RuntimeError(f"{bn.layer.name}: BatchNorm backward apply before its reductions")
            a.gsum, a.gsumx, a.gsum_slots, a.gsum_ld = bn.gsums
            if bn in self.pending_sums:
                a.fold_sum, a.fold_sumx = bn.dbeta.data_ptr(), bn.dgamma.data_ptr()
                self.pending_sums.remove(bn)
        a.inv_n = 1.0 / float(x.M)
        a.dst, a.lddst = dst.ptr, dst.ld
        a.dst_f32 = 1 if dst.is_f32 else 0
        a.accumulate = 1 if accumulate else 0
        a.M, a.C = x.M, x.C
        if bn.mode == 1 and (bn.dbeta is None):
            raise RuntimeError("batch-mode BN backward needs gradient workspaces")
        self.emit(nat.OP_BN_BWD_APPLY, a)

    def bn_bwd_reduce(self, dy: Tensor4, x: Tensor4, bn: BNRef, dz: Tensor4):
        """dZ = dy * act'(bn(x)) and its reductions; an fp32 ``dz`` receives gamma*rstd*dZ (the
        A*dZ part of the BatchNorm backward, the rest pending for the consumers)."""
        a = nat.BnBwdReduceArgs()
        a.dy, a.lddy, a.dy_f32 = dy.ptr, dy.ld, 1 if dy.is_f32 else 0
        a.x, a.ldx = x.ptr, x.ld
        a.bn = bn.args()
        a.dz, a.lddz = dz.ptr, dz.ld
        a.dz_f32 = 1 if dz.is_f32 else 0
        a.gsum, a.gsumx, a.gsum_slots, a.gsum_ld = self.grad_sums(bn, x.M, self._rows_grid(x.M, x.C, 4) if self.det else 0)
        a.M, a.C = x.M, x.C
        self.emit(nat.OP_BN_BWD_REDUCE, a)
        self.finish_grad_sums(bn)

    def pool(self, x: Tensor4, y: Tensor4, *, k, s, pt=0, pl=0, pro=None, is_max=True,
             argmax: Optional[torch.Tensor] = None, stats: Optional[Stats] = None, stats_off=0):
        a = nat.PoolArgs()
        a.x, a.ldx = x.ptr, x.ld
        a.N, a.H, a.W, a.C = x.N, x.H, x.W, x.C
        a.pro = pro if pro is not None else act_only(0)
        a.k, a.s, a.pt, a.pl = k, s, pt, pl
        a.Ho, a.Wo = y.H, y.W
        a.y, a.ldy = y.ptr, y.ld
        a.argmax = nat.ptr(argmax)
        if stats is not None:
            a.stats, a.stats_ld, a.stats_off = stats.ptr, stats.ld, stats_off
            a.stats_slots = stats.slots
            a.stats_shift = stats.shift_ptr(stats_off)
            if self.det:
                a.stats, a.stats_ld, a.stats_off, a.stats_slots = self._det_stats_slots(
                    x.C, self._pool_grid(x.N * y.H * y.W, x.C, 1), stats, stats_off)
        self.emit(nat.OP_MAXPOOL if is_max else nat.OP_AVGPOOL, a)

    def pool_bwd(self, dy: Tensor4, dx: Tensor4, *, k, s, pt=0, pl=0, is_max=True, argmax=None,
                 x: Optional[Tensor4] = None, bn: Optional[BNRef] = None, act=0,
                 dyaff: Optional[nat.BwdAff] = None):
        """Pool backward (+ backward through the pending BN+act of the forward input ``x``).
        ``dyaff``: dy is staged through a pending BatchNorm backward; an fp32 ``dx`` receives
        gamma*rstd*dZ instead of dZ."""
        a = nat.PoolBwdArgs()
        if dyaff is not None:
            a.dyaff = dyaff
        a.dx_f32 = 1 if dx.is_f32 else 0
        a.dy, a.lddy, a.dy_f32 = dy.ptr, dy.ld, 1 if dy.is_f32 else 0
        a.argmax = nat.ptr(argmax)
        a.N, a.H, a.W, a.C = dx.N, dx.H, dx.W, dx.C
        a.k, a.s, a.pt, a.pl = k, s, pt, pl
        a.Ho, a.Wo = dy.H, dy.W
        if x is not None:
            a.x, a.ldx = x.ptr, x.ld
            a.bn = bn.args() if bn is not None else act_only(act)
            if bn is not None:
                grid = self._pool_grid(dx.M, dx.C, 4 if k <= s else 2) if self.det else 0
                a.gsum, a.gsumx, a.gsum_slots, a.gsum_ld = self.grad_sums(bn, dx.M, grid)
        else:
            a.bn = act_only(0)
        a.dx, a.lddx = dx.ptr, dx.ld
        a.is_avg = 0 if is_max else 1
        self.emit(nat.OP_POOL_BWD, a)
        self.finish_grad_sums(bn if x is not None else None)

    def bn_apply(self, x: Tensor4, bn: "BNRef", y: Tensor4, *, act: Optional[int] = None,
                 res: Optional[Tensor4] = None, stats: Optional[Stats] = None):
        """Materialise y = act(BN(x)) [+ res] (bf16), optionally reducing y's statistics."""
        self._no_det("bn_apply")
        if stats is not None and stats.shift is not None:
            raise NotImplementedError("bn_apply statistics are not shifted; allocate them with "
                                      "IDC_STATS_SHIFT=0 or reduce through a conv epilogue")
        args = bn.args()
        if act is not None:
            args.act = act
        self.emit(nat.OP_BN_APPLY, args,
                  ints=(x.ld, res.ld if res is not None else 0, y.ld, x.M, x.C,
                        stats.ld if stats is not None else 0, stats.slots if stats is not None else 1),
                  ptrs=(x.ptr, res.ptr if res is not None else 0, y.ptr,
                        stats.ptr if stats is not None else 0))

    def _dw_args(self, x: Tensor4, layer, Ho: int, Wo: int, stride: int, pads, pro) -> nat.DwArgs:
        kh, kw = layer.kernel_size
        a = nat.DwArgs()
        a.x, a.ldx = x.ptr, x.ld
        a.N, a.H, a.W, a.C = x.N, x.H, x.W, x.C
        a.pro = pro if pro is not None else act_only(0)
        a.w = layer.depthwise_kernel.data_ptr()  # fp32 master (KH, KW, C, 1), read directly
        a.KH, a.KW, a.S, a.PT, a.PL, a.Ho, a.Wo = kh, kw, stride, pads[0], pads[1], Ho, Wo
        return a

    def mb_infer(self, x: Tensor4, xbn: nat.BnArgs, res: Optional[Tensor4], ex, ebn: Optional["BNRef"], dwl,
                 dbn: "BNRef", prj, pbn: "BNRef", y: Tensor4, *, stride: int, pads, residual: bool) -> bool:
        """One MobileNetV2 block in inference mode as ONE launch (csrc/kernels/mb_infer.hip):
        y = pbn(prj(ReLU6(dbn(dw(ReLU6(ebn(ex(x_eff)))))))) (+ x_eff), x_eff = xbn(x) (+ res).
        ``ex`` None: no expand layer (block 0).  Every BatchNorm must be in inference mode.  Returns
        False (nothing emitted) when the shape is outside the kernel's limits or the program is
        grouped / deterministic; the caller then lowers the block layer by layer."""
        if os.environ.get("IDC_MB_INFER", "1") != "1" or getattr(self, "grouped", False):
            return False
        if any(bn is not None and bn.mode != 2 for bn in (ebn, dbn, pbn)):
            return False
        ext = nat.load()
        a = nat.MbInferArgs()
        a.x, a.ldx = x.ptr, x.ld
        a.xbn = xbn
        if res is not None:
            a.res, a.ldres = res.ptr, res.ld
        cexp = ex.filters if ex is not None else x.C
        if ex is not None:
            a.we = self.conv_weight(ex, cin_pad=x.C)["fwd"].data_ptr()
            a.ebn = ebn.args()
        a.wd = dwl.depthwise_kernel.data_ptr()
        a.dbn = dbn.args()
        a.wp = self.conv_weight(prj, cin_pad=cexp)["fwd"].data_ptr()
        a.pbn = pbn.args()
        a.y, a.ldy = y.ptr, y.ld
        a.N, a.H, a.W, a.Cin, a.Cexp, a.Cout = x.N, x.H, x.W, x.C, cexp, y.C
        a.Ho, a.Wo, a.S, a.PT, a.PL = y.H, y.W, stride, pads[0], pads[1]
        a.residual = 1 if residual else 0
        # whole images per workgroup: enough output rows for the 16-row MFMA tiles (>= 64), as few
        # images as that takes (every image a workgroup on the large maps); expanded channels per
        # workgroup: enough slices for >= 256 workgroups (nat.mb_infer_default_cs)
        hw = y.H * y.W
        ipg = max(1, min(x.N, -(-64 // hw)))
        if os.environ.get("IDC_MB_INFER_IPG"):
            ipg = max(1, int(os.environ["IDC_MB_INFER_IPG"]))
        for cand in (ipg, max(1, ipg // 2), max(1, ipg // 4), 1):
            a.ipg = cand
            groups = -(-x.N // cand)
            cs = nat.mb_infer_default_cs(cexp, groups, ex is not None)
            if os.environ.get("IDC_MB_INFER_CS") and ex is not None:
                cs = max(32, int(os.environ["IDC_MB_INFER_CS"]) // 32 * 32)
            while cs >= 32:
                a.cs = cs
                if -(-cexp // cs) > 1:  # several slices: the shared split-K slab + a ticket per group
                    if self.splitk_slab is None:
                        self.splitk_slab = self.alloc((self.SLAB_FLOATS,), F32)
                    a.slab = self.splitk_slab.data_ptr()
                    a.tickets = self.alloc((groups,), torch.int32).data_ptr()
                else:
                    a.slab, a.tickets = 0, 0
                if int(ext.mb_infer_smem(nat.raw(a))) >= 0 and \
                        int(ext.mb_infer_slab_floats(nat.raw(a))) <= self.SLAB_FLOATS:
                    self.emit(nat.OP_MB_INFER, a)
                    return True
                if ex is None:
                    break
                cs -= 32
        return False

    def _no_det(self, what: str):
        if self.det:
            raise NotImplementedError(f"IDC_DETERMINISTIC: {what} has no fixed-order reduction yet "
                                      "(covered: VGG16 and the DenseNet family)")

    def dwconv(self, x: Tensor4, layer, y: Tensor4, *, stride=1, pads=(1, 1), pro=None,
               stats: Optional[Stats] = None):
        self._no_det("depthwise conv")
        a = self._dw_args(x, layer, y.H, y.W, stride, pads, pro)
        a.y, a.ldy = y.ptr, y.ld
        if stats is not None:
            a.stats, a.stats_ld = stats.ptr, stats.ld
            a.stats_slots = stats.slots
            a.stats_shift = stats.shift_ptr()
        self.emit(nat.OP_DW_FWD, a)

    def _dw_dyaff(self, a: nat.DwArgs, layer, dyaff: Optional[nat.BwdAff]):
        if dyaff is None:
            return
        if tuple(layer.kernel_size) != (3, 3) or a.S not in (1, 2) or a.C % 8 or a.C > 2048:
            raise RuntimeError(f"{layer.name}: the depthwise backward-affine prologue is 3x3-only")
        a.dyaff = dyaff

    def dw_bwd_data(self, x: Tensor4, layer, dy: Tensor4, dz: Tensor4, *, stride=1, pads=(1, 1),
                    bn: Optional["BNRef"] = None, dyaff: Optional[nat.BwdAff] = None):
        """dz = (dy conv^T w) * act'(BN(x)), sums into bn's dbeta/dgamma (x = raw dw input).
        ``dyaff``: dy is staged through the pending backward of the BatchNorm after this conv."""
        a = self._dw_args(x, layer, dy.H, dy.W, stride, pads, bn.args() if bn is not None else None)
        self._dw_dyaff(a, layer, dyaff)
        a.dy, a.lddy = dy.ptr, dy.ld
        a.dx, a.lddx = dz.ptr, dz.ld
        if bn is not None:
            # slot copies: the depthwise backward runs hundreds of workgroups per channel chunk
            a.gsum, a.gsumx, a.gsum_slots, a.gsum_ld = self.grad_sums(
                bn, dz.M, slotted=os.environ.get("IDC_DW_STAT_SLOTS", "1") != "0")
        self.emit(nat.OP_DW_BWD_DATA, a)
        self.finish_grad_sums(bn)

    def dw_bwd_fused(self, x: Tensor4, layer, dy: Tensor4, dz: Tensor4, dw: torch.Tensor, *, pads=(1, 1),
                     bn: Optional["BNRef"] = None) -> bool:
        """Stride-1 3x3 depthwise backward with the data and weight gradients in ONE pass
        (dwconv.hip dw_bwd3_fused_kernel): dz as dw_bwd_data, the weight gradient's per-block
        partials into a workspace whose column sums run as a side-lane op.  Returns False (nothing
        emitted) outside the kernel's shapes."""
        kh, kw = layer.kernel_size
        a = self._dw_args(x, layer, dy.H, dy.W, 1, pads, bn.args() if bn is not None else None)
        a.dy, a.lddy = dy.ptr, dy.ld
        a.dx, a.lddx = dz.ptr, dz.ld
        a.dw = dw.data_ptr()
        ws = self.alloc((int(nat.load().dw_wgrad_ws_floats(dy.M, dy.C, kh * kw)),), F32)
        a.ws = ws.data_ptr()
        if not nat.load().dw_bwd_fused_ok(nat.raw(a)):
            return False
        if bn is not None:
            a.gsum, a.gsumx, a.gsum_slots, a.gsum_ld = self.grad_sums(
                bn, dz.M, slotted=os.environ.get("IDC_DW_STAT_SLOTS", "1") != "0")
        self.emit(nat.OP_DW_BWD_DATA, a, ints=(1,))
        self.finish_grad_sums(bn)
        self.emit(nat.OP_DW_WGRAD, a, ints=(2,), lane=1)  # column sums of the partials
        return True

    def dw_wgrad(self, x: Tensor4, layer, dy: Tensor4, dw: torch.Tensor, *, stride=1, pads=(1, 1),
                 pro=None, lane=0, dyaff: Optional[nat.BwdAff] = None):
        a = self._dw_args(x, layer, dy.H, dy.W, stride, pads, pro)
        self._dw_dyaff(a, layer, dyaff)
        a.dy, a.lddy = dy.ptr, dy.ld
        a.dw = dw.data_ptr()
        kh, kw = layer.kernel_size
        ws = self.alloc((int(nat.load().dw_wgrad_ws_floats(dy.M, dy.C, kh * kw)),), F32)
        a.ws = ws.data_ptr()  # per-op workspace: two-stage reduction, no global atomics
        self.emit(nat.OP_DW_WGRAD, a, lane=lane)

    def memset(self, t: torch.Tensor, nbytes: Optional[int] = None):
        self.emit(nat.OP_MEMSET, longs=(nbytes if nbytes is not None else t.numel() * t.element_size(),),
                  ptrs=(t.data_ptr(),))
