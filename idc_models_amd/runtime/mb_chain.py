"""Persistent MobileNetV2 block chain: lowering side of ``csrc/kernels/mb_chain.hip``.

``MbChain`` collects the expand / depthwise / project convs of consecutive inverted-residual
blocks as PHASES of one work-queue launch (OP_MB_CHAIN) instead of emitting one kernel each.
Every phase keeps the exact buffers, statistics arrays and weights of its per-layer form, so the
backward, the moving-average update and the next kernel's prologue read the same memory; a phase
additionally produces its output BatchNorm's [scale | shift] table for the next phase (written once
by the phase's last tile).  When any phase fails the kernel's shape rules (``mb_phase_ok``) or the
launch is switched off (``IDC_MB_CHAIN=0``, deterministic mode, persistent launches disabled after
a give-up), ``emit`` replays the recorded per-layer emissions instead, in the same order.

Off by default (IDC_MB_CHAIN=1 turns it on).  Measured on one MI355X, MobileNetV2 bs 256
(tools/mb_stamps.py, profiles/mobilenetv2_chain_stamps.md): the 51-phase launch spans 1.64 ms
against ~0.76 ms for the per-layer forward (3.67 vs 2.36 ms/step with the first version).  Phase
hand-offs cost ~0.5 us, but a tile is a chain of dependent memory round trips (agent-coherent
operand loads, B fragments, output stores and the arrival count) of 2-3 us each under load, with
one or two workgroups per CU to overlap them, and every phase's last tile finalises its statistics
(5-14 us) on the critical path; the per-layer kernels keep thousands of tiles in flight instead.

Reference: the MobileNetV2 base of /root/reference/dist_model_tf_mobile.py:119-121,135-138.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Callable, Dict, List, Optional, Tuple

import torch

from ..ops import _native as nat

F32 = torch.float32

# target work items per phase: two workgroups per CU on 256 CUs
_TILES = 512


def chain_enabled(b) -> bool:
    from .builder import persistent_disabled
    return os.environ.get("IDC_MB_CHAIN", "0") == "1" and not b.det and not persistent_disabled() \
        and b.persist_ok


class MbChain:
    def __init__(self, b):
        self.b = b
        self.descs: List[nat.MbPhaseDesc] = []
        self.fallback: List[Callable[[], None]] = []
        self.tab_size = 0
        self.tab_of: Dict[int, Tuple[int, int]] = {}  # id(BNRef) -> (table offset, phase index)
        self.ok = True

    # ------------------------------------------------------------------ tables
    def _tab(self, C_: int) -> int:
        off = self.tab_size
        self.tab_size += (2 * C_ + 3) // 4 * 4
        return off

    def _table(self, bn) -> Tuple[int, int]:
        """(offset, phase) of ``bn``'s [scale | shift] table; a BatchNorm produced before the launch
        gets a one-tile TAB phase (common.h bn_coeffs over its statistics, slot copies included)."""
        key = id(bn)
        if key not in self.tab_of:
            d = nat.MbPhaseDesc()
            d.kind, d.tiles, d.dep, d.N, d.Cout = nat.MB_TAB, 1, -1, 1, bn.C
            d.pre = bn.args()
            d.tab_out = self._tab(bn.C)
            self.descs.append(d)
            self.fallback.append(lambda: None)
            self.tab_of[key] = (d.tab_out, len(self.descs) - 1)
        return self.tab_of[key]

    def _out(self, d: nat.MbPhaseDesc, y, stats, bn, tiles: int):
        """Output side of a conv phase: raw tensor, statistics (single copy), BatchNorm table."""
        d.y, d.ldy = y.ptr, y.ld
        d.tiles = tiles
        d.bn_mode = bn.mode if bn is not None else 0
        if bn is not None:
            d.gamma, d.beta = bn.gamma.data_ptr(), bn.beta.data_ptr()
            d.mmean, d.mvar = bn.layer.moving_mean.data_ptr(), bn.layer.moving_variance.data_ptr()
            d.eps = bn.layer.epsilon
            d.tab_out = self._tab(bn.C)
        else:
            d.tab_out = -1
        if bn is not None and bn.mode == 1:
            if stats is None or stats.slots != 1 or stats.ld != y.C:
                self.ok = False
            else:
                d.stats, d.shift = stats.ptr, stats.shift_ptr()
                d.inv_count = 1.0 / float(stats.count)
                d.slots = max(1, min(8, -(-tiles // 64)))
                d.slotbuf = self.b._stats_floats(2 * y.C * d.slots).data_ptr()
        self.descs.append(d)
        if bn is not None:
            self.tab_of[id(bn)] = (d.tab_out, len(self.descs) - 1)

    def _operand(self, d: nat.MbPhaseDesc, pro_bn, act: int, block_out: bool):
        if pro_bn is None:
            d.pro, d.dep, d.tab_in = 0, -1, -1
            return
        d.tab_in, d.dep = self._table(pro_bn)
        d.pro = 2 if block_out else 1
        d.act_in = 0 if block_out else act

    # ------------------------------------------------------------------ phases
    def pw(self, layer, x, y, stats, bn_out, *, pro_bn=None, act=0, res=None, aout=None,
           fallback: Callable[[], None]):
        """1x1 conv ``layer``: y = W . T(x), T = BN(+act) of ``pro_bn`` (or, with ``block_out``
        semantics when ``aout``/``res`` are given, the block output BN(p) [+ res], stored to aout)."""
        block_out = aout is not None or res is not None
        d = nat.MbPhaseDesc()
        d.kind = nat.MB_PW
        M = x.N * x.H * x.W
        d.N, d.H, d.W, d.Ho, d.Wo, d.S = x.N, x.H, x.W, x.H, x.W, 1
        d.Cin, d.Cout = x.C, y.C
        d.x, d.ldx = x.ptr, x.ld
        if res is not None:
            d.res = res.ptr
            if res.ld != x.C or res.M != x.M:
                self.ok = False
        if aout is not None:
            d.aout = aout.ptr
            if aout.ld != x.C or aout.M != x.M:
                self.ok = False
        d.w16 = self.b.conv_weight(layer, cin_pad=x.C)["fwd"].data_ptr()
        self._operand(d, pro_bn, act, block_out)
        if block_out and pro_bn is None:
            self.ok = False
        # tiles: 64 rows where that still makes >= 256 row tiles; whole-K chunks of <= 256 keep all
        # columns of a row block in one tile when that leaves >= _TILES tiles
        d.tm = 64 if -(-M // 64) >= 256 else 32
        rows, cch = -(-M // d.tm), -(-y.C // 64)
        g = 1 if x.C > 256 else max(1, min(cch, (rows * cch) // _TILES))
        d.tn = 64 * g
        self._out(d, y, stats, bn_out, rows * -(-cch // g))
        self.fallback.append(fallback)

    def dw(self, layer, x, y, stride: int, pads, stats, pro_bn, act: int, bn_out, *,
           fallback: Callable[[], None]):
        d = nat.MbPhaseDesc()
        d.kind = nat.MB_DW
        d.N, d.H, d.W, d.Ho, d.Wo = x.N, x.H, x.W, y.H, y.W
        d.S, d.PT, d.PL = stride, pads[0], pads[1]
        d.Cin = d.Cout = x.C
        d.x, d.ldx = x.ptr, x.ld
        d.w32 = layer.depthwise_kernel.data_ptr()
        if tuple(layer.kernel_size) != (3, 3):
            self.ok = False
        self._operand(d, pro_bn, act, False)
        C_ = x.C
        limit = int(nat.load().MB_SMEM_LIMIT)
        cw = next((c for c in (64, 32, 16) if C_ % c == 0 and (4 * c + x.H * x.W * c) * 4 <= limit), 0)
        if cw == 0:
            self.ok = False
            cw = 16
        nch = C_ // cw
        imax = max(1, (limit // 4 - 4 * cw) // (x.H * x.W * cw))
        d.tn = cw
        d.tm = max(1, min(imax, (x.N * nch) // _TILES))
        self._out(d, y, stats, bn_out, -(-x.N // d.tm) * nch)
        self.fallback.append(fallback)

    # ------------------------------------------------------------------ emission
    def emit(self) -> bool:
        """Emit the launch (True) or, if any phase is outside the kernel's rules, the per-layer
        ops (False)."""
        b = self.b
        ext = nat.load()
        ok = self.ok and chain_enabled(b) and any(d.kind != nat.MB_TAB for d in self.descs) and \
            len(self.descs) <= int(ext.MB_MAX_PHASES)
        first = 0
        smem = 0
        if ok:
            for i, d in enumerate(self.descs):
                d.first = first
                first += d.tiles
                if d.dep >= i or (d.bn_mode not in (0, 1, 2)) or not ext.mb_phase_ok(nat.raw(d)):
                    ok = False
                    break
                smem = max(smem, int(ext.mb_phase_smem(nat.raw(d))))
        if not ok:
            for f in self.fallback:
                f()
            return False
        n = len(self.descs)
        arr = (nat.MbPhaseDesc * n)(*self.descs)
        host = torch.frombuffer(bytearray(C.string_at(C.addressof(arr), C.sizeof(arr))), dtype=torch.uint8)
        tab = host.to(b.device)
        b.keep.append(tab)
        if getattr(b, "dense_err", None) is None:
            b.dense_err = b.alloc((4,), torch.int32)
        sync = b._stats_floats(2 + 10 * n)  # mb_chain.h MB_SYNC_PER_PHASE
        if not b.training:
            b.memset(sync)
        tabs = b.alloc((max(self.tab_size, 4),), F32)
        a = nat.MbChainArgs()
        a.phases, a.sync, a.tabs, a.err = tab.data_ptr(), sync.data_ptr(), tabs.data_ptr(), b.dense_err.data_ptr()
        a.nphases, a.ntickets = n, first
        a.max_polls = int(os.environ.get("IDC_DS_MAX_POLLS", "0"))
        b._fail_words(a)
        if os.environ.get("IDC_MB_STAMPS", "0") == "1":
            stamps = b.alloc((8 * first,), torch.int64)
            a.stamps = stamps.data_ptr()
            b.mb_stamps = getattr(b, "mb_stamps", []) + [(stamps, [(d.kind, d.first, d.tiles) for d in self.descs])]
        grid = int(os.environ.get("IDC_MB_GRID", "256"))
        b.emit(nat.OP_MB_CHAIN, a, ints=(grid, smem, n), ptrs=(tab.data_ptr(),))
        b.mb_chains = getattr(b, "mb_chains", 0) + 1
        return True
