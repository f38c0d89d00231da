"""Functional NHWC ops on MI355X kernels (``torch.Tensor`` in / out, one launch each).

These are thin wrappers that fill the kernel argument structs and launch on the current stream.
They are what the numerics tests compare against PyTorch fp32 references, and a usable
standalone API (``torch.nn.functional``-style, but NHWC bf16 with fused BN/activation).

BN prologue/epilogue descriptors are passed as ``BN(...)`` objects:
    BN(stats=[2C] sum|sumsq, gamma, beta, count)               batch statistics (mode 1)
    BN(mean=..., var=..., gamma, beta, mode=2)                 inference statistics
    BN(act=RELU)                                               activation only
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import torch

from . import _native as nat

RELU, RELU6 = 1, 2


@dataclass
class BN:
    stats: Optional[torch.Tensor] = None
    gamma: Optional[torch.Tensor] = None
    beta: Optional[torch.Tensor] = None
    mean: Optional[torch.Tensor] = None
    var: Optional[torch.Tensor] = None
    count: int = 1
    eps: float = 1e-3
    mode: int = 1
    act: int = 0
    ld: Optional[int] = None
    shift: Optional[torch.Tensor] = None  # statistics shift K (stats hold sums of y - K)

    def args(self) -> nat.BnArgs:
        if self.stats is None and self.mean is None:
            return nat.bn_args(mode=0, act=self.act)
        C = self.ld or (self.stats.numel() // 2 if self.stats is not None else self.mean.numel())
        return nat.bn_args(stats=self.stats, gamma=self.gamma, beta=self.beta, mmean=self.mean,
                           mvar=self.var, count=self.count, eps=self.eps,
                           mode=self.mode if self.stats is not None or self.mode == 2 else 2,
                           act=self.act, C_=C, shift=self.shift)


def _ident():
    return nat.bn_args(mode=0, act=0)


def bwd_aff(x: torch.Tensor, bn: BN, gsum: Optional[torch.Tensor] = None,
            gsumx: Optional[torch.Tensor] = None, unit_alpha: bool = False,
            fold: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> nat.BwdAff:
    """Pending BatchNorm backward (csrc/kernels/common.h BwdAff) for a consumer kernel:
    the operand v it stages becomes A*v + B*x + C with A = gamma*rstd (1 with ``unit_alpha``),
    B, C from the reductions gsum = sum(dZ), gsumx = sum(dZ*xhat) over ``bn.count`` rows.
    ``fold=(dbeta, dgamma)``: the consumer's block 0 also adds gsum/gsumx into them."""
    a = nat.BwdAff()
    a.x, a.ldx = x.data_ptr(), x.shape[-1]
    a.bn = bn.args()
    a.gsum, a.gsumx = nat.ptr(gsum), nat.ptr(gsumx)
    a.gsum_slots, a.gsum_ld = 1, 0
    a.inv_n = 1.0 / float(max(bn.count, 1))
    a.unit_alpha = 1 if unit_alpha else 0
    a.mode = 1
    if fold is not None:
        a.fold_C = x.shape[-1]
        a.fgsum, a.fgsumx = nat.ptr(gsum), nat.ptr(gsumx)
        a.fold_sum, a.fold_sumx = fold[0].data_ptr(), fold[1].data_ptr()
    a._keep = (x, bn, gsum, gsumx, fold)  # the struct holds raw pointers only
    return a


def weight_fwd_layout(kernel_hwio: torch.Tensor, cpad: Optional[int] = None) -> torch.Tensor:
    """Keras HWIO fp32 -> bf16 [Cout][KH][KW][Cpad]."""
    kh, kw, cin, cout = kernel_hwio.shape
    w = kernel_hwio.permute(3, 0, 1, 2)
    if cpad and cpad > cin:
        w = torch.nn.functional.pad(w, (0, cpad - cin))
    return w.contiguous().to(torch.bfloat16)


def weight_dgrad_layout(kernel_hwio: torch.Tensor) -> torch.Tensor:
    """Keras HWIO -> bf16 flipped [Cin][KH][KW][Cout]."""
    return kernel_hwio.flip(0, 1).permute(2, 0, 1, 3).contiguous().to(torch.bfloat16)


def conv2d(x: torch.Tensor, kernel_hwio: torch.Tensor, stride=(1, 1), pads=(0, 0),
           out_hw: Optional[Tuple[int, int]] = None, pro: Optional[BN] = None,
           bias: Optional[torch.Tensor] = None, act: int = 0, out_f32: bool = False,
           stats: Optional[torch.Tensor] = None, tile: int = -1,
           w_layout: Optional[torch.Tensor] = None, ksplit: int = 1,
           stats_shift: Optional[torch.Tensor] = None, tickets: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = act(conv(pro(x)) + bias); x NHWC (bf16 or fp32), Cin % 8 == 0.  Optional output
    statistics [sum|sumsq] accumulated into ``stats`` (sums of y - ``stats_shift`` when given)."""
    N, H, W, Cin = x.shape
    kh, kw, kcin, cout = kernel_hwio.shape
    if out_hw is None:
        out_hw = ((H + 2 * pads[0] - kh) // stride[0] + 1, (W + 2 * pads[1] - kw) // stride[1] + 1)
    Ho, Wo = out_hw
    y = torch.empty((N, Ho, Wo, cout), dtype=torch.float32 if out_f32 else torch.bfloat16,
                    device=x.device)
    wl = w_layout if w_layout is not None else weight_fwd_layout(kernel_hwio, Cin)
    a = nat.ConvArgs()
    a.x = x.data_ptr()
    a.N, a.H, a.W, a.Cin, a.ldx = N, H, W, Cin, Cin
    a.Ho, a.Wo, a.Cout = Ho, Wo, cout
    a.y, a.ldy = y.data_ptr(), cout
    a.w = wl.data_ptr()
    a.KH, a.KW, a.SH, a.SW = kh, kw, stride[0], stride[1]
    a.PT, a.PL = pads
    a.pro = pro.args() if pro is not None else _ident()
    a.epi_mode = 0
    a.bias = nat.ptr(bias)
    a.epi_act = act
    a.out_mode = nat.OUT_F32 if out_f32 else nat.OUT_BF16
    if stats is not None:
        a.stats_out, a.stats_ld, a.stats_off = stats.data_ptr(), cout, 0
        a.stats_shift = nat.ptr(stats_shift)
    a.mbn = _ident()
    keep = _splitk_args(a, N * Ho * Wo, cout, ksplit, tile)
    if tickets is not None:  # a plan op's zeroed ticket array (the image kernel keeps its slots there)
        a.tickets, a.tickets_n = tickets.data_ptr(), tickets.numel()
    nat.require().conv(nat.raw(a), tile, 1 if x.dtype == torch.float32 else 0, nat.stream_handle())
    del keep
    return y


def _splitk_args(a, M: int, cout: int, ksplit: int, tile: int):
    """Split-K workspace for a one-off launch: fp32 partial slabs + zeroed tickets, sized for the
    tile shape that will actually run (the launcher rejects an undersized workspace)."""
    if ksplit <= 1:
        return None
    ext = nat.require()
    if tile < 0:
        tile = ext.pick_tile(M, cout)
    if tile in (ext.TILE_BIG128, ext.TILE_BIG128D, ext.TILE_BIG256):
        bm, bn = 256, (256 if tile == ext.TILE_BIG256 else 128)
    else:
        bm, bn = ext.tile_bm(tile), ext.tile_bn(tile)
    tiles = -(-M // bm) * -(-cout // bn)
    slab = torch.empty(tiles * ksplit * bm * bn, dtype=torch.float32, device="cuda")
    tickets = torch.zeros(tiles, dtype=torch.int32, device="cuda")
    a.slab, a.tickets, a.ksplit = slab.data_ptr(), tickets.data_ptr(), ksplit
    a.slab_floats, a.tickets_n = slab.numel(), tiles
    return slab, tickets


def conv2d_dgrad(dy: torch.Tensor, kernel_hwio: torch.Tensor, in_hw: Tuple[int, int], pads=(0, 0),
                 mx: Optional[torch.Tensor] = None, mbn: Optional[BN] = None,
                 gsum: Optional[torch.Tensor] = None, gsumx: Optional[torch.Tensor] = None,
                 out_f32: bool = False, tile: int = -1, ksplit: int = 1,
                 bpro: Optional[nat.BwdAff] = None, bepi: Optional[nat.BwdAff] = None,
                 acc: Optional[torch.Tensor] = None, aout: Optional[torch.Tensor] = None,
                 tickets: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Stride-1 data gradient.  With ``mx``/``mbn``: returns dZ = dX * act'(bn(mx)) and
    accumulates sum(dZ) into gsum, sum(dZ*xhat) into gsumx.  ``bpro``: dy staged through a
    pending BatchNorm backward.  ``bepi`` + ``acc`` (fp32): epilogue mode 2, acc += gamma*rstd*dZ
    + bepi's B*mx + C (returns ``acc``)."""
    N, Ho, Wo, Cout = dy.shape
    kh, kw, cin, _ = kernel_hwio.shape
    H, W = in_hw
    if acc is not None:
        dx = acc
    else:
        dx = torch.empty((N, H, W, cin), dtype=torch.float32 if out_f32 else torch.bfloat16,
                         device=dy.device)
    wl = weight_dgrad_layout(kernel_hwio)
    a = nat.ConvArgs()
    a.x = dy.data_ptr()
    a.N, a.H, a.W, a.Cin, a.ldx = N, Ho, Wo, Cout, Cout
    a.Ho, a.Wo, a.Cout = H, W, cin
    a.y, a.ldy = dx.data_ptr(), cin
    a.w = wl.data_ptr()
    a.KH, a.KW, a.SH, a.SW = kh, kw, 1, 1
    a.PT, a.PL = kh - 1 - pads[0], kw - 1 - pads[1]
    a.pro = _ident()
    a.mbn = _ident()
    if bpro is not None:
        a.bpro = bpro
        if aout is not None:  # the staged (affine-applied) dy, bf16, shaped like dy
            a.aout, a.ldaout = aout.data_ptr(), aout.shape[-1]
    if bepi is not None:
        a.bepi = bepi
    if mx is not None:
        a.epi_mode = 2 if bepi is not None else 1
        a.mx, a.ldmx = mx.data_ptr(), cin
        a.mbn = mbn.args()
        a.gsum, a.gsumx = nat.ptr(gsum), nat.ptr(gsumx)
    else:
        a.out_mode = nat.OUT_F32 if out_f32 else nat.OUT_BF16
    keep = _splitk_args(a, N * H * W, cin, ksplit, tile)
    if tickets is not None:
        a.tickets, a.tickets_n = tickets.data_ptr(), tickets.numel()
    nat.require().conv(nat.raw(a), tile, 1 if dy.dtype == torch.float32 else 0, nat.stream_handle())
    del keep
    return dx


def _wgrad_args(x, dy, kernel_shape, stride, pads, pro, cin_real, out, gpro):
    N, H, W, Cin = x.shape
    _, Ho, Wo, Cout = dy.shape
    a = nat.WgradArgs()
    a.x = x.data_ptr()
    a.N, a.H, a.W, a.Cin, a.ldx = N, H, W, Cin, Cin
    a.g, a.ldg = dy.data_ptr(), Cout
    a.Ho, a.Wo, a.Cout = Ho, Wo, Cout
    a.KH, a.KW, a.SH, a.SW = kernel_shape[0], kernel_shape[1], stride[0], stride[1]
    a.PT, a.PL = pads
    a.pro = pro.args() if pro is not None else _ident()
    a.dw = out.data_ptr() if out is not None else 0
    a.scale = 1.0
    a.cin_real = cin_real
    if gpro is not None:
        a.gpro = gpro
    return a


def wgrad_big_applies(x, dy, kernel_shape, stride=(1, 1), pads=(0, 0), variant: int = 1) -> bool:
    """Whether ``conv2d_wgrad(..., variant=variant)`` runs the large-tile kernel (wgrad_big.hip)."""
    a = _wgrad_args(x, dy, kernel_shape, stride, pads, None, 0, None, None)
    return bool(nat.require().wgrad_big_ok(nat.raw(a), 1 if dy.dtype == torch.float32 else 0, variant))


def conv2d_wgrad(x: torch.Tensor, dy: torch.Tensor, kernel_shape, stride=(1, 1), pads=(0, 0),
                 pro: Optional[BN] = None, cin_real: int = 0, splits: int = -1,
                 out: Optional[torch.Tensor] = None, gpro: Optional[nat.BwdAff] = None,
                 variant: int = 0, part: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dW (Keras HWIO fp32) accumulated into ``out`` (zeros if not given).  ``variant`` > 0 picks a
    large-tile kernel (``wgrad_big.hip``) where it applies; ``part`` (zeros, with ``splits``)
    selects the deterministic per-slice partial slab, summed here in slice order."""
    Cin, Cout = x.shape[3], dy.shape[3]
    kh, kw = kernel_shape[0], kernel_shape[1]
    creal = cin_real or Cin
    if out is None:
        out = torch.zeros((kh, kw, creal, Cout), dtype=torch.float32, device=x.device)
    a = _wgrad_args(x, dy, kernel_shape, stride, pads, pro, cin_real, out, gpro)
    if part is not None:
        a.part, a.part_floats = part.data_ptr(), part.numel()
    nat.require().wgrad(nat.raw(a), splits, 1 if dy.dtype == torch.float32 else 0, nat.stream_handle(), variant)
    if part is not None:
        out += part.view(-1, out.numel()).sum(0).view_as(out)
    return out


def conv2d_wgrad_batch(members) -> list:
    """Several weight gradients in ONE batched launch (OP_WGRAD_BATCH, conv_wgrad.h): ``members``
    is a list of dicts with the ``conv2d_wgrad`` arguments x, dy, kernel_shape and optionally
    stride, pads, pro, splits, out.  All members must share one batch signature (kernel shape
    class).  Returns the dW tensors."""
    ext = nat.require()
    outs, raws, splits = [], [], []
    for mb in members:
        x, dy, ks = mb["x"], mb["dy"], mb["kernel_shape"]
        out = mb.get("out")
        if out is None:
            out = torch.zeros((ks[0], ks[1], x.shape[3], dy.shape[3]), dtype=torch.float32, device=x.device)
        a = _wgrad_args(x, dy, ks, mb.get("stride", (1, 1)), mb.get("pads", (0, 0)), mb.get("pro"), 0, out, None)
        sp = mb.get("splits", -1)
        if sp < 0:
            sp = ext.pick_splits(dy.shape[0] * dy.shape[1] * dy.shape[2], ks[0] * ks[1] * x.shape[3], dy.shape[3])
        outs.append(out)
        raws.append(nat.raw(a))
        splits.append(int(sp))
    tab, begins, total, smem, sig = ext.wgrad_batch_pack(raws, splits)
    dev = members[0]["x"].device
    tdev = torch.frombuffer(bytearray(tab), dtype=torch.uint8).to(dev)
    bdev = torch.tensor(begins, dtype=torch.int32).to(dev)
    _plan1(nat.OP_WGRAD_BATCH, ints=(len(members), int(total), int(sig)), longs=(int(smem),),
           ptrs=(tdev.data_ptr(), bdev.data_ptr()))
    torch.cuda.current_stream(dev).synchronize()  # the tables die with this frame
    return outs


def _plan1(kind, payload=None, ints=(), floats=(), longs=(), ptrs=()):
    p = nat.require().Plan()
    p.add(kind, nat.raw(payload) if payload is not None else b"", list(ints), list(floats),
          list(longs), [int(q) for q in ptrs])
    p.run(0, -1, nat.stream_handle())


def pool2d(x: torch.Tensor, k: int, s: int, pads=(0, 0), is_max=True, pro: Optional[BN] = None,
           stats: Optional[torch.Tensor] = None, out_hw=None):
    N, H, W, C = x.shape
    if out_hw is None:
        out_hw = ((H + 2 * pads[0] - k) // s + 1, (W + 2 * pads[1] - k) // s + 1)
    Ho, Wo = out_hw
    y = torch.empty((N, Ho, Wo, C), dtype=torch.bfloat16, device=x.device)
    am = torch.empty((N * Ho * Wo * C,), dtype=torch.uint8, device=x.device) if is_max else None
    a = nat.PoolArgs()
    a.x, a.ldx = x.data_ptr(), C
    a.N, a.H, a.W, a.C = N, H, W, C
    a.pro = pro.args() if pro is not None else _ident()
    a.k, a.s, a.pt, a.pl, a.Ho, a.Wo = k, s, pads[0], pads[1], Ho, Wo
    a.y, a.ldy = y.data_ptr(), C
    a.argmax = nat.ptr(am)
    if stats is not None:
        a.stats, a.stats_ld, a.stats_off = stats.data_ptr(), C, 0
    _plan1(nat.OP_MAXPOOL if is_max else nat.OP_AVGPOOL, a)
    return y, am


def pool2d_bwd(dy: torch.Tensor, in_shape, k: int, s: int, pads=(0, 0), is_max=True, argmax=None,
               x: Optional[torch.Tensor] = None, bn: Optional[BN] = None, gsum=None, gsumx=None,
               dyaff: Optional[nat.BwdAff] = None, out_f32: bool = False):
    """Pool backward [through bn(x)]; ``dyaff``: dy staged through a pending BatchNorm
    backward; ``out_f32``: returns gamma*rstd*dZ in fp32 instead of dZ."""
    N, H, W, C = in_shape
    _, Ho, Wo, _ = dy.shape
    dx = torch.empty((N, H, W, C), dtype=torch.float32 if out_f32 else torch.bfloat16, device=dy.device)
    a = nat.PoolBwdArgs()
    if dyaff is not None:
        a.dyaff = dyaff
    a.dx_f32 = 1 if out_f32 else 0
    a.dy, a.lddy, a.dy_f32 = dy.data_ptr(), C, 1 if dy.dtype == torch.float32 else 0
    a.argmax = nat.ptr(argmax)
    a.N, a.H, a.W, a.C, a.k, a.s, a.pt, a.pl, a.Ho, a.Wo = N, H, W, C, k, s, pads[0], pads[1], Ho, Wo
    if x is not None:
        a.x, a.ldx = x.data_ptr(), C
        a.bn = bn.args()
        a.gsum, a.gsumx = nat.ptr(gsum), nat.ptr(gsumx)
    else:
        a.bn = _ident()
    a.dx, a.lddx = dx.data_ptr(), C
    a.is_avg = 0 if is_max else 1
    _plan1(nat.OP_POOL_BWD, a)
    return dx


def bn_bwd_apply(dz, x, bn: BN, gsum, gsumx, out_f32=False, dst=None, accumulate=False):
    M, C = x.reshape(-1, x.shape[-1]).shape
    if dst is None:
        dst = torch.zeros(x.shape, dtype=torch.float32 if out_f32 else torch.bfloat16, device=x.device)
    a = nat.BnBwdApplyArgs()
    a.dz, a.lddz, a.x, a.ldx = dz.data_ptr(), C, x.data_ptr(), C
    a.bn = bn.args()
    a.gsum, a.gsumx = nat.ptr(gsum), nat.ptr(gsumx)
    a.inv_n = 1.0 / M
    a.dst, a.lddst = dst.data_ptr(), C
    a.dst_f32 = 1 if dst.dtype == torch.float32 else 0
    a.accumulate = 1 if accumulate else 0
    a.M, a.C = M, C
    _plan1(nat.OP_BN_BWD_APPLY, a)
    return dst


def bn_bwd_reduce(dy, x, bn: BN, gsum, gsumx, store_dz=True, dz_f32=False):
    """dZ = dy * act'(bn(x)) + reductions; ``dz_f32`` returns gamma*rstd*dZ in fp32."""
    M, C = x.reshape(-1, x.shape[-1]).shape
    dz = torch.empty(x.shape, dtype=torch.float32 if dz_f32 else torch.bfloat16,
                     device=x.device) if store_dz else None
    a = nat.BnBwdReduceArgs()
    a.dy, a.lddy, a.dy_f32 = dy.data_ptr(), C, 1 if dy.dtype == torch.float32 else 0
    a.x, a.ldx = x.data_ptr(), C
    a.bn = bn.args()
    a.dz, a.lddz = nat.ptr(dz), C
    a.gsum, a.gsumx = nat.ptr(gsum), nat.ptr(gsumx)
    a.M, a.C = M, C
    a.dz_f32 = 1 if dz_f32 else 0
    _plan1(nat.OP_BN_BWD_REDUCE, a)
    return dz


def bn_stats(x: torch.Tensor) -> torch.Tensor:
    M, C = x.reshape(-1, x.shape[-1]).shape
    st = torch.zeros(2 * C, dtype=torch.float32, device=x.device)
    _plan1(nat.OP_BN_STATS, ints=(C, M, C, C, 0), ptrs=(x.data_ptr(), st.data_ptr()))
    return st


def dwconv(x, kernel, stride=1, pads=(1, 1), out_hw=None, pro: Optional[BN] = None, stats=None):
    N, H, W, C = x.shape
    kh, kw = kernel.shape[0], kernel.shape[1]
    if out_hw is None:
        out_hw = ((H + 2 * pads[0] - kh) // stride + 1, (W + 2 * pads[1] - kw) // stride + 1)
    Ho, Wo = out_hw
    y = torch.empty((N, Ho, Wo, C), dtype=torch.bfloat16, device=x.device)
    a = _dw_args(x, kernel, stride, pads, Ho, Wo, pro)
    a.y, a.ldy = y.data_ptr(), C
    if stats is not None:
        a.stats, a.stats_ld = stats.data_ptr(), C
    _plan1(nat.OP_DW_FWD, a)
    return y


def mb_infer(x: torch.Tensor, we_hwio: Optional[torch.Tensor], ebn: Optional[BN], wd: torch.Tensor, dbn: BN,
             wp_hwio: torch.Tensor, pbn: BN, stride=1, pads=(1, 1), out_hw=None, xbn: Optional[BN] = None,
             res: Optional[torch.Tensor] = None, residual=False, ipg: int = 1,
             cs: Optional[int] = None) -> torch.Tensor:
    """One MobileNetV2 block in inference mode as one launch (csrc/kernels/mb_infer.hip):
    y = pbn(conv1x1_p(dbn(dw3x3(ebn(conv1x1_e(x_eff)))))) (+ x_eff), x_eff = xbn(x) (+ res);
    ``we_hwio`` None: no expand (block 0).  BNs in mode 2 (moving statistics), ebn/dbn with ReLU6."""
    N, H, W, Cin = x.shape
    cexp = we_hwio.shape[3] if we_hwio is not None else Cin
    cout = wp_hwio.shape[3]
    if out_hw is None:
        out_hw = ((H + 2 * pads[0] - 3) // stride + 1, (W + 2 * pads[1] - 3) // stride + 1)
    Ho, Wo = out_hw
    y = torch.empty((N, Ho, Wo, cout), dtype=torch.bfloat16, device=x.device)
    we = weight_fwd_layout(we_hwio) if we_hwio is not None else None
    wp = weight_fwd_layout(wp_hwio)
    wdc = wd.contiguous()
    a = nat.MbInferArgs()
    a.x, a.ldx = x.data_ptr(), Cin
    a.xbn = xbn.args() if xbn is not None else _ident()
    if res is not None:
        a.res, a.ldres = res.data_ptr(), res.shape[-1]
    a.we = nat.ptr(we)
    a.ebn = ebn.args() if ebn is not None else _ident()
    a.wd = wdc.data_ptr()
    a.dbn, a.wp, a.pbn = dbn.args(), wp.data_ptr(), pbn.args()
    a.y, a.ldy = y.data_ptr(), cout
    a.N, a.H, a.W, a.Cin, a.Cexp, a.Cout = N, H, W, Cin, cexp, cout
    a.Ho, a.Wo, a.S, a.PT, a.PL = Ho, Wo, stride, pads[0], pads[1]
    a.residual, a.ipg = 1 if residual else 0, ipg
    a.cs = cs or nat.mb_infer_default_cs(cexp, -(-N // ipg), we is not None)
    slab = tickets = None
    if -(-cexp // a.cs) > 1:  # several slices per image group: a partial slab + a ticket per group
        tickets = torch.zeros(-(-N // ipg), dtype=torch.int32, device=x.device)
        a.tickets = tickets.data_ptr()
        slab = torch.empty(int(nat.require().mb_infer_slab_floats(nat.raw(a))), dtype=torch.float32,
                           device=x.device)
        a.slab = slab.data_ptr()
    if nat.require().mb_infer_smem(nat.raw(a)) < 0:
        raise ValueError("mb_infer: shape outside the kernel's limits")
    _plan1(nat.OP_MB_INFER, a)
    torch.cuda.current_stream(x.device).synchronize()  # weights, slab and tickets die with this frame
    return y


def _dw_args(x, kernel, stride, pads, Ho, Wo, pro):
    N, H, W, C = x.shape
    a = nat.DwArgs()
    a.x, a.ldx = x.data_ptr(), C
    a.N, a.H, a.W, a.C = N, H, W, C
    a.pro = pro.args() if pro is not None else _ident()
    a.w = kernel.contiguous().data_ptr()
    a.KH, a.KW, a.S, a.PT, a.PL, a.Ho, a.Wo = kernel.shape[0], kernel.shape[1], stride, pads[0], pads[1], Ho, Wo
    return a


def dwconv_bwd(x, kernel, dy, stride=1, pads=(1, 1), pro: Optional[BN] = None, gsum=None, gsumx=None):
    N, H, W, C = x.shape
    _, Ho, Wo, _ = dy.shape
    a = _dw_args(x, kernel, stride, pads, Ho, Wo, pro)
    dx = torch.empty_like(x)
    dw = torch.zeros(kernel.shape, dtype=torch.float32, device=x.device)
    a.dy, a.lddy = dy.data_ptr(), C
    a.dx, a.lddx = dx.data_ptr(), C
    a.gsum, a.gsumx = nat.ptr(gsum), nat.ptr(gsumx)
    a.dw = dw.data_ptr()
    ws = torch.empty(int(nat.require().dw_wgrad_ws_floats(N * Ho * Wo, C, kernel.shape[0] * kernel.shape[1])),
                     dtype=torch.float32, device=x.device)
    a.ws = ws.data_ptr()
    _plan1(nat.OP_DW_BWD_DATA, a)
    _plan1(nat.OP_DW_WGRAD, a)
    return dx, dw


def dwconv_bwd_fused(x, kernel, dy, pads=(1, 1), pro: Optional[BN] = None, gsum=None, gsumx=None):
    """Stride-1 3x3 depthwise backward, data and weight gradients in one pass
    (dwconv.hip dw_bwd3_fused_kernel) plus the partials' column sums: returns (dx, dw)."""
    N, H, W, C = x.shape
    a = _dw_args(x, kernel, 1, pads, H, W, pro)
    dx = torch.empty_like(x)
    dw = torch.zeros(kernel.shape, dtype=torch.float32, device=x.device)
    a.dy, a.lddy = dy.data_ptr(), C
    a.dx, a.lddx = dx.data_ptr(), C
    a.gsum, a.gsumx = nat.ptr(gsum), nat.ptr(gsumx)
    a.dw = dw.data_ptr()
    ws = torch.empty(int(nat.require().dw_wgrad_ws_floats(N * H * W, C, 9)), dtype=torch.float32, device=x.device)
    a.ws = ws.data_ptr()
    if not nat.require().dw_bwd_fused_ok(nat.raw(a)):
        raise ValueError("dwconv_bwd_fused: stride-1 3x3 'same' only")
    _plan1(nat.OP_DW_BWD_DATA, a, ints=(1,))
    _plan1(nat.OP_DW_WGRAD, a, ints=(2,))
    torch.cuda.current_stream(x.device).synchronize()  # ws dies with this frame
    return dx, dw


def bn_moments(stats: torch.Tensor, count: int, shift: Optional[torch.Tensor] = None):
    """(mean, unbiased variance) per channel as the BatchNorm consumers compute them from
    [sum|sumsq] statistics (with ``shift``: sums of y - K), read out through the moving-statistics
    kernel at momentum 0."""
    C = stats.numel() // 2
    mean = torch.zeros(C, dtype=torch.float32, device=stats.device)
    var = torch.zeros_like(mean)
    d = nat.BnMovingDesc()
    d.stats, d.C, d.ld, d.slots = stats.data_ptr(), C, C, 1
    d.inv_count = 1.0 / float(count)
    d.unbias = count / max(count - 1, 1)
    d.mmean, d.mvar, d.momentum = mean.data_ptr(), var.data_ptr(), 0.0
    d.shift = nat.ptr(shift)
    dev = torch.frombuffer(bytearray(bytes(d)), dtype=torch.uint8).to(stats.device)
    _plan1(nat.OP_BN_MOVING, ints=(1, C), ptrs=(dev.data_ptr(),))
    torch.cuda.synchronize()
    return mean, var


def dense_stage(buf: torch.Tensor, sstats: torch.Tensor, layers, sshift: Optional[torch.Tensor] = None,
                act: int = RELU, grid: int = 256, k2: int = 3, max_polls: int = 0, stamps: bool = False,
                infer: bool = False, ksplit: int = 1, rows: int = 0):
    """All dense layers of a DenseNet stage in one persistent launch (csrc/kernels/dense_stage.hip).

    ``buf``: NHWC bf16 stage buffer [N, H, W, ld] whose channels [0, c0) are filled and whose
    ``sstats`` ([2*ld] fp32, shifted by ``sshift``) hold their statistics; ``layers``: dicts with
    w1 ([128][cin] bf16 kernel layout), w2 ([32][k2][k2][128] bf16), g1, b1 ([cin]), g2, b2 ([128]),
    t ([N,H,W,128] bf16 output), tstats ([256] zeroed fp32), tshift ([128] or None), eps1, eps2, cin.
    ``max_polls``: bound on each wait (0: the kernel's default; tests force timeouts with 1).
    ``infer``: inference-mode BatchNorms from each layer's mm1 / mv1 ([cin]) and mm2 / mv2 ([128])
    moving statistics; no statistics are produced (``sstats`` may be None).
    ``ksplit``: work items per 1x1 tile (split K of the older channels, <= DS_MAX_KSPLIT).
    ``rows``: 1 runs the row-resident launch (dense_rows.hip) where its geometry fits; 2 the
    per-image launch of large maps (dense_infer.hip dense_img_fwd; the buffer exactly c0 + 32 L).
    Returns (sync counters [ticket, 16 per layer, last-slice count, fail], err counter, stamps or
    None) for inspection."""
    N, H, W, ld = buf.shape
    ext = nat.require()
    if max(L["cin"] for L in layers) > int(ext.DS_MAX_CIN) or \
            (rows != 2 and not ext.dense_stage_shape_ok(N, H, W, 0)):
        raise ValueError("dense_stage: shape outside the persistent launch's limits")
    arr = (nat.DenseLayerDesc * len(layers))()
    for d, L in zip(arr, layers):
        d.w1, d.w2 = L["w1"].data_ptr(), L["w2"].data_ptr()
        d.g1, d.b1, d.g2, d.b2 = (L[k].data_ptr() for k in ("g1", "b1", "g2", "b2"))
        d.t, d.tstats, d.tshift = L["t"].data_ptr(), L["tstats"].data_ptr(), nat.ptr(L.get("tshift"))
        d.eps1, d.eps2, d.cin = L["eps1"], L["eps2"], L["cin"]
        if infer:
            d.mm1, d.mv1, d.mm2, d.mv2 = (L[k].data_ptr() for k in ("mm1", "mv1", "mm2", "mv2"))
    import ctypes
    tab = torch.frombuffer(bytearray(ctypes.string_at(ctypes.addressof(arr), ctypes.sizeof(arr))),
                           dtype=torch.uint8).to(buf.device)
    M = N * H * W
    sync = torch.zeros(int(ext.dense_stage_sync_words(M, len(layers))), dtype=torch.int32, device=buf.device)
    pfl = int(ext.dense_stage_partial_floats(M, ksplit))
    partials = torch.zeros(max(pfl, 1), dtype=torch.float32, device=buf.device)
    err = torch.zeros(1, dtype=torch.int32, device=buf.device)
    scratch = torch.zeros(int(ext.DS_SCRATCH_PER_LAYER) * len(layers), dtype=torch.float32, device=buf.device)
    a = nat.DenseStageArgs()
    a.buf, a.sstats, a.sshift = buf.data_ptr(), nat.ptr(sstats), nat.ptr(sshift)
    a.infer = 1 if infer else 0
    a.layers, a.sync, a.err = tab.data_ptr(), sync.data_ptr(), err.data_ptr()
    a.scratch = scratch.data_ptr()
    a.N, a.H, a.W, a.ld, a.nlayers, a.k2 = N, H, W, ld, len(layers), k2
    a.act1 = a.act2 = act
    a.inv_count = 1.0 / float(N * H * W)
    a.max_polls = max_polls
    a.ksplit = ksplit
    a.partials = partials.data_ptr() if pfl else 0
    a.rows = rows
    st = None
    if stamps:  # (the per-image launch: one row per layer and workgroup, at most 256 workgroups)
        n = len(layers) * 256 if rows == 2 else int(ext.dense_stage_tasks(nat.raw(a)))
        st = torch.zeros(8 * n, dtype=torch.int64, device=buf.device)
        a.stamps = st.data_ptr()
    _plan1(nat.OP_DENSE_STAGE, a, ints=(grid, len(layers)), ptrs=(tab.data_ptr(),))
    torch.cuda.current_stream().synchronize()
    return sync[:3 + 16 * len(layers)], err, st


def dense_infer(buf: torch.Tensor, layers, act: int = RELU, ipg: int = 1):
    """A whole dense block in inference mode as one launch (csrc/kernels/dense_infer.hip).
    ``buf``: NHWC bf16 stage buffer [N, H, W, ld] with channels [0, c0) filled; ``layers``: dicts
    with w1 ([128][cin] bf16), w2 ([32][3][3][128] bf16; on 1x1 maps the centre slice [32][128]),
    g1, b1, mm1, mv1 ([cin]), g2, b2, mm2, mv2
    ([128]), eps1, eps2, cin (= c0 + 32 i).  Writes channels [c0, c0 + 32 L) of ``buf``."""
    N, H, W, ld = buf.shape
    arr = (nat.DenseLayerDesc * len(layers))()
    for d, L in zip(arr, layers):
        d.w1, d.w2 = L["w1"].data_ptr(), L["w2"].data_ptr()
        d.g1, d.b1, d.g2, d.b2 = (L[k].data_ptr() for k in ("g1", "b1", "g2", "b2"))
        d.mm1, d.mv1, d.mm2, d.mv2 = (L[k].data_ptr() for k in ("mm1", "mv1", "mm2", "mv2"))
        d.eps1, d.eps2, d.cin = L["eps1"], L["eps2"], L["cin"]
    import ctypes
    tab = torch.frombuffer(bytearray(ctypes.string_at(ctypes.addressof(arr), ctypes.sizeof(arr))),
                           dtype=torch.uint8).to(buf.device)
    a = nat.DenseInferArgs()
    a.buf, a.ld = buf.data_ptr(), ld
    a.N, a.H, a.W, a.c0, a.L, a.ipg, a.act = N, H, W, layers[0]["cin"], len(layers), ipg, act
    a.layers = tab.data_ptr()
    if nat.require().dense_infer_smem(nat.raw(a)) < 0:
        raise ValueError("dense_infer: shape outside the kernel's limits")
    _plan1(nat.OP_DENSE_INFER, a)
    torch.cuda.current_stream(buf.device).synchronize()  # the layer table dies with this frame


def dense_bwd_queue(L: int, nmt: int, c0: int, kg: int):
    """Work queue of a persistent dense-stage backward launch (dense_stage_bwd.hip), in ticket
    order: (first ticket, kind, layer, tiles).  Kinds: 1 P, 2 QN, 3 G, 4 GIN, 5 FIN1, 6 FIN2."""
    ph = []

    def add(kind, layer, tiles):
        ph.append((ph[-1][0] + ph[-1][3] if ph else 0, kind, layer, tiles))

    ncg = c0 // 32
    for l in range(L - 1, -1, -1):
        add(1, l, nmt)
        add(2, l, nmt)
        if l >= 2:
            add(3, l - 2, nmt * -(-(L - l) // kg))
        if l == 1:
            add(4, 0, nmt * ncg * -(-(L - 1) // kg))
    add(5, 0, nmt * ncg)
    add(6, 0, nmt * -(-c0 // 64))
    return ph


def dense_stage_bwd(buf: torch.Tensor, sstats: torch.Tensor, layers, dbuf: torch.Tensor, pend: nat.BwdAff,
                    sshift: Optional[torch.Tensor] = None, act: int = RELU, grid: int = 256, k2: int = 3,
                    max_polls: int = 0, rows: int = 0):
    """Data gradients of all dense layers of a DenseNet stage in one persistent launch
    (csrc/kernels/dense_stage_bwd.hip).

    ``buf`` / ``sstats`` / ``sshift``: the forward stage buffer [N,H,W,ld] (bf16) and its shifted
    statistics; ``dbuf``: fp32 [N,H,W,ld], A*dZ of the stage's consumer BatchNorm (updated in place);
    ``pend``: that BatchNorm's pending backward affine (``bwd_aff(buf, ..., unit_alpha=True)``);
    ``layers``: dicts with w1d ([cin][128] bf16), w2d ([128][k2][k2][32] bf16, flipped), g1, b1,
    g2, b2, t ([N,H,W,128] bf16), tstats, tshift, eps1, eps2, cin, and outputs dO16 ([N,H,W,32]
    bf16), dt ([N,H,W,128] bf16), dbeta1 / dgamma1 ([cin]), dbeta2 / dgamma2 ([128]).
    Returns (dx16 [N,H,W,c0] bf16, sync counters, err counter)."""
    ext = nat.require()
    N, H, W, ld = buf.shape
    M = N * H * W
    L = len(layers)
    c0 = layers[0]["cin"]
    S = int(ext.DS_SLOTS)
    nmt = -(-M // 32)
    dev = buf.device
    arr = (nat.DenseBwdLayerDesc * L)()
    keep = []
    for d, Ly in zip(arr, layers):
        cin = Ly["cin"]
        for k in ("w1d", "w2d", "g1", "b1", "g2", "b2", "t", "tstats", "dO16", "dt", "dbeta1", "dgamma1",
                  "dbeta2", "dgamma2"):
            setattr(d, k, Ly[k].data_ptr())
        d.tshift = nat.ptr(Ly.get("tshift"))
        r1 = torch.zeros(S * 2 * cin, device=dev)
        r2 = torch.zeros(S * 256, device=dev)
        keep += [r1, r2]
        d.r1, d.r2 = r1.data_ptr(), r2.data_ptr()
        d.eps1, d.eps2, d.cin = Ly["eps1"], Ly["eps2"], cin
    ph = dense_bwd_queue(L, nmt, c0, int(ext.DSB_KG))
    parr = (nat.DenseBwdPhase * len(ph))(*[nat.DenseBwdPhase(*p) for p in ph])
    import ctypes
    blob = ctypes.string_at(ctypes.addressof(arr), ctypes.sizeof(arr)) + \
        ctypes.string_at(ctypes.addressof(parr), ctypes.sizeof(parr))
    tab = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
    sync = torch.zeros(int(ext.dsb_sync_words(L)), dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    btot = torch.zeros(2 * ld, device=dev)
    dnew = torch.zeros(2 * M * 32, device=dev)
    z2 = torch.zeros(M * 128, dtype=torch.bfloat16, device=dev)
    dx16 = torch.zeros(N, H, W, c0, dtype=torch.bfloat16, device=dev)
    a = nat.DenseBwdArgs()
    a.buf, a.sstats, a.sshift = buf.data_ptr(), sstats.data_ptr(), nat.ptr(sshift)
    a.dbuf, a.dnew, a.dx16, a.z2 = dbuf.data_ptr(), dnew.data_ptr(), dx16.data_ptr(), z2.data_ptr()
    a.pend = pend
    a.layers, a.phases = tab.data_ptr(), tab.data_ptr() + ctypes.sizeof(arr)
    a.sync, a.btot, a.err = sync.data_ptr(), btot.data_ptr(), err.data_ptr()
    a.N, a.H, a.W, a.ld, a.c0, a.nlayers = N, H, W, ld, c0, L
    a.k2, a.act, a.nphases, a.ntickets = k2, act, len(ph), ph[-1][0] + ph[-1][3]
    a.inv_count = 1.0 / float(M)
    a.max_polls = max_polls
    a.rows = rows  # 1: the row-resident launch (dense_rows_bwd.hip) where its geometry fits
    if rows:
        ok, _ipg, g = ext.dense_rows_bwd_geometry(N, H, W, ld, L)
        if ok:
            n = int(ext.dense_rows_bwd_part_floats(c0, L, g))
            rpart = torch.zeros(n, device=dev)
            keep.append(rpart)
            a.rpart, a.rpart_floats = rpart.data_ptr(), n
    _plan1(nat.OP_DENSE_STAGE_BWD, a, ints=(grid, L), ptrs=(tab.data_ptr(),))
    torch.cuda.current_stream().synchronize()
    del keep
    return dx16, sync, err
