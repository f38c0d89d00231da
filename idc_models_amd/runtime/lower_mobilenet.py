"""MobileNetV2 lowering (``dist_model_tf_mobile.py`` backbone; SURVEY §2.4.2, north-star FL model).

MI355X structure:

* pointwise (1x1) convs are MFMA implicit GEMMs whose operand prologue applies the producer's
  pending BN + ReLU6 (expand -> depthwise BN and depthwise -> project BN never materialise);
* depthwise 3x3 convs are bandwidth kernels (``dwconv.hip``) that read the fp32 master kernel,
  apply the pending expand-BN + ReLU6 on load and reduce their own output statistics;
* each block output ``BN_project(p) [+ residual]`` is built by its consumer -- the next expand
  conv (or Conv_1) applies the project BN and adds the residual while staging its operand
  (common.h BwdAff mode 2) and stores the result from its first column tiles, because it is also
  the next identity block's residual and the expand weight gradient's input (IDC_MBV2_FOLD_OUT=0:
  a separate ``bn_apply`` pass);
* backward: every BatchNorm backward is reduced once by its producer and APPLIED BY ITS CONSUMERS;
  the project BN's reductions come from the epilogue of the dgrad that produces the block-output
  gradient G (next expand / Conv_1, fp32, residual-accumulated), so no reduce pass runs for them
  (common.h BwdAff: A*dZ + B*x + C staged while loading dZ) — the pointwise dgrads for the
  Conv_1, project and expand BNs (they also write the staged operand for the side-lane weight
  gradient); only the depthwise BN keeps an apply pass (its depthwise consumers re-read dZ ~4.5x,
  so staging there costs more than the pass); the project dgrad's epilogue goes through
  depthwise-BN + ReLU6, the depthwise backward-data epilogue through expand-BN + ReLU6, and the
  expand dgrad ACCUMULATES into the fp32 residual gradient in place.
Keras ``correct_pad`` asymmetric padding of stride-2 layers = top/left pad + implicit bottom/right.
"""
from __future__ import annotations

import os

import torch

from ..models.layers import correct_pad
from ..ops import _native as nat
from .builder import F32, BNRef, Builder, Tensor4, act_only
from .lower_common import RELU6, FreezeInfo, HeadIO, emit_head, emit_head_bwd, emit_input


def _dw_geometry(h, w, stride):
    if stride == 1:
        return (1, 1), h, w
    pad = correct_pad(h, w, 3)
    ho = (h + pad[0][0] + pad[0][1] - 3) // 2 + 1
    wo = (w + pad[1][0] + pad[1][1] - 3) // 2 + 1
    return (pad[0][0], pad[1][0]), ho, wo


def lower_mobilenet(b: Builder, net, U: int, input_dtype):
    from ..models.mobilenet_v2 import MBV2_BLOCKS
    base, dense = net.base, net.head
    B, training = b.B, b.training
    fz = FreezeInfo(base, training)
    L = {l.name: l for l in base.layers}
    H, W, Cimg = base.input_shape
    io = HeadIO(b, U)
    from .mb_chain import chain_enabled as _chain_on
    if _chain_on(b):
        b.stat_slots_on = False  # the chain keeps its own slot copies over single-copy statistics

    # ------------------------------------------------------------------ forward
    b.segment = "fwd"
    if training:
        b.memset(b.stats_arena)
    xin, x8 = emit_input(b, H, W, Cimg, input_dtype)
    conv1, bnl0 = L["Conv1"], L["bn_Conv1"]
    pad = correct_pad(H, W, 3)
    H1 = (H + pad[0][0] + pad[0][1] - 3) // 2 + 1
    W1 = (W + pad[1][0] + pad[1][1] - 3) // 2 + 1
    stem_pads = (pad[0][0], pad[1][0])
    y0 = b.nhwc(B, H1, W1, conv1.filters)
    s0 = b.stats(conv1.filters, B * H1 * W1, slotted=True) if training else None  # (stem: ~1k workgroups)
    b.conv(x8, conv1, y0, stride=(2, 2), pads=stem_pads, stats=s0)
    bn0 = BNRef(bnl0, b, s0, RELU6)
    b.add_moving(bn0)

    blocks = []
    h_in = None                 # materialised block input (None for block 0: pending y0/bn0)
    cin, h, w = conv1.filters, H1, W1
    # a block output BN_project(p) [+ h_in] is built by its consumer (the next expand conv or
    # Conv_1) while staging its operand, and stored from there (no separate apply pass)
    pending_out = None          # (p, bn_p, residual tensor or None) of the block just lowered
    fold_out = os.environ.get("IDC_MBV2_FOLD_OUT", "1") != "0"
    dw_slots = os.environ.get("IDC_DW_STAT_SLOTS", "1") != "0"
    dw_aff = os.environ.get("IDC_MBV2_DW_AFF", "0") == "1"

    def consume(layer, out, stats):
        """1x1 conv of the current block input; materialises it first if it is pending."""
        if pending_out is None:
            b.conv(h_in, layer, out, stats=stats)
            return
        p_, bnp_, res_ = pending_out
        b.conv(p_, layer, out, stats=stats, bpro=b.fwd_aff(bnp_, p_, res_), aout=h_in)

    # the blocks from IDC_MB_CHAIN_FROM on run as ONE persistent launch (runtime/mb_chain.py,
    # csrc/kernels/mb_chain.hip): same buffers and statistics, single-copy depthwise statistics
    from .mb_chain import MbChain, chain_enabled
    chain_from = int(os.environ.get("IDC_MB_CHAIN_FROM", "0"))
    chain = MbChain(b) if (fold_out and chain_enabled(b)) else None
    for bid, (filters, stride, t) in enumerate(MBV2_BLOCKS):
        pre = f"block_{bid}_" if bid else "expanded_conv_"
        blk = {"bid": bid, "stride": stride, "h_in": h_in}
        ch_on = chain is not None and bid >= chain_from
        # a block no gradient reaches, whose BatchNorms all run on moving statistics (evaluate(),
        # the frozen base of phase 1, the frozen prefix of the fine-tune phase): ONE launch for
        # expand -> depthwise -> project (builder.mb_infer, csrc/kernels/mb_infer.hip)
        # Only the blocks with <= IDC_MB_INFER_MAX_CEXP expanded channels (default 576: blocks 0-13):
        # there one launch beats the three per-layer ones (block 1, 25x25 -> 13x13, 96 channels: 33
        # vs 92 us); on the 2x2 blocks with 960 channels the per-layer launches are still faster
        # (frozen-base step 0.687-0.688 ms at 576, 0.703-0.708 at 192, 0.712-0.726 with every block
        # fused, 0.833-0.847 per-layer: profiles/mobilenetv2_mb_infer_blocks.md)
        prjbn_l = L[pre + "project_BN"]
        cexp_b = L[pre + "expand"].filters if bid else cin
        if not ch_on and not fz.at_or_before(prjbn_l) and \
                cexp_b <= int(os.environ.get("IDC_MB_INFER_MAX_CEXP", "576")):
            ex = L[pre + "expand"] if bid else None
            bn_e = BNRef(L[pre + "expand_BN"], b, None, RELU6) if bid else None
            dwl = L[pre + "depthwise"]
            bn_d = BNRef(L[pre + "depthwise_BN"], b, None, RELU6)
            prj = L[pre + "project"]
            bn_p = BNRef(prjbn_l, b, None, 0)
            pads, ho, wo = _dw_geometry(h, w, stride)
            pw = prj.filters
            residual = (cin == pw and stride == 1)
            hout = b.nhwc(B, ho, wo, pw)
            if bid == 0:
                xsrc, xbn, xres = y0, bn0.args(), None
            elif pending_out is not None:
                xsrc, xbn, xres = pending_out[0], pending_out[1].args(), pending_out[2]
            else:
                xsrc, xbn, xres = h_in, act_only(0), None
            if b.mb_infer(xsrc, xbn, xres, ex, bn_e, dwl, bn_d, prj, bn_p, hout, stride=stride, pads=pads,
                          residual=residual):
                blk.update(ex=ex, e=None, bn_in=bn_e if bid else bn0, dwl=dwl, pads=pads, d=None, bn_d=bn_d,
                           prj=prj, p=None, bn_p=bn_p, residual=residual, h_out=hout, fused=True)
                blocks.append(blk)
                pending_out = None
                h_in, cin, h, w = hout, pw, ho, wo
                continue
        if bid:
            ex, exbn = L[pre + "expand"], L[pre + "expand_BN"]
            e = b.nhwc(B, h, w, ex.filters)
            se = b.stats(ex.filters, B * h * w) if training else None
            bn_e = BNRef(exbn, b, se, RELU6)
            if ch_on:
                fb = (lambda ex=ex, e=e, se=se, po=pending_out, hi=h_in:
                      b.conv(hi, ex, e, stats=se) if po is None else
                      b.conv(po[0], ex, e, stats=se, bpro=b.fwd_aff(po[1], po[0], po[2]), aout=hi))
                if pending_out is None:
                    chain.pw(ex, h_in, e, se, bn_e, fallback=fb)
                else:
                    p_, bnp_, res_ = pending_out
                    chain.pw(ex, p_, e, se, bn_e, pro_bn=bnp_, res=res_, aout=h_in, fallback=fb)
            else:
                consume(ex, e, se)
            pending_out = None
            b.add_moving(bn_e)
            blk.update(ex=ex, e=e, bn_in=bn_e)
            dw_in, bn_in = e, bn_e
        else:
            dw_in, bn_in = y0, bn0
            blk.update(ex=None, e=y0, bn_in=bn0)
        dwl, dwbn = L[pre + "depthwise"], L[pre + "depthwise_BN"]
        pads, ho, wo = _dw_geometry(h, w, stride)
        ch = dw_in.C
        d = b.nhwc(B, ho, wo, ch)
        # the depthwise kernels run ~300-700 workgroups per channel chunk: one statistics copy took
        # that many float atomics per address (H=25 C=32: 28.6 us with, 14.5 us without the
        # statistics epilogue; 16.9 us with slot copies, tools/bench_dw.py); the chain reduces its
        # slot copies in-launch and keeps ONE copy
        sd = b.stats(ch, B * ho * wo, slotted=dw_slots and not ch_on) if training else None
        bn_d = BNRef(dwbn, b, sd, RELU6)
        if ch_on:
            chain.dw(dwl, dw_in, d, stride, pads, sd, bn_in, RELU6, bn_d,
                     fallback=lambda dwl=dwl, dw_in=dw_in, d=d, stride=stride, pads=pads, bn_in=bn_in, sd=sd:
                     b.dwconv(dw_in, dwl, d, stride=stride, pads=pads, pro=bn_in.args(), stats=sd))
        else:
            b.dwconv(dw_in, dwl, d, stride=stride, pads=pads, pro=bn_in.args(), stats=sd)
        b.add_moving(bn_d)
        prj, prjbn = L[pre + "project"], L[pre + "project_BN"]
        pw = prj.filters
        p = b.nhwc(B, ho, wo, pw)
        sp = b.stats(pw, B * ho * wo) if training else None
        bn_p = BNRef(prjbn, b, sp, 0)
        if ch_on:
            chain.pw(prj, d, p, sp, bn_p, pro_bn=bn_d, act=RELU6,
                     fallback=lambda prj=prj, d=d, p=p, bn_d=bn_d, sp=sp: b.conv(d, prj, p, pro=bn_d.args(), stats=sp))
        else:
            b.conv(d, prj, p, pro=bn_d.args(), stats=sp)
        b.add_moving(bn_p)
        residual = (cin == pw and stride == 1)
        hout = b.nhwc(B, ho, wo, pw)
        if fold_out:
            pending_out = (p, bn_p, h_in if residual else None)
        else:
            b.bn_apply(p, bn_p, hout, res=h_in if residual else None)
        blk.update(dwl=dwl, pads=pads, d=d, bn_d=bn_d, prj=prj, p=p, bn_p=bn_p, residual=residual,
                   h_out=hout)
        blocks.append(blk)
        h_in, cin, h, w = hout, pw, ho, wo

    if chain is not None:
        chain.emit()
    c1l, c1bnl = L["Conv_1"], L["Conv_1_bn"]
    c1 = b.nhwc(B, h, w, c1l.filters)
    sc1 = b.stats(c1l.filters, B * h * w) if training else None
    consume(c1l, c1, sc1)
    pending_out = None
    bn_c1 = BNRef(c1bnl, b, sc1, RELU6)
    b.add_moving(bn_c1)
    emit_head(b, c1, bn_c1.args(), dense, U, io, training)
    if training:
        b.emit("MOVING")
    b.xin, b.io = xin, io
    b.debug = {"y0": y0, "blocks": blocks, "c1": c1}
    if not training:
        return

    # ------------------------------------------------------------------ backward
    b.segment = "bwd"
    b.memset(b.arena.grad)
    need_base = fz.at_or_before(c1bnl)
    dA = emit_head_bwd(b, c1, dense, U, io, need_dA=need_base)
    if not need_base:
        return
    zc = b.nhwc(c1.N, c1.H, c1.W, c1.C)
    b.bn_bwd_reduce(dA, c1, bn_c1, zc)
    if not fz.before(c1bnl):
        b.mark_grads_ready([bn_c1.gamma, bn_c1.beta])
        return
    dc1 = b.nhwc(c1.N, c1.H, c1.W, c1.C)
    h_last = blocks[-1]["h_out"]
    if not fz.before(c1l):
        b.bn_bwd_apply(zc, c1, bn_c1, dc1, accumulate=False)
        b.mark_grads_ready([bn_c1.gamma, bn_c1.beta])
        if fz.trainable(c1l):
            b.wgrad(h_last, c1l, dc1, b.arena.grad_of(c1l.kernel), lane=1)
        b.mark_grads_ready([c1l.kernel])
        return
    # the BatchNorm backward of Conv_1_bn is staged by its consumer: the dgrad applies
    # A*dZ + B*x + C while loading dZ (and folds the BN's reductions), and writes the staged
    # operand for the side-lane weight gradient (no separate apply pass)
    def fold_ok(blk):
        # the block-output gradient G's producer (the next expand dgrad, or Conv_1's) reduces the
        # project BN's backward sums in its epilogue when the block continues into its project
        # dgrad (which then reads G in fp32 through the BN-backward prologue): no reduce pass
        return fz.before(blk["bn_p"].layer) and fz.before(blk["prj"])

    def g_epilogue(blk):
        if not fold_ok(blk):
            return {}
        return {"mx": blk["p"], "mbn": blk["bn_p"].args(), "gbn": blk["bn_p"]}

    G = b.nhwc(h_last.N, h_last.H, h_last.W, h_last.C, F32)
    b.dgrad(zc, c1l, G, out_mode=nat.OUT_F32, bpro=b.bwd_aff(bn_c1, c1, fold=True), aout=dc1,
            **g_epilogue(blocks[-1]))
    b.mark_grads_ready([bn_c1.gamma, bn_c1.beta])
    if fz.trainable(c1l):
        b.wgrad(h_last, c1l, dc1, b.arena.grad_of(c1l.kernel), lane=1)
    b.mark_grads_ready([c1l.kernel])

    for blk in reversed(blocks):
        p, bn_p, d, bn_d = blk["p"], blk["bn_p"], blk["d"], blk["bn_d"]
        prj, dwl = blk["prj"], blk["dwl"]
        # project BN (no activation): G is the gradient of BN_p(p) (+ residual passthrough)
        if fold_ok(blk):
            zp = G  # reduced by G's producer; the project dgrad stages A*G + B*p + C from fp32
        else:
            zp = b.nhwc(p.N, p.H, p.W, p.C)
            b.bn_bwd_reduce(G, p, bn_p, zp)
        if not fz.before(bn_p.layer):
            b.mark_grads_ready([bn_p.gamma, bn_p.beta])
            return
        dp = b.nhwc(p.N, p.H, p.W, p.C)
        if not fz.before(prj):
            b.bn_bwd_apply(zp, p, bn_p, dp, accumulate=False)
            b.mark_grads_ready([bn_p.gamma, bn_p.beta])
            if fz.trainable(prj):
                b.wgrad(d, prj, dp, b.arena.grad_of(prj.kernel), pro=bn_d.args(), lane=1)
            b.mark_grads_ready([prj.kernel])
            return
        # project dgrad: prologue = project-BN backward, epilogue = backward through the
        # depthwise BN + ReLU6 (dZ_d and its reductions); dp side output for the wgrad
        zd = b.nhwc(d.N, d.H, d.W, d.C)
        b.dgrad(zp, prj, zd, mx=d, mbn=bn_d.args(), gbn=bn_d, bpro=b.bwd_aff(bn_p, p, fold=True), aout=dp)
        b.mark_grads_ready([bn_p.gamma, bn_p.beta])
        if fz.trainable(prj):
            b.wgrad(d, prj, dp, b.arena.grad_of(prj.kernel), pro=bn_d.args(), lane=1)
        b.mark_grads_ready([prj.kernel])
        if not fz.before(bn_d.layer):
            b.mark_grads_ready([bn_d.gamma, bn_d.beta])
            return
        e, bn_in = blk["e"], blk["bn_in"]
        # depthwise BN backward: materialised once (the depthwise kernels re-read dZ ~4.5x; staging
        # the affine there re-reads the BN input as often and rebuilds the slot-summed A/B/C table
        # in every workgroup, measured slower than this pass: IDC_MBV2_DW_AFF=1 stages it, 2.424-2.429
        # vs 2.322-2.327 ms/step, round 4)
        if dw_aff and bn_d.mode == 1:
            dd, aff_d = zd, b.bwd_aff(bn_d, d, fold=True)
        else:
            dd, aff_d = b.nhwc(d.N, d.H, d.W, d.C), None
            b.bn_bwd_apply(zd, d, bn_d, dd, accumulate=False)
            b.mark_grads_ready([bn_d.gamma, bn_d.beta])
        # IDC_DW_FUSED_BWD=1: stride-1 blocks run the depthwise data and weight gradients as one
        # pass over dd and e (dwconv.hip dw_bwd3_fused_kernel)
        fused_dw = False
        if fz.before(dwl) or aff_d is not None:
            ze = b.nhwc(e.N, e.H, e.W, e.C)
            if fz.before(dwl):
                if os.environ.get("IDC_DW_FUSED_BWD", "0") == "1" and blk["stride"] == 1 and aff_d is None \
                        and fz.trainable(dwl):
                    fused_dw = b.dw_bwd_fused(e, dwl, dd, ze, b.arena.grad_of(dwl.depthwise_kernel),
                                              pads=blk["pads"], bn=bn_in)
                if not fused_dw:
                    b.dw_bwd_data(e, dwl, dd, ze, stride=blk["stride"], pads=blk["pads"], bn=bn_in, dyaff=aff_d)
        if aff_d is not None:
            b.mark_grads_ready([bn_d.gamma, bn_d.beta])
        if fz.trainable(dwl) and not fused_dw:
            b.dw_wgrad(e, dwl, dd, b.arena.grad_of(dwl.depthwise_kernel), stride=blk["stride"],
                       pads=blk["pads"], pro=bn_in.args(), lane=1,
                       dyaff=b.bwd_aff(bn_d, d) if aff_d is not None else None)
        b.mark_grads_ready([dwl.depthwise_kernel])
        if not fz.before(dwl):
            return
        if not fz.before(bn_in.layer):
            b.mark_grads_ready([bn_in.gamma, bn_in.beta])
            return
        ex = blk["ex"]
        de = b.nhwc(e.N, e.H, e.W, e.C)
        if ex is None or not fz.before(ex):
            b.bn_bwd_apply(ze, e, bn_in, de, accumulate=False)
            b.mark_grads_ready([bn_in.gamma, bn_in.beta])
            if ex is None:  # block 0: de is the gradient of the raw stem conv output
                if fz.trainable(conv1):
                    b.wgrad(x8, conv1, de, b.arena.grad_of(conv1.kernel), stride=(2, 2), pads=stem_pads,
                            cin_real=Cimg, lane=1)
                b.mark_grads_ready([conv1.kernel])
            else:
                if fz.trainable(ex):
                    b.wgrad(blk["h_in"], ex, de, b.arena.grad_of(ex.kernel), lane=1)
                b.mark_grads_ready([ex.kernel])
            return
        h_prev = blk["h_in"]
        aff_in = b.bwd_aff(bn_in, e, fold=True)
        gep = g_epilogue(blocks[blk["bid"] - 1])
        if blk["residual"]:
            # dL/dh_prev = G (identity shortcut) + expand^T de: accumulate into G in place
            b.dgrad(ze, ex, G, out_mode=nat.OUT_F32_ACC, bpro=aff_in, aout=de, **gep)
        else:
            G = b.nhwc(h_prev.N, h_prev.H, h_prev.W, h_prev.C, F32)
            b.dgrad(ze, ex, G, out_mode=nat.OUT_F32, bpro=aff_in, aout=de, **gep)
        b.mark_grads_ready([bn_in.gamma, bn_in.beta])
        if fz.trainable(ex):
            b.wgrad(h_prev, ex, de, b.arena.grad_of(ex.kernel), lane=1)
        b.mark_grads_ready([ex.kernel])
