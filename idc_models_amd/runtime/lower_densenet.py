"""DenseNet-121/169/201 lowering (the north-star benchmark model).

MI355X-specific structure:

* **concat-free stage buffers** — each dense stage owns ONE NHWC buffer holding all of its
  channels; every 3x3 conv writes its 32 new channels into its slice in place,
  every 1x1 conv reads the ``[0:Cin)`` prefix with the buffer's pixel stride;
* **statistics computed once per channel** — a channel's batch mean/var is identical for every
  later ``_0_bn`` that normalises it (SURVEY §2.4.3 "exact shortcut"), so the producer's epilogue
  reduces [sum|sumsq] ONCE into the stage's stats row and each consumer applies its own gamma/beta
  in its operand prologue;
* **transition = pool first** — ``BN->ReLU->conv1x1->avgpool`` is computed as
  ``BN->ReLU->avgpool->conv1x1`` (a 1x1 conv commutes with 2x2 averaging): 4x fewer MFMA FLOPs;
* **gradient of the concat buffer** — one fp32 gradient buffer per stage; the transition (or the
  head) STORES it, every dense layer's dgrad cv1 epilogue ACCUMULATES into its channel prefix,
  so the slice a layer reads is complete when backward reaches it and no zeroing pass is needed;
* **no BatchNorm-backward passes** — each BN backward is applied by its consumers while they stage
  their operands (the backward chain below), 2 main-lane kernels per dense layer.
"""
from __future__ import annotations

import os

import torch

from ..ops import _native as nat
from .builder import BF16, F32, BNRef, Builder, Tensor4
from .lower_common import RELU, FreezeInfo, HeadIO, emit_head, emit_head_bwd, emit_input


def lower_densenet(b: Builder, net, U: int, input_dtype):
    base, dense = net.base, net.head
    B = b.B
    training = b.training
    fz = FreezeInfo(base, training)
    L = {l.name: l for l in base.layers}
    H, W, Cimg = base.input_shape
    io = HeadIO(b, U)

    # ---------------------------------------------------------------- forward
    b.segment = "fwd"
    if training:
        b.memset(b.stats_arena)  # size patched at finalize
    xin, x8 = emit_input(b, H, W, Cimg, input_dtype)
    conv1, bn1l = L["conv1/conv"], L["conv1/bn"]
    H1, W1 = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
    ys = b.nhwc(B, H1, W1, 64)
    # (slot copies: the stem conv runs ~1k workgroups, each adding every channel's sums)
    ss = b.stats(64, B * H1 * W1, slotted=True) if training else None
    b.conv(x8, conv1, ys, stride=(2, 2), pads=(3, 3), stats=ss)
    bn_stem = BNRef(bn1l, b, ss, RELU)
    b.add_moving(bn_stem)
    Hs, Ws = (H1 + 2 - 3) // 2 + 1, (W1 + 2 - 3) // 2 + 1

    # Late stages (M <= IDC_DENSE_STAGE_MAXM pixels; default 2304: stages 3-4 at bs 256, stages 3-4
    # of a bs-32 federated client) run all their dense layers as ONE persistent work-queue launch
    # each (builder.dense_stage, dense_stage.hip) instead of 2 launch-latency-bound convs per layer.
    # DenseNet-121 bs 256 on 1x MI355X (bench.py, repeated A/B): stages 3+4 in-kernel 4.27-4.29
    # ms/step, stage 4 only 4.31, per-layer 4.35-4.41; stage 2 (9,216 rows) measured slower
    stage_maxm = int(os.environ.get("IDC_DENSE_STAGE_MAXM", "2304"))
    # IDC_IMG_SLOTS=1: stages whose dense layers run per-layer convs on >= 8192 rows keep their batch
    # statistics in slot copies, so the image-resident 3x3 kernels (conv_img.hip), whose workgroups
    # all finish together, add <= 16 times per address instead of folding in-kernel; measured
    # neutral (3.69-3.73 vs 3.66-3.69 ms/step, bench.py A/B round 5), so off by default.
    img_slots = os.environ.get("IDC_IMG_SLOTS", "0") == "1"

    bwd_maxm_env = int(os.environ.get("IDC_DENSE_STAGE_BWD_MAXM", "256"))

    def slotted_stage(rows):  # (never a stage a persistent launch takes: those need single copies)
        return img_slots and rows > max(stage_maxm, bwd_maxm_env) and rows >= 8192

    stages = []
    c0 = 64
    nblocks = base.blocks
    ctot = c0 + 32 * nblocks[0]
    buf = b.nhwc(B, Hs, Ws, ctot)
    sbuf = b.stats(ctot, B * Hs * Ws, slotted=slotted_stage(B * Hs * Ws),
                   single=b.dense_img_candidate(B * Hs * Ws, Hs, Ws)) if training else None
    argmax = b.alloc((B * Hs * Ws * 64,), torch.uint8)
    b.pool(ys, buf.slice(0, 64), k=3, s=2, pt=1, pl=1, pro=bn_stem.args(), is_max=True,
           argmax=argmax, stats=sbuf, stats_off=0)

    for si, nb in enumerate(nblocks):
        st = {"buf": buf, "stats": sbuf, "c0": c0, "ctot": ctot, "H": Hs, "W": Ws, "layers": []}
        M = B * Hs * Ws
        for li in range(nb):
            name = f"conv{si + 2}_block{li + 1}"
            cin = c0 + 32 * li
            bn1 = BNRef(L[name + "_0_bn"], b, sbuf, RELU)
            cv1, bn2l, cv2 = L[name + "_1_conv"], L[name + "_1_bn"], L[name + "_2_conv"]
            t = b.nhwc(B, Hs, Ws, 128)
            stt = b.stats(128, M, single=b.dense_img_candidate(M, Hs, Ws)) if training else None
            bn2 = BNRef(bn2l, b, stt, RELU)
            st["layers"].append({"cin": cin, "bn1": bn1, "cv1": cv1, "bn2": bn2, "cv2": cv2, "t": t, "stt": stt})
        # a stage no statistics are needed from (every BatchNorm reading it on moving statistics:
        # evaluation, a frozen base, the frozen stages of the fine-tune phase): ONE dense_infer
        # launch for the whole block (dense_infer.hip).  The stages the persistent launches take
        # (M <= IDC_DENSE_STAGE_MAXM: stages 3-4 at 50x50) stay on them unless IDC_DENSE_INFER_LATE=1:
        # measured 435 us (stage 3) and 208 us (stage 4) as dense_infer against 260 / 136 us for the
        # row-resident / work-queue launches (frozen phase 1.23 vs 0.98-1.02 ms/step)
        consumer = L[f"pool{si + 2}_bn"] if si < len(nblocks) - 1 else L["bn"]
        consumer_infer = not (b.training and consumer.trainable)
        late_ok = M > stage_maxm or os.environ.get("IDC_DENSE_INFER_LATE", "0") == "1"
        if late_ok and consumer_infer and b.dense_infer(buf, st["layers"], RELU):
            st["infer"] = True
        elif M <= stage_maxm and b.dense_stage_ok(sbuf, st["layers"], Hs, Ws):
            b.dense_stage(buf, sbuf, st["layers"], RELU)
        elif M > stage_maxm and b.dense_img_ok(buf, sbuf, st["layers"]):
            # training stages of large maps (1-2 at 50x50): one per-image launch, BatchNorm
            # statistics through two barriers per layer (dense_infer.hip dense_img_fwd)
            b.dense_stage(buf, sbuf, st["layers"], RELU, img=True)
        else:
            for lay in st["layers"]:
                cin, t = lay["cin"], lay["t"]
                b.conv(buf.slice(0, cin), lay["cv1"], t, pro=lay["bn1"].args(), stats=lay["stt"])
                b.conv(t, lay["cv2"], buf.slice(cin, 32), pads=(1, 1), pro=lay["bn2"].args(), stats=sbuf,
                       stats_off=cin)
        for lay in st["layers"]:
            b.add_moving(lay["bn1"])
            b.add_moving(lay["bn2"])
        if si < len(nblocks) - 1:
            bnt = BNRef(L[f"pool{si + 2}_bn"], b, sbuf, RELU)
            cvt = L[f"pool{si + 2}_conv"]
            Hn, Wn = Hs // 2, Ws // 2
            p = b.nhwc(B, Hn, Wn, ctot)
            b.pool(buf, p, k=2, s=2, pro=bnt.args(), is_max=False)
            c0n = ctot // 2
            ctotn = c0n + 32 * nblocks[si + 1]
            bufn = b.nhwc(B, Hn, Wn, ctotn)
            sbufn = b.stats(ctotn, B * Hn * Wn, slotted=slotted_stage(B * Hn * Wn),
                            single=b.dense_img_candidate(B * Hn * Wn, Hn, Wn)) if training else None
            b.conv(p, cvt, bufn.slice(0, c0n), stats=sbufn, stats_off=0)
            b.add_moving(bnt)
            st["trans"] = {"bn": bnt, "conv": cvt, "p": p}
            stages.append(st)
            buf, sbuf, c0, ctot, Hs, Ws = bufn, sbufn, c0n, ctotn, Hn, Wn
        else:
            stages.append(st)

    bnf = BNRef(L["bn"], b, sbuf, RELU)
    b.add_moving(bnf)
    emit_head(b, buf, bnf.args(), dense, U, io, training)
    if training:
        b.emit("MOVING")

    b.xin, b.io = xin, io
    b.debug = {"ys": ys, "ss": ss, "stages": stages, "x8": x8}
    if not training:
        return

    # ---------------------------------------------------------------- backward
    # Every BatchNorm backward dX = A*dZ + B*X + C (csrc/kernels/common.h BwdAff) is applied by its
    # CONSUMERS, never materialised by a pass of its own:
    #   * bn2 (inside a dense layer): dgrad cv1 and wgrad cv1 stage A*z2 + B*t + C from the
    #     per-layer z2 (= dZ of bn2) and the saved raw t;
    #   * bn1 / transition / final BatchNorms feed the stage's fp32 concat-gradient buffer: their
    #     producer ADDS A*dZ into it, and the B*x + C part of exactly ONE BatchNorm — ``pend``, the
    #     last one processed — is outstanding at any time: the next dgrad cv1 epilogue folds it
    #     into every channel it updates, and the consumers of the other channels (dgrad/wgrad cv2
    #     of the next layer, the transition conv, the stem pool) apply it while staging.
    #   The first main-lane consumer of a BatchNorm also folds its statistics-slot copies into
    #   d beta / d gamma (BwdAff fold), so no standalone BN-backward kernel runs at all.
    b.segment = "bwd"
    b.memset(b.arena.grad)
    last = stages[-1]
    need_base = fz.at_or_before(L["bn"])
    dA = emit_head_bwd(b, last["buf"], dense, U, io, need_dA=need_base)
    if not need_base:
        return
    lb = last["buf"]
    if not fz.before(L["bn"]):
        zf = b.nhwc(lb.N, lb.H, lb.W, last["ctot"])
        b.bn_bwd_reduce(dA, lb, bnf, zf)
        b.mark_grads_ready([bnf.gamma, bnf.beta])
        return
    dbuf = b.nhwc(lb.N, last["H"], last["W"], last["ctot"], F32)
    b.bn_bwd_reduce(dA, lb, bnf, dbuf)  # fp32 dbuf = A_f * dZ_f
    pend = bnf

    def pend_params():
        return [pend.gamma, pend.beta]

    # Late stages (M <= IDC_WG_BATCH_MAXM pixels; default 9216: stages 2-4 at bs 256) batch their weight
    # gradients: each dense layer's wgrads are launch-latency bound (10-20 us for < 1 us of MFMA
    # work, 2 side-lane launches + a fork per layer), and their operands (the per-layer staged
    # gradients dO16 / dt, the forward buffers) are final once the stage's dgrad chain has run, so
    # the stage issues them as one OP_WGRAD_BATCH per kernel shape that fills the GPU beside the
    # previous stage's data gradients (builder.flush_wgrad_batch).
    batch_maxm = int(os.environ.get("IDC_WG_BATCH_MAXM", "9216"))
    # The smallest stages (M <= IDC_DENSE_STAGE_BWD_MAXM pixels, default 256: stage 4 at bs 256) run
    # the data gradients of all their dense layers as ONE persistent launch (builder.dense_stage_bwd,
    # dense_stage_bwd.hip); it hands the stage input's final gradient (bf16) to the transition
    # (the row-resident form, IDC_DS_ROWS_BWD=1, runs stage 3 as well: M = 2,304)
    from .builder import rows_bwd_enabled
    bwd_maxm = int(os.environ.get("IDC_DENSE_STAGE_BWD_MAXM", "2304" if rows_bwd_enabled() else "256"))
    for si in range(len(stages) - 1, -1, -1):
        st = stages[si]
        buf = st["buf"]
        N, Hs, Ws = buf.N, st["H"], st["W"]
        wb = N * Hs * Ws <= batch_maxm
        dx16 = None
        lays = st["layers"]
        if N * Hs * Ws <= bwd_maxm and fz.before(lays[0]["bn1"].layer) and \
                all(fz.trainable(lay[k]) for lay in lays for k in ("cv1", "cv2")) and \
                all(fz.trainable(lay[k].layer) for lay in lays for k in ("bn1", "bn2")) and \
                b.dense_stage_bwd_ok(buf, lays, pend):
            for lay in lays:
                lay["dO16"] = b.nhwc(N, Hs, Ws, 32)
                lay["dt"] = b.nhwc(N, Hs, Ws, 128)
            dx16 = b.dense_stage_bwd(buf, st["stats"], lays, pend, dbuf, RELU)
            for lay in lays:
                b.wgrad(lay["t"], lay["cv2"], lay["dO16"], b.arena.grad_of(lay["cv2"].kernel), pads=(1, 1),
                        pro=lay["bn2"].args(), lane=1, batch=wb)
                b.wgrad(buf.slice(0, lay["cin"]), lay["cv1"], lay["dt"], b.arena.grad_of(lay["cv1"].kernel),
                        pro=lay["bn1"].args(), lane=1, batch=wb)
                b.mark_grads_ready([lay["cv2"].kernel, lay["cv1"].kernel, lay["bn2"].gamma, lay["bn2"].beta,
                                    lay["bn1"].gamma, lay["bn1"].beta])
            b.mark_grads_ready(pend_params())
            pend = lays[0]["bn1"]
        z2 = b.nhwc(N, Hs, Ws, 128) if dx16 is None else None  # dZ of bn2, consumed by the next dgrad
        for lay in (reversed(st["layers"]) if dx16 is None else ()):
            cin, bn1, cv1, bn2, cv2, t = lay["cin"], lay["bn1"], lay["cv1"], lay["bn2"], lay["cv2"], lay["t"]
            dO = dbuf.slice(cin, 32)
            xO = buf.slice(cin, 32)
            # Weight gradients run on the side lane and read plain bf16 gradients that the dgrads
            # store while staging them (dO16, dt: per layer, never overwritten later); where the
            # backward stops at a layer (no dgrad), the wgrad applies the pending affine itself.
            if not fz.before(cv2):
                if fz.trainable(cv2):
                    b.wgrad(t, cv2, dO, b.arena.grad_of(cv2.kernel), pads=(1, 1), pro=bn2.args(), lane=1,
                            gpro=b.bwd_aff(pend, xO, c0=cin, unit_alpha=True))
                b.mark_grads_ready([cv2.kernel] + pend_params())
                return
            dO16 = b.nhwc(N, Hs, Ws, 32)
            b.dgrad(dO, cv2, z2, pads=(1, 1), mx=t, mbn=bn2.args(), gbn=bn2,
                    bpro=b.bwd_aff(pend, xO, c0=cin, unit_alpha=True, fold=True), aout=dO16,
                    slotted=slotted_stage(N * Hs * Ws))
            if fz.trainable(cv2):
                b.wgrad(t, cv2, dO16, b.arena.grad_of(cv2.kernel), pads=(1, 1), pro=bn2.args(), lane=1,
                        batch=wb)
            if not fz.before(bn2.layer):
                b.mark_grads_ready([cv2.kernel, bn2.gamma, bn2.beta] + pend_params())
                return
            ready = [cv2.kernel, cv1.kernel, bn2.gamma, bn2.beta] + pend_params()
            if not fz.before(cv1):
                if fz.trainable(cv1):
                    b.wgrad(buf.slice(0, cin), cv1, z2, b.arena.grad_of(cv1.kernel), pro=bn1.args(), lane=1,
                            gpro=b.bwd_aff(bn2, t))
                b.mark_grads_ready(ready)
                return
            # concat gradient [0, cin) += A1*dZ1 + (pend's B*x + C); reductions of bn1
            dt = b.nhwc(N, Hs, Ws, 128)
            b.dgrad(z2, cv1, dbuf.slice(0, cin), mx=buf.slice(0, cin), mbn=bn1.args(), gbn=bn1,
                    bpro=b.bwd_aff(bn2, t, fold=True),
                    bepi=b.bwd_aff(pend, buf.slice(0, cin), unit_alpha=True), aout=dt)
            if fz.trainable(cv1):
                b.wgrad(buf.slice(0, cin), cv1, dt, b.arena.grad_of(cv1.kernel), pro=bn1.args(), lane=1,
                        batch=wb)
            b.mark_grads_ready(ready)
            pend = bn1
            if not fz.before(bn1.layer):
                b.mark_grads_ready(pend_params())
                return
        b.flush_wgrad_batch()
        if si == 0:
            break
        # transition of the previous stage (wrote this stage's channels [0:c0)), through pend
        prev = stages[si - 1]
        tr = prev["trans"]
        bnt, cvt, p = tr["bn"], tr["conv"], tr["p"]
        c0 = st["c0"]
        dO = dbuf.slice(0, c0)
        xO = buf.slice(0, c0)
        if not fz.before(cvt):
            if fz.trainable(cvt) and dx16 is not None:
                b.wgrad(p, cvt, dx16, b.arena.grad_of(cvt.kernel), lane=1)
            elif fz.trainable(cvt):
                b.wgrad(p, cvt, dO, b.arena.grad_of(cvt.kernel), lane=1,
                        gpro=b.bwd_aff(pend, xO, unit_alpha=True))
            b.mark_grads_ready([cvt.kernel] + pend_params())
            return
        dp = b.nhwc(p.N, p.H, p.W, p.C)
        if dx16 is not None:
            # the persistent backward finished these channels' gradient (every pending affine included)
            dO16 = dx16
            b.dgrad(dO16, cvt, dp)
        else:
            dO16 = b.nhwc(N, Hs, Ws, c0)
            b.dgrad(dO, cvt, dp, bpro=b.bwd_aff(pend, xO, unit_alpha=True, fold=True), aout=dO16)
        if fz.trainable(cvt):
            b.wgrad(p, cvt, dO16, b.arena.grad_of(cvt.kernel), lane=1)
        b.mark_grads_ready(pend_params())
        pbuf = prev["buf"]
        dbuf = b.nhwc(pbuf.N, prev["H"], prev["W"], prev["ctot"], F32)
        b.pool_bwd(dp, dbuf, k=2, s=2, is_max=False, x=pbuf, bn=bnt)  # fp32: A_t * dZ_t
        b.mark_grads_ready([cvt.kernel])
        pend = bnt
        if not fz.before(bnt.layer):
            b.mark_grads_ready(pend_params())
            return

    # stem: max-pool backward through BN+ReLU of conv1 (dy = concat gradient + pend), conv1 wgrad
    if not fz.at_or_before(bn1l):
        b.mark_grads_ready(pend_params())
        return
    st0 = stages[0]
    zs = b.nhwc(B, H1, W1, 64)
    if dx16 is not None:  # stage 1 ran the persistent backward: its input gradient is final
        b.pool_bwd(dx16, zs, k=3, s=2, pt=1, pl=1, is_max=True, argmax=argmax, x=ys, bn=bn_stem)
    else:
        b.pool_bwd(dbuf.slice(0, 64), zs, k=3, s=2, pt=1, pl=1, is_max=True, argmax=argmax, x=ys,
                   bn=bn_stem, dyaff=b.bwd_aff(pend, st0["buf"].slice(0, 64), unit_alpha=True, fold=True))
    if fz.trainable(conv1):
        # the stem wgrad consumes the LAST main-lane op's output, so it can never overlap the
        # dgrad chain; on the main lane it starts at once and overlaps the side lane's backlog of
        # stage-1 weight gradients instead of queueing behind it (IDC_STEM_SIDE=1: side lane)
        stem_lane = 1 if os.environ.get("IDC_STEM_SIDE", "0") == "1" else 0
        b.wgrad(x8, conv1, zs, b.arena.grad_of(conv1.kernel), stride=(2, 2), pads=(3, 3),
                cin_real=Cimg, lane=stem_lane, gpro=b.bwd_aff(bn_stem, ys))
    b.mark_grads_ready([conv1.kernel, bn_stem.gamma, bn_stem.beta] + pend_params())
