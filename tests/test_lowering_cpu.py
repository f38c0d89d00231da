"""Lowering dry-runs on the CPU: every model family x freeze mode lowers to a plan whose every raw
device pointer lies inside a live tensor (no dangling or out-of-range argument), whose ctypes
argument structs match the native layouts, and whose backward stops where Keras freezing says."""
import ctypes as C

import pytest
import torch

from idc_models_amd.ops import _native as nat

pytestmark = pytest.mark.skipif(not nat.available(), reason="native extension not built")

CASES = [("densenet121", None), ("densenet121", 150), ("densenet121", "frozen"), ("vgg16", None),
         ("vgg16", 15), ("mobilenetv2", None), ("mobilenetv2", 100), ("mobilenetv2", "frozen"),
         ("tinycnn", None)]


def _lower(arch, ft, training, B=4):
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model
    from idc_models_amd.parallel import OneDeviceStrategy
    from idc_models_amd.runtime.builder import Builder
    from idc_models_amd.runtime.program import _lowering_for
    net = build_model(arch, None, 1, seed=0)
    base = getattr(net, "base", net)
    if ft == "frozen":
        base.trainable = False
    elif ft:
        for l in base.layers[:ft]:
            l.trainable = False
    m = Model(net, OneDeviceStrategy("cpu"))
    m.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="eager")
    b = Builder(net, m.arena, torch.device("cpu"), B, training)
    _lowering_for(net)(b, net, 1, torch.uint8)
    b.finalize_casts()
    b.finalize_moving()
    return m, net, b


STRUCTS = {nat.OP_CONV: nat.ConvArgs, nat.OP_WGRAD: nat.WgradArgs, nat.OP_BN_BWD_APPLY: nat.BnBwdApplyArgs,
           nat.OP_BN_BWD_REDUCE: nat.BnBwdReduceArgs, nat.OP_MAXPOOL: nat.PoolArgs,
           nat.OP_AVGPOOL: nat.PoolArgs, nat.OP_POOL_BWD: nat.PoolBwdArgs, nat.OP_HEAD_FWD: nat.HeadArgs,
           nat.OP_HEAD_BWD: nat.HeadBwdArgs, nat.OP_DW_FWD: nat.DwArgs, nat.OP_DW_BWD_DATA: nat.DwArgs,
           nat.OP_DW_WGRAD: nat.DwArgs, nat.OP_BN_APPLY: nat.BnArgs, nat.OP_MLP_FWD: nat.Mlp2Args,
           nat.OP_MLP_BWD: nat.Mlp2Args, nat.OP_DENSE_STAGE: nat.DenseStageArgs,
           nat.OP_DENSE_STAGE_BWD: nat.DenseBwdArgs, nat.OP_MB_CHAIN: nat.MbChainArgs,
           nat.OP_MB_INFER: nat.MbInferArgs, nat.OP_DENSE_INFER: nat.DenseInferArgs}


def _pointers(obj, out):
    for f in obj._fields_:
        v = getattr(obj, f[0])
        if isinstance(v, C.Structure):
            _pointers(v, out)
        elif f[1] is C.c_void_p and v:
            out.append((f[0], v))


@pytest.mark.parametrize("arch,ft", CASES)
def test_plan_pointers_are_live(arch, ft):
    m, net, b = _lower(arch, ft, True)
    ranges = [(t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()) for t in
              b.keep + [b.stats_arena, m.arena.data, m.arena.grad] + list(net.parameters()) +
              list(net.buffers())]
    bad = []
    for i, (seg, kind, raw, ints, floats, longs, ptrs, lane) in enumerate(b.ops):
        vals = [("ptr", p) for p in ptrs if p]
        if kind in STRUCTS:
            assert len(raw) == C.sizeof(STRUCTS[kind]), (i, kind)
            _pointers(STRUCTS[kind].from_buffer_copy(raw), vals)
        if kind == nat.OP_WGRAD_BATCH:  # the member table's argument structs
            tab = next(t for t in b.keep if t.data_ptr() == ptrs[0])
            n = ints[0]
            raw_tab = bytes(tab.cpu().numpy().tobytes())
            assert len(raw_tab) == n * C.sizeof(nat.WgBatchEntry), (i, n)
            for j in range(n):
                e = nat.WgBatchEntry.from_buffer_copy(raw_tab, j * C.sizeof(nat.WgBatchEntry))
                _pointers(e.a, vals)
        if kind == nat.OP_DENSE_STAGE:  # the per-layer descriptor table of a persistent stage
            tab = next(t for t in b.keep if t.data_ptr() == ptrs[0])
            n = ints[1]
            raw_tab = bytes(tab.cpu().numpy().tobytes())
            assert len(raw_tab) == n * C.sizeof(nat.DenseLayerDesc), (i, n)
            for j in range(n):
                e = nat.DenseLayerDesc.from_buffer_copy(raw_tab, j * C.sizeof(nat.DenseLayerDesc))
                assert e.cin % 32 == 0 and e.cin <= 1024, (i, j, e.cin)
                _pointers(e, vals)
        if kind == nat.OP_MB_CHAIN:  # the phase table of a persistent MobileNetV2 block chain
            tab = next(t for t in b.keep if t.data_ptr() == ptrs[0])
            n = ints[2]
            raw_tab = bytes(tab.cpu().numpy().tobytes())
            assert len(raw_tab) == n * C.sizeof(nat.MbPhaseDesc), (i, n)
            for j in range(n):
                e = nat.MbPhaseDesc.from_buffer_copy(raw_tab, j * C.sizeof(nat.MbPhaseDesc))
                assert nat.load().mb_phase_ok(nat.raw(e)), (i, j)
                _pointers(e, vals)
        for name, v in vals:
            if name == "hostflag":  # pinned host memory (persist.h FailSink)
                continue
            if not any(lo <= v < hi for lo, hi in ranges):
                bad.append((i, kind, name))
    assert not bad, bad[:10]


@pytest.mark.parametrize("arch,ft", CASES)
def test_forward_only_plan_has_no_backward(arch, ft):
    _, _, b = _lower(arch, ft, False)
    assert {op[0] for op in b.ops} == {"fwd"}
    assert not b.moving  # inference never updates moving statistics


def test_frozen_base_backward_is_head_only():
    _, _, b = _lower("mobilenetv2", "frozen", True)
    bwd = [op[1] for op in b.ops if op[0] == "bwd"]
    assert nat.OP_HEAD_BWD in bwd
    assert not any(k in (nat.OP_WGRAD, nat.OP_DW_WGRAD, nat.OP_CONV) for k in bwd)


@pytest.mark.parametrize("ft,training,fused", [("frozen", True, 17), (None, False, 17), (100, True, None),
                                               (None, True, 0)])
def test_mb_infer_lowering(monkeypatch, ft, training, fused):
    """Blocks no gradient reaches, with every BatchNorm on moving statistics, lower to ONE
    OP_MB_INFER each (csrc/kernels/mb_infer.hip): all 17 in evaluation and in the frozen-base phase
    (IDC_MB_INFER_MAX_CEXP lifted: by default only the blocks with <= 576 expanded channels), the
    frozen prefix only when fine-tuning from layer 100, none in full training; IDC_MB_INFER=0
    restores the three per-layer launches."""
    from idc_models_amd.runtime.lower_common import FreezeInfo
    _, _, bdef = _lower("mobilenetv2", ft, training)
    ndef = [op[1] for op in bdef.ops if op[0] == "fwd"].count(nat.OP_MB_INFER)
    assert ndef == (min(fused, 14) if fused is not None else ndef)
    monkeypatch.setenv("IDC_MB_INFER_MAX_CEXP", "4096")
    _, net, b = _lower("mobilenetv2", ft, training)
    kinds = [op[1] for op in b.ops if op[0] == "fwd"]
    n = kinds.count(nat.OP_MB_INFER)
    if fused is None:  # the blocks entirely inside the frozen prefix
        fz = FreezeInfo(net.base, True)
        names = ["expanded_conv_project_BN"] + [f"block_{i}_project_BN" for i in range(1, 17)]
        L = {l.name: l for l in net.base.layers}
        fused = sum(1 for nm in names if not fz.at_or_before(L[nm]))
        assert 0 < fused < 17
    assert n == fused
    if fused == 17:
        assert nat.OP_DW_FWD not in kinds
    for op in b.ops:
        if op[1] == nat.OP_MB_INFER:
            assert nat.load().mb_infer_smem(op[2]) > 0
    monkeypatch.setenv("IDC_MB_INFER", "0")
    _, _, b0 = _lower("mobilenetv2", ft, training)
    assert nat.OP_MB_INFER not in [op[1] for op in b0.ops]


@pytest.mark.parametrize("ft,training,n", [("frozen", True, 4), (None, False, 4), (150, True, 2), (None, True, 0)])
def test_dense_infer_lowering(monkeypatch, ft, training, n):
    """DenseNet stages whose BatchNorms (and the stage's consumer BatchNorm) all run on moving
    statistics lower to ONE OP_DENSE_INFER each (dense_infer.hip): with IDC_DENSE_INFER_LATE=1 all
    four stages in evaluation and the frozen base, stages 1-2 in the fine-tune phase (its cut falls
    in stage 3); never in full training.  By default stages 3-4 (M <= 2304 rows, batch 128 here)
    stay on the persistent launches; IDC_DENSE_INFER=0 restores the per-layer convs."""
    monkeypatch.setenv("IDC_DENSE_INFER_LATE", "1")
    _, _, b = _lower("densenet121", ft, training, B=128)
    kinds = [op[1] for op in b.ops if op[0] == "fwd"]
    assert kinds.count(nat.OP_DENSE_INFER) == n
    shapes = []
    for op in b.ops:
        if op[1] == nat.OP_DENSE_INFER:
            a = nat.DenseInferArgs.from_buffer_copy(op[2])
            shapes.append((a.H, a.L, a.ipg))
            assert nat.load().dense_infer_smem(op[2]) > 0
    assert shapes == [(13, 6, 1), (6, 12, 1), (3, 24, 1), (1, 16, 16)][:n]
    monkeypatch.delenv("IDC_DENSE_INFER_LATE")
    _, _, bl = _lower("densenet121", ft, training, B=128)
    assert [op[1] for op in bl.ops].count(nat.OP_DENSE_INFER) == min(n, 2)
    monkeypatch.setenv("IDC_DENSE_INFER", "0")
    _, _, b0 = _lower("densenet121", ft, training, B=128)
    assert nat.OP_DENSE_INFER not in [op[1] for op in b0.ops]


def test_dense_img_lowering(monkeypatch):
    """Training DenseNet-121 at 50x50: stages 1-2 (13x13 / 6x6, more rows than the persistent
    launches take) lower to ONE per-image launch each (OP_DENSE_STAGE with rows 2: dense_infer.hip
    dense_img_fwd) whose statistics (stage buffers, every t) have the single copy it reads; stage 3
    keeps the row-resident launch, stage 4 the work queue.  Opt-in (IDC_DENSE_IMG=1: measured slower
    than the per-layer convs); off, per-layer convs on slotted statistics.  Never in the fine-tune
    phase's frozen stages (dense_infer there)."""
    monkeypatch.setenv("IDC_DENSE_IMG", "1")

    def stages(b):
        return [(a.H, a.rows) for a in (nat.DenseStageArgs.from_buffer_copy(op[2]) for op in b.ops
                                        if op[1] == nat.OP_DENSE_STAGE)]
    _, _, b = _lower("densenet121", None, True, B=256)
    assert stages(b) == [(13, 2), (6, 2), (3, 1), (1, 0)]
    for op in b.ops:
        if op[1] == nat.OP_DENSE_STAGE and nat.DenseStageArgs.from_buffer_copy(op[2]).rows == 2:
            assert nat.load().dense_img_ok(op[2])
    _, _, bf = _lower("densenet121", 150, True, B=256)
    assert stages(bf) == [(3, 1), (1, 0)]
    monkeypatch.setenv("IDC_DENSE_IMG", "0")
    _, _, b0 = _lower("densenet121", None, True, B=256)
    assert stages(b0) == [(3, 1), (1, 0)]
    assert sum(1 for op in b0.ops if op[0] == "fwd") == sum(1 for op in b.ops if op[0] == "fwd") + 34


def test_dw_fused_backward_lowering(monkeypatch):
    """IDC_DW_FUSED_BWD=1: every stride-1 depthwise layer's data and weight gradients lower to ONE
    main-lane op (OP_DW_BWD_DATA, ints[0] 1) plus the partials' column sums on the side lane
    (OP_DW_WGRAD, ints[0] 2); the stride-2 layers keep their two kernels."""
    _, _, b0 = _lower("mobilenetv2", None, True)
    monkeypatch.setenv("IDC_DW_FUSED_BWD", "1")
    _, _, b1 = _lower("mobilenetv2", None, True)

    def ops(b, kind):
        return [op[3][0] if op[3] else 0 for op in b.ops if op[1] == kind]
    fused = [i for i in ops(b1, nat.OP_DW_BWD_DATA) if i == 1]
    sums = [(op[3][0] if op[3] else 0, op[7]) for op in b1.ops if op[1] == nat.OP_DW_WGRAD]
    assert len(fused) == 13
    assert sum(1 for i, lane in sums if i == 2 and lane == 1) == 13
    assert sum(1 for i, lane in sums if i != 2) == 4  # the stride-2 layers' own weight gradients
    assert len(ops(b0, nat.OP_DW_BWD_DATA)) == len(ops(b1, nat.OP_DW_BWD_DATA)) == 17
    assert not [i for i in ops(b0, nat.OP_DW_BWD_DATA) if i == 1]


def test_fine_tune_backward_stops_at_first_trainable_layer():
    m, net, b = _lower("mobilenetv2", 100, True)
    n_wgrad = sum(1 for op in b.ops if op[1] in (nat.OP_WGRAD, nat.OP_DW_WGRAD))
    trainable_convs = [l for l in net.base.layers[100:] if l.keras_class in ("Conv2D", "DepthwiseConv2D")]
    assert n_wgrad == len(trainable_convs)


@pytest.mark.parametrize("maxm", ["0", "2304", "9216", "100000000"])
def test_weight_gradients_are_on_the_side_lane(monkeypatch, maxm):
    monkeypatch.setenv("IDC_WG_BATCH_MAXM", maxm)
    _, net, b = _lower("densenet121", None, True, B=256)
    wg = [op for op in b.ops if op[1] == nat.OP_WGRAD]
    batches = [op for op in b.ops if op[1] == nat.OP_WGRAD_BATCH]
    # every weight gradient but the stem's (it consumes the last main-lane op's output, so it
    # runs on the main lane next to the side lane's backlog) is on the side lane, single or batched
    assert {op[7] for op in wg[:-1] + batches} == ({1} if b.side_lane else {0})
    assert wg[-1][7] == 0
    assert all(op[7] == 0 for op in b.ops if op[1] not in (nat.OP_WGRAD, nat.OP_WGRAD_BATCH))
    # every conv's weight gradient is computed exactly once
    convs = [l for l in net.base.layers if l.keras_class == "Conv2D"]
    assert len(wg) + sum(op[3][0] for op in batches) == len(convs)
    # stages 3-4 at bs 256 (M = 2304 / 256 pixels) batch by default: one launch per kernel shape
    if maxm == "2304":
        assert len(batches) == 4 and len(wg) == len(convs) - 80
    if maxm == "9216":  # the default: stages 2-4
        assert len(batches) == 6 and len(wg) == len(convs) - 104
    if maxm == "0":
        assert not batches


def test_struct_layouts_match_native():
    sizes = nat.load().struct_sizes()
    for name, st in nat._STRUCTS.items():
        assert C.sizeof(st) == sizes[name], name


def test_dense_stage_lowering(monkeypatch):
    """Late DenseNet stages lower to one OP_DENSE_STAGE each (per-layer convs otherwise); the
    deterministic mode and slotted statistics keep the per-layer convs.  (Stages 1-2's per-image
    launch is off here: test_dense_img_lowering.)"""
    monkeypatch.setenv("IDC_DENSE_IMG", "0")

    def count(env):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        _, _, b = _lower("densenet121", None, True, B=256)
        kinds = [k for (_, k, *_r) in b.ops]
        return kinds.count(nat.OP_DENSE_STAGE), kinds.count(nat.OP_CONV)
    n_on, conv_on = count({"IDC_DENSE_STAGE": "1", "IDC_DENSE_STAGE_MAXM": "2304"})
    n_off, conv_off = count({"IDC_DENSE_STAGE": "0"})
    assert (n_on, n_off) == (2, 0)
    assert conv_off - conv_on == 2 * (24 + 16)  # stages 3 and 4: two convs per dense layer
    monkeypatch.delenv("IDC_DENSE_STAGE_MAXM")
    assert count({"IDC_DENSE_STAGE": "1"})[0] == 2  # default: stages 3 and 4 (M <= 2304)
    assert count({"IDC_DENSE_STAGE_MAXM": "512"})[0] == 1  # stage 4 only
    monkeypatch.delenv("IDC_DENSE_STAGE_MAXM")
    assert count({"IDC_DENSE_STAGE": "1", "IDC_DETERMINISTIC": "1"})[0] == 0
    monkeypatch.delenv("IDC_DETERMINISTIC")
    assert count({"IDC_STAT_SLOTS": "1"})[0] == 2  # stage 3/4 rows (<= 4096) keep one copy


def test_dense_stage_bwd_lowering(monkeypatch):
    """The smallest stages' dense-layer data gradients lower to one OP_DENSE_STAGE_BWD each (by
    default stage 4 at bs 256, M <= 256; with IDC_DENSE_STAGE_BWD_MAXM=2304 stages 3 and 4; with
    fine_tune_at=150 stage 3 is partly frozen and keeps the per-layer dgrads); the deterministic
    mode and IDC_DENSE_STAGE_BWD=0 keep the per-layer dgrads everywhere."""
    def count(ft=None, **env):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        _, _, b = _lower("densenet121", ft, True, B=256)
        kinds = [k for (_, k, *_r) in b.ops]
        for k in env:
            monkeypatch.delenv(k)
        return kinds.count(nat.OP_DENSE_STAGE_BWD), kinds.count(nat.OP_CONV)
    n_def, conv_def = count()
    n_on, conv_on = count(IDC_DENSE_STAGE_BWD_MAXM="2304")
    n_off, conv_off = count(IDC_DENSE_STAGE_BWD="0")
    assert (n_def, n_on, n_off) == (1, 2, 0)
    assert conv_off - conv_def == 2 * 16  # two dgrads per dense layer of stage 4
    assert conv_off - conv_on == 2 * (24 + 16)  # ... and of stage 3
    assert count(150, IDC_DENSE_STAGE_BWD_MAXM="2304")[0] == 1
    assert count(IDC_DETERMINISTIC="1")[0] == 0
    # stage 2 (6x6 maps) fits the launch too when its statistics are single copies (the launch
    # needs them; by default its 9,216-row reductions keep 4 slot copies)
    assert count(IDC_DENSE_STAGE_BWD_MAXM="9216", IDC_STAT_SLOTS="0")[0] == 3
    assert count(IDC_DENSE_STAGE_BWD_MAXM="9216")[0] == 2


def test_mb_chain_lowering(monkeypatch):
    """MobileNetV2's blocks lower to ONE OP_MB_CHAIN with IDC_MB_CHAIN=1 (expand / depthwise /
    project of every block from IDC_MB_CHAIN_FROM on); the default keeps the per-layer ops.
    Tickets are contiguous per phase, every phase depends on an earlier one, and every conv phase's
    output BatchNorm gets a table the next phase reads."""
    def lower(**env):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        _, _, b = _lower("mobilenetv2", None, True, B=256)
        for k in env:
            monkeypatch.delenv(k)
        return b

    def kinds(b):
        return [k for (_, k, *_r) in b.ops]

    on, off = lower(IDC_MB_CHAIN="1"), lower(IDC_MB_CHAIN="0")
    assert kinds(lower()).count(nat.OP_MB_CHAIN) == 0  # off by default (runtime/mb_chain.py)
    k_on, k_off = kinds(on), kinds(off)
    assert k_on.count(nat.OP_MB_CHAIN) == 1 and k_off.count(nat.OP_MB_CHAIN) == 0
    fwd_on = [op[1] for op in on.ops if op[0] == "fwd"]
    fwd_off = [op[1] for op in off.ops if op[0] == "fwd"]
    # 17 blocks: 16 expand + 17 depthwise + 17 project convs leave the forward
    assert fwd_off.count(nat.OP_DW_FWD) - fwd_on.count(nat.OP_DW_FWD) == 17
    assert fwd_off.count(nat.OP_CONV) - fwd_on.count(nat.OP_CONV) == 33
    # the backward is unchanged
    assert [op[1] for op in on.ops if op[0] == "bwd"] == [op[1] for op in off.ops if op[0] == "bwd"]
    op = next(o for o in on.ops if o[1] == nat.OP_MB_CHAIN)
    tab = next(t for t in on.keep if t.data_ptr() == op[6][0])
    raw = bytes(tab.cpu().numpy().tobytes())
    n = op[3][2]
    descs = [nat.MbPhaseDesc.from_buffer_copy(raw, j * C.sizeof(nat.MbPhaseDesc)) for j in range(n)]
    assert sum(d.kind == nat.MB_TAB for d in descs) == 1  # the stem BatchNorm
    first = 0
    for j, d in enumerate(descs):
        assert d.first == first and d.dep < j
        first += d.tiles
        if d.kind != nat.MB_TAB:
            assert d.bn_mode == 1 and d.slots >= 1 and d.tab_out >= 0
    a = nat.MbChainArgs.from_buffer_copy(op[2])
    assert a.ntickets == first and a.nphases == n
    part = lower(IDC_MB_CHAIN="1", IDC_MB_CHAIN_FROM="10")
    d10 = [op for op in part.ops if op[1] == nat.OP_MB_CHAIN]
    assert len(d10) == 1 and d10[0][3][2] == 1 + 3 * 7  # TAB of block 9's project BN + blocks 10-16


def test_stat_slot_copies_default_and_cap(monkeypatch):
    """Large-map reductions keep statistics slot copies by default, at most 4 (the consumers'
    batched table loads take <= 4: builder.stat_slots_for); IDC_STAT_SLOTS_CAP moves the cap and
    IDC_STAT_SLOTS=0 keeps one copy everywhere.  (With stages 1-2 as per-image launches their
    statistics have the one copy those read: test_dense_img_lowering; off here.)"""
    from idc_models_amd.runtime.builder import stat_slots_for
    monkeypatch.setenv("IDC_DENSE_IMG", "0")
    monkeypatch.delenv("IDC_STAT_SLOTS_CAP", raising=False)
    assert [stat_slots_for(r) for r in (256, 2304, 4096, 9216, 43264, 160000)] == [1, 1, 1, 4, 4, 4]
    monkeypatch.setenv("IDC_STAT_SLOTS_CAP", "16")
    assert stat_slots_for(43264) == 16 and stat_slots_for(9216) == 4
    monkeypatch.delenv("IDC_STAT_SLOTS_CAP")

    def slots(**env):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        _, _, b = _lower("densenet121", None, True, B=256)
        for k in env:
            monkeypatch.delenv(k)
        return sorted({s.slots for s in b.all_stats}), sum(1 for s in b.all_stats if s.slots > 1)
    (kinds, n_on), (kinds_off, n_off) = slots(), slots(IDC_STAT_SLOTS="0")
    assert kinds == [1, 4]  # stages 3-4 one copy; stages 1-2, the stem and the transitions 4
    assert n_off == 1 and n_on > 1  # off: only the stem conv's reduction (always slotted) keeps copies


def _grad_writes(b, arena):
    """{op index: arena offsets (floats) of the gradient tensors the op's operands point at}."""
    lo, hi = arena.grad.data_ptr(), arena.grad.data_ptr() + 4 * arena.numel
    out = {}
    for i, (seg, kind, raw, ints, floats, longs, ptrs, lane) in enumerate(b.ops):
        if seg != "bwd" or kind == nat.OP_MEMSET:
            continue
        vals = [("ptr", p) for p in ptrs if p]
        if kind in STRUCTS:
            _pointers(STRUCTS[kind].from_buffer_copy(raw), vals)
        tabs = {nat.OP_WGRAD_BATCH: (0, 0, nat.WgBatchEntry), nat.OP_DENSE_STAGE_BWD: (0, 1, nat.DenseBwdLayerDesc)}
        if kind in tabs:
            ps, ns, typ = tabs[kind]
            tab = next(t for t in b.keep if t.data_ptr() == ptrs[ps])
            raw_tab = bytes(tab.cpu().numpy().tobytes())
            for j in range(ints[ns]):
                e = typ.from_buffer_copy(raw_tab, j * C.sizeof(typ))
                _pointers(e.a if kind == nat.OP_WGRAD_BATCH else e, vals)
        offs = [(v - lo) // 4 for _, v in vals if lo <= v < hi]
        if offs:
            out[i] = offs
    return out


@pytest.mark.parametrize("arch,ft", [("vgg16", 15), ("vgg16", None), ("densenet121", 150),
                                     ("densenet121", None), ("mobilenetv2", 100)])
def test_allreduce_placement_world4(arch, ft):
    """Data parallelism at world 4 (``dist_model_tf_vgg.py:115-117,141-151``): every gradient bucket's
    all-reduce is placed after every backward op that writes into the bucket, exactly once, inside
    the backward; with the phase-2 cuts (VGG16 15, DenseNet 150) the buckets start mid-network."""
    from idc_models_amd.parallel.buckets import DEFAULT_BUCKET_BYTES, GradBucketer
    from idc_models_amd.runtime.program import place_buckets
    m, net, b = _lower(arch, ft, True, B=64)
    gb = GradBucketer(m.arena, DEFAULT_BUCKET_BYTES // 4)  # several buckets per model
    buckets = [(bk.param_ids, bk.start, bk.end) for bk in gb.buckets]
    assert len(buckets) >= 2
    placed = place_buckets(b.ops, b.bwd_marks, buckets)
    where = {}
    for i, lst in placed.items():
        for s0, s1 in lst:
            assert (s0, s1) not in where, "bucket placed twice"
            where[(s0, s1)] = i
    assert sorted(where) == sorted((s0, s1) for _, s0, s1 in buckets)
    bwd = [i for i, op in enumerate(b.ops) if op[0] == "bwd"]
    writes = _grad_writes(b, m.arena)
    assert writes  # the backward writes gradients through pointers we can see
    covered = set()
    for (s0, s1), at in where.items():
        assert bwd[0] < at <= bwd[-1] + 1, (s0, s1, at)
        for i, offs in writes.items():
            if any(s0 <= o < s1 for o in offs):
                assert i < at, f"op {i} writes into bucket [{s0},{s1}) all-reduced before op {at}"
                covered.add((s0, s1))
    assert covered == set(where)  # every bucket has a producer before its all-reduce
    # overlap: at least one bucket is released before the backward ends (mid-network start)
    assert min(where.values()) <= bwd[-1], where


def test_uneven_share_weight_scales_the_gradient_seed():
    """a rank's weight in an unevenly split global batch scales its loss head's
    gradient seed (before the all-reduce), not the optimizer's factor after it."""
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model
    from idc_models_amd.parallel import OneDeviceStrategy
    from idc_models_amd.runtime.builder import Builder
    from idc_models_amd.runtime.program import _lowering_for
    for arch, kind, typ in (("vgg16", nat.OP_HEAD_FWD, nat.HeadArgs), ("tinycnn", nat.OP_MLP_FWD, nat.Mlp2Args)):
        net = build_model(arch, None, 1, seed=0)
        m = Model(net, OneDeviceStrategy("cpu"))
        m.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="eager")
        b = Builder(net, m.arena, torch.device("cpu"), 6, True)
        b.grad_weight = 1.5
        _lowering_for(net)(b, net, 1, torch.uint8)
        a = typ.from_buffer_copy(next(op[2] for op in b.ops if op[1] == kind))
        assert a.loss_scale == pytest.approx(1 / 6)
        assert a.dl_scale == pytest.approx(1.5 / 6)


def test_persistent_launches_need_a_guarded_update():
    """persistent launches only where a give-up can skip the update on every
    replica: the fused RMSprop (not a host optimizer) and, under data parallelism, the native
    communicator's guard all-reduce (not the torch bucketer or central storage)."""
    from types import SimpleNamespace as NS
    from idc_models_amd.engine import SGD, RMSprop
    from idc_models_amd.runtime.program import persistent_allowed

    def model(opt, active=False, native=None, central=False):
        st = NS(active=active, native_comm=native, central_storage=central)
        return NS(optimizer=opt, strategy=st, arena=NS(params=[1]))
    assert persistent_allowed(model(RMSprop(1e-3)), True)
    assert persistent_allowed(model(RMSprop(1e-3), active=True, native=object()), True)
    assert not persistent_allowed(model(SGD(0.1)), True)
    assert not persistent_allowed(model(RMSprop(1e-3, momentum=0.9)), True)
    assert not persistent_allowed(model(RMSprop(1e-3), active=True, native=None), True)
    assert not persistent_allowed(model(RMSprop(1e-3), active=True, native=object(), central=True), True)
    assert persistent_allowed(model(SGD(0.1)), False)  # evaluation programs
