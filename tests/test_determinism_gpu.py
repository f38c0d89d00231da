"""IDC_DETERMINISTIC=1 (SURVEY §5 race detection / reproducibility): every float reduction of the
fused step has a fixed order — per-workgroup private statistic slots collapsed in order, per-slice
weight-gradient partials reduced in order, no LDS float atomics, fixed tiles — so the same program
on the same inputs gives the same bits.  Checked against the eager fp32 reference as well, so the
deterministic kernels are also correct ones.  Reference: ``dist_model_tf_dense.py:131-144``."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _model(arch, seed=0):
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model
    net = build_model(arch, None, num_outputs=1, seed=seed)
    ref = copy.deepcopy(net).to(DEV)
    m = Model(net, device=DEV)
    m.compile(RMSprop(1e-3), "binary_crossentropy", [], backend="fused")
    return m, ref


@pytest.mark.miopen_ref
@pytest.mark.parametrize("arch,B", [("densenet121", 64), ("vgg16", 32)])
def test_deterministic_mode_is_bitwise_reproducible(monkeypatch, arch, B):
    monkeypatch.setenv("IDC_DETERMINISTIC", "1")
    g = torch.Generator().manual_seed(3)
    H = 50
    x = torch.randint(0, 256, (B, H, H, 3), generator=g, dtype=torch.uint8)
    y = torch.randint(0, 2, (B,), generator=g)
    m1, ref = _model(arch)
    p = m1.impl._prog(B, True, torch.uint8)
    grads = []
    for _ in range(2):  # the same program twice, from the same state (statistics shift K = 0)
        p.reset_stats_shift()
        m1.impl._stage_inputs(p, x, y)
        p.run_segment("fwd")
        p.run_segment("bwd")
        torch.cuda.synchronize()
        grads.append(m1.arena.grad.clone())
    assert torch.equal(grads[0], grads[1])
    # and still the right gradients: per parameter vs the eager fp32 reference, within the bf16
    # autocast precision floor (the same criterion as the non-deterministic fused tests)
    from tests.test_fused_gpu import _check
    _check(m1, ref, x, y)
    # two independent models / programs, two full training steps each: identical weights
    m2, _ = _model(arch)
    p.reset_stats_shift()  # m1's program already ran steps: start both from the same state
    for _ in range(2):
        m1.impl.train_step(x, y)
        m2.impl.train_step(x, y)
    torch.cuda.synchronize()
    for a, b in zip(m1.net.trainable_weights, m2.net.trainable_weights):
        assert torch.equal(a, b)


@pytest.mark.miopen_ref
@pytest.mark.parametrize("arch,B", [("densenet121", 64), ("vgg16", 32)])
def test_dual_graph_backward_matches_direct_issue(monkeypatch, arch, B):
    """The backward replayed as two graphs (main lane + side lane joined by external events,
    plan.cpp capture_dual) must order every weight-gradient kernel after the dgrad that stages
    its operand: under IDC_DETERMINISTIC=1 it gives the same bits as direct issue, step after step
    (a side-lane kernel that ran early would read the previous step's gradients)."""
    monkeypatch.setenv("IDC_DETERMINISTIC", "1")
    g = torch.Generator().manual_seed(5)
    xs = [torch.randint(0, 256, (B, 50, 50, 3), generator=g, dtype=torch.uint8) for _ in range(3)]
    ys = [torch.randint(0, 2, (B,), generator=g) for _ in range(3)]
    monkeypatch.setenv("IDC_DUAL_GRAPH", "1")
    m1, _ = _model(arch)
    p1 = m1.impl._prog(B, True, torch.uint8)
    assert "bwd" in p1.graph_segments and p1.dual_graphs
    monkeypatch.setenv("IDC_DUAL_GRAPH", "0")
    monkeypatch.setenv("IDC_GRAPH_SEGMENTS", "fwd,opt")
    m2, _ = _model(arch)
    p2 = m2.impl._prog(B, True, torch.uint8)
    assert "bwd" not in p2.graph_segments
    for x, y in zip(xs, ys):
        m1.impl.train_step(x, y)
        m2.impl.train_step(x, y)
    torch.cuda.synchronize()
    assert any(k[0] == "dual" for k in p1.graphs if isinstance(k, tuple) and len(k) == 3)
    assert torch.equal(m1.arena.grad, m2.arena.grad)
    for a, b in zip(m1.net.trainable_weights, m2.net.trainable_weights):
        assert torch.equal(a, b)
