"""Gradient fidelity of a bf16 training step against an fp32 eager reference.

A randomly initialised DenseNet-121 in training mode (batch-statistics BN) has an ill-conditioned
gradient: in fp32 eager, perturbing its 50x50 inputs by 1e-6 moves the whole gradient by 2.5 %
(relative L2), rounding the inputs to bf16 moves it by 45 %, and PyTorch's own bf16 autocast is
79 % away from fp32 (batch 64, seed 7; see profiles/densenet121_spread_bs64.md). So "close to
fp32" can only be judged per parameter RELATIVE to what bf16 rounding does to that parameter:
the yardsticks here are bf16 autocast and fp32-on-bf16-rounded-inputs, both computed by this
module on the same network and batch.

Used by tests/rccl_worker.py (data-parallel step), tests/test_fused_gpu.py (bench-batch
fused-vs-eager) and tools/grad_fidelity.py (the committed measurement).
"""
from __future__ import annotations

import copy
from typing import Dict, List, Sequence

import os

import torch
import torch.nn.functional as F


def eager_grads(net, x_u8: torch.Tensor, y: torch.Tensor, mode: str = "fp32") -> List[torch.Tensor]:
    """Gradients of BCE-with-logits wrt every trainable Parameter of a deep copy of ``net``
    (training mode), on uint8 NHWC inputs scaled by 1/255. ``mode``: ``fp32``; ``autocast``
    (bf16 autocast forward); ``bf16in`` (fp32 network on inputs rounded to bf16)."""
    ref = copy.deepcopy(net)
    dev = next(iter(ref.parameters())).device
    xs = x_u8.to(dev).float() / 255.0
    if mode == "bf16in":
        xs = xs.bfloat16().float()
    yy = y.to(dev).float().reshape(-1)
    ref.train()
    with torch.autocast(dev.type, dtype=torch.bfloat16, enabled=(mode == "autocast")):
        lg = ref(xs)
    loss = F.binary_cross_entropy_with_logits(lg.float().reshape(-1), yy)
    ps = [p for p in ref.trainable_weights if isinstance(p, torch.nn.Parameter)]
    return [g.detach().double() for g in torch.autograd.grad(loss, ps)]


def eager_loss(net, x_u8: torch.Tensor, y: torch.Tensor, mode: str = "fp32") -> float:
    """Training-mode BCE-with-logits loss of a deep copy of ``net`` (``mode`` as in eager_grads)."""
    ref = copy.deepcopy(net)
    dev = next(iter(ref.parameters())).device
    xs = x_u8.to(dev).float() / 255.0
    ref.train()
    with torch.no_grad(), torch.autocast(dev.type, dtype=torch.bfloat16, enabled=(mode == "autocast")):
        lg = ref(xs)
    return float(F.binary_cross_entropy_with_logits(lg.float().reshape(-1), y.to(dev).float().reshape(-1)))


def eager_activations(net, x_u8: torch.Tensor, names: Sequence[str], mode: str = "fp32") -> Dict[str, torch.Tensor]:
    """Outputs of the named layers of a deep copy of ``net`` (training-mode forward, ``mode`` as
    in ``eager_grads``), as float64 NHWC tensors."""
    ref = copy.deepcopy(net)
    dev = next(iter(ref.parameters())).device
    xs = x_u8.to(dev).float() / 255.0
    if mode == "bf16in":
        xs = xs.bfloat16().float()
    base = getattr(ref, "base", ref)
    out: Dict[str, torch.Tensor] = {}
    hooks = [base.get_layer(n).register_forward_hook(
        lambda _m, _i, o, n=n: out.__setitem__(n, o.detach().double())) for n in names]
    ref.train()
    with torch.no_grad(), torch.autocast(dev.type, dtype=torch.bfloat16, enabled=(mode == "autocast")):
        ref(xs)
    for h in hooks:
        h.remove()
    return out


def _cos(a: torch.Tensor, b: torch.Tensor) -> float:
    a, b = a.reshape(-1).double(), b.reshape(-1).double()
    return float(a @ b / (a.norm() * b.norm() + 1e-300))


def _rel(a: torch.Tensor, ref: torch.Tensor) -> float:
    a, ref = a.reshape(-1).double(), ref.reshape(-1).double()
    return float((a - ref).norm() / ref.norm().clamp_min(1e-300))


def param_report(arena, grad: torch.Tensor, g32: Sequence[torch.Tensor],
                 yardsticks: Dict[str, Sequence[torch.Tensor]]) -> List[dict]:
    """Per parameter: cosine and relative error of the fused gradient (flat ``grad`` in
    ``arena`` layout) vs fp32, and the same two numbers for every yardstick gradient."""
    rows = []
    for i, gr in enumerate(g32):
        if float(gr.norm()) < 1e-12:
            continue
        gf = arena.view(grad, i).to(gr.device)
        row = {"param": i, "shape": list(gr.shape), "cos": _cos(gf, gr), "rel": _rel(gf, gr)}
        for k, gs in yardsticks.items():
            row[f"cos_{k}"] = _cos(gs[i], gr)
            row[f"rel_{k}"] = _rel(gs[i], gr)
        rows.append(row)
    return rows


FACTOR = 1.5
# (0.02 was tried in round 6: a DenseNet-201 head-bias gradient -- 10 values, cos 1.0 -- drew
# rel 0.039 against autocast's < 0.01 after a change that only reordered fp32 statistics sums; the
# floor is the absolute noise a chaotic random-init forward leaves on tiny parameters)
FLOOR = 0.05
# every parameter must stay within HARD_FACTOR x autocast's error; at most SOFT_FRACTION of them
# (at least one) may exceed FACTOR x: each parameter's error is one random draw of the rounding
# noise, and a network with ~600 parameter tensors occasionally draws one past 1.5x (DenseNet-201
# at batch 32: 1.16 vs a 1.14 bound), while a systematic error moves many, or one by far more
# (round 6: 3.0 -> 2.0; the worst non-invariant draw measured is 1.19x,
# profiles/densenet121_gradient_fidelity.md)
HARD_FACTOR = 2.0
SOFT_FRACTION = 0.01
# Parameters whose fp32 per-element RMS gradient is below 1e-2 x the network's median are
# directions the loss is invariant to.  Measured (fp32, CPU): DenseNet-121/201 stem BN gamma at
# 8e-4 / 1.6e-3 x median, MobileNetV2 project-BN betas at 1e-7..1e-6 x median (a per-channel
# constant before a 1x1 conv and a batch-statistics BN cancels), every other parameter >= 0.09 x.
INVARIANT = 1e-2
# bf16 rounding noise allowed on them, in units of the median per-element RMS (measured on one
# MI355X: 0.25-1.5 x; the exact gradient is 0 and an update along them does not change the loss)
INVARIANT_NOISE = 2.0


def grad_failures(arena, grad: torch.Tensor, g32: Sequence[torch.Tensor], g16: Sequence[torch.Tensor],
                  factor: float = FACTOR, floor: float = FLOOR) -> List[dict]:
    """Parameters whose fused gradient is further from fp32 than bf16 autocast's, beyond
    ``rel(fused) <= factor * rel(autocast) + floor`` (relative L2 per parameter: direction AND
    magnitude; a cosine alone misses a gradient that is right in direction and 300x too large).
    Measured on DenseNet-121 at batch 64 / 256 (profiles/densenet121_gradient_fidelity.md): the
    ratio rel(fused)/rel(autocast) has median 0.96-1.00, 99th percentile 1.17-1.19.  Every
    parameter must stay within HARD_FACTOR x; at most SOFT_FRACTION of them past ``factor`` x.
    Directions the loss is invariant to (see INVARIANT) are bounded on the network's gradient
    scale."""
    bad, soft = [], []
    rms = [float(g.norm()) / max(g.numel(), 1) ** 0.5 for g in g32]
    med = sorted(rms)[len(rms) // 2] if rms else 0.0
    rows = param_report(arena, grad, g32, {"autocast": g16})
    for r in rows:
        i = r["param"]
        if rms[i] < INVARIANT * med:
            # a direction the loss is (numerically) invariant to: DenseNet's stem BN gamma at
            # beta = 0 feeds ReLU -> max-pool -> only batch-statistics BatchNorms, so scaling it
            # changes nothing (exact gradient 0, fp32 leaves ~1e-6 of eps effects).  Its bf16
            # gradient is rounding noise by construction; require the noise to stay small on the
            # network's gradient scale instead of relative to an ~0 reference
            frms = float(arena.view(grad, i).double().norm()) / max(g32[i].numel(), 1) ** 0.5
            if frms > INVARIANT_NOISE * med:
                bad.append({"param": i, "shape": r["shape"], "invariant": True, "rms_fused": frms, "median_rms": med})
            continue
        row = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}
        if r["rel"] > HARD_FACTOR * r["rel_autocast"] + floor:
            bad.append(row)
        elif r["rel"] > factor * r["rel_autocast"] + floor:
            soft.append(row)
    if len(soft) > max(1, int(SOFT_FRACTION * len(rows))):
        bad += soft
    if os.environ.get("IDC_FIDELITY_LOG") == "1":  # margin report: the worst ratio and its bound
        ratios = sorted(r["rel"] / max(r["rel_autocast"], 1e-300) for r in rows if rms[r["param"]] >= INVARIANT * med)
        if ratios:
            print(f"[fidelity] {len(ratios)} params: ratio p50 {ratios[len(ratios) // 2]:.3f} "
                  f"p99 {ratios[int(0.99 * (len(ratios) - 1))]:.3f} max {ratios[-1]:.3f} "
                  f"(soft {factor}x + {floor}, hard {HARD_FACTOR}x)", flush=True)
    return bad


def whole_rel(arena, grad: torch.Tensor, g32: Sequence[torch.Tensor]) -> float:
    """Relative L2 error of the whole fused gradient vs fp32."""
    num = den = 0.0
    for i, gr in enumerate(g32):
        gf = arena.view(grad, i).to(gr.device).double()
        num += float((gf.reshape(-1) - gr.reshape(-1)).pow(2).sum())
        den += float(gr.pow(2).sum())
    return (num / max(den, 1e-300)) ** 0.5


def whole_rel_list(gs: Sequence[torch.Tensor], g32: Sequence[torch.Tensor]) -> float:
    num = sum(float((a - b).pow(2).sum()) for a, b in zip(gs, g32))
    den = sum(float(b.pow(2).sum()) for b in g32)
    return (num / max(den, 1e-300)) ** 0.5
