"""Run-to-run reproducibility of the fused training step: the same program, weights and inputs,
fwd+bwd twice; per-parameter gradient cosine / relative difference (worst first).  With
IDC_DETERMINISTIC=1 every reduction has a fixed order and the two runs must agree bit for bit.

    python tools/run_to_run.py [--model densenet121] [--batch 256]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="densenet121")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args()
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model
    dev = torch.device("cuda", 0)
    net = build_model(a.model, num_outputs=1, seed=0)
    m = Model(net, device=dev)
    m.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="fused")
    g = torch.Generator().manual_seed(1)
    H, W, C = net.input_shape
    x = torch.randint(0, 256, (a.batch, H, W, C), generator=g, dtype=torch.uint8)
    y = torch.randint(0, 2, (a.batch,), generator=g)
    p = m.impl._prog(a.batch, True, torch.uint8)
    gs, ls = [], []
    for _ in range(3):
        m.impl._stage_inputs(p, x, y)
        p.run_segment("fwd")
        p.run_segment("bwd")
        torch.cuda.synchronize()
        gs.append(m.arena.grad.double().clone())
        ls.append(float(p.io.loss.item()))
    ar = m.arena
    rows = []
    for i, prm in enumerate(ar.params):
        a0, a1 = ar.view(gs[1], i).reshape(-1), ar.view(gs[2], i).reshape(-1)
        cos = float(a0 @ a1 / (a0.norm() * a1.norm() + 1e-300))
        rel = float((a0 - a1).norm() / (a1.norm() + 1e-300))
        rows.append((rel, cos, i, tuple(prm.shape), getattr(prm, "_keras_name", "")))
    rows.sort(reverse=True)
    tot = float((gs[1] - gs[2]).norm() / gs[2].norm())
    print(f"{a.model} bs{a.batch} loss runs {ls}  whole-arena rel diff {tot:.3e}  identical={bool(torch.equal(gs[1], gs[2]))}")
    for rel, cos, i, shp, nm in rows[:a.top]:
        print(f"  param {i:4d} {str(shp):22s} rel {rel:.3e} cos {cos:.6f} {nm}")
    print("  median rel", sorted(r[0] for r in rows)[len(rows) // 2])


if __name__ == "__main__":
    main()
