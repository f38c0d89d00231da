"""Per-parameter gradient fidelity of the fused bf16 step vs fp32 eager, next to bf16 yardsticks.

For one model / batch: the fp32 eager gradient of the seed's network; two yardsticks (PyTorch bf16
autocast; fp32 on bf16-rounded inputs); and R fused first-step gradients (default program, float
atomics) plus one deterministic one. Prints per-group medians / worst parameters and the per-
parameter error ratio rel(fused) / rel(autocast) -- the quantity tests bound.

    python tools/grad_fidelity.py [--model densenet121] [--batch 64] [--runs 3] [--md out.md]
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def fused_grads(model, batch, x, y, det, runs, seed):
    import torch

    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model
    os.environ["IDC_DETERMINISTIC"] = "1" if det else "0"
    m = Model(build_model(model, None, 1, seed=seed), device=torch.device("cuda", 0))
    m.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="fused")
    p = m.impl._prog(batch, True, torch.uint8)
    out = []
    for _ in range(runs):
        p.reset_stats_shift()
        m.impl._stage_inputs(p, x, y)
        p.run_segment("fwd")
        p.run_segment("bwd")
        torch.cuda.synchronize()
        out.append(m.arena.grad.detach().clone())
    return m, out


def main():
    import torch

    from idc_models_amd.models import build_model
    from idc_models_amd.utils import fidelity as fd
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="densenet121")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    net = build_model(a.model, None, 1, seed=a.seed).to(dev)
    g = torch.Generator().manual_seed(3)
    H, W, C = net.input_shape
    x = torch.randint(0, 256, (a.batch, H, W, C), generator=g, dtype=torch.uint8)
    y = torch.randint(0, 2, (a.batch,), generator=g)
    g32 = fd.eager_grads(net, x, y, "fp32")
    yard = {"autocast": fd.eager_grads(net, x, y, "autocast"), "bf16in": fd.eager_grads(net, x, y, "bf16in")}
    m, fused = fused_grads(a.model, a.batch, x, y, False, a.runs, a.seed)
    md, det = fused_grads(a.model, a.batch, x, y, True, 1, a.seed)
    L = [f"# Gradient fidelity vs fp32 eager ({a.model}, batch {a.batch}, seed {a.seed}, tools/grad_fidelity.py)",
         "", "Whole-gradient relative L2 error vs the fp32 eager gradient of the same network and batch:", "",
         "| gradient | rel L2 vs fp32 | median param cos | worst param cos | worst ratio rel/rel_autocast |",
         "|---|---:|---:|---:|---:|"]
    import statistics as st
    for k, gs in yard.items():
        cs = [fd._cos(u, v) for u, v in zip(gs, g32) if float(v.norm()) > 1e-12]
        L.append(f"| {k} | {fd.whole_rel_list(gs, g32):.3f} | {st.median(cs):.3f} | {min(cs):.3f} | |")
    all_rows = []
    for name, mm, gl in [(f"fused run {i}", m, [gg]) for i, gg in enumerate(fused)] + [("fused deterministic", md, det)]:
        rows = fd.param_report(mm.arena, gl[0], g32, yard)
        all_rows.append((name, rows))
        cs = [r["cos"] for r in rows]
        ratio = max(r["rel"] / max(r["rel_autocast"], 1e-12) for r in rows)
        L.append(f"| {name} | {fd.whole_rel(mm.arena, gl[0], g32):.3f} | {st.median(cs):.3f} | {min(cs):.3f} | {ratio:.2f} |")
    L += ["", "Per-parameter error ratio rel(fused)/rel(autocast), all fused runs pooled:", ""]
    ratios = sorted(r["rel"] / max(r["rel_autocast"], 1e-12) for _, rows in all_rows for r in rows)
    qs = [0.5, 0.9, 0.99, 1.0]
    L.append("| quantile | " + " | ".join(f"{q:g}" for q in qs) + " |")
    L.append("|---|" + "---:|" * len(qs) + "")
    L.append("| ratio | " + " | ".join(f"{ratios[min(len(ratios) - 1, int(q * (len(ratios) - 1)))]:.2f}" for q in qs) + " |")
    L += ["", "Ten worst parameters by ratio (first fused run):", "",
          "| param | shape | cos fused | cos autocast | cos bf16in | rel fused | rel autocast | rel bf16in |",
          "|---:|---|---:|---:|---:|---:|---:|---:|"]
    rows = sorted(all_rows[0][1], key=lambda r: -r["rel"] / max(r["rel_autocast"], 1e-12))
    for r in rows[:10]:
        L.append(f"| {r['param']} | {r['shape']} | {r['cos']:.3f} | {r['cos_autocast']:.3f} | {r['cos_bf16in']:.3f} "
                 f"| {r['rel']:.3f} | {r['rel_autocast']:.3f} | {r['rel_bf16in']:.3f} |")
    out = "\n".join(L) + "\n"
    print(out, flush=True)
    if a.md:
        with open(a.md, "w") as f:
            f.write(out)
    m.impl.close()
    md.impl.close()


if __name__ == "__main__":
    main()
