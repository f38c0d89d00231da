"""Where does the run-to-run spread of the fused training step come from?

Two runs of the SAME program on the same weights and batch, every statistics shift reset to the
first-step state before each run, compared by the relative L2 difference of the whole gradient
arena and the worst / median per-parameter cosine -- for the default program and with each source
of non-deterministic float-atomic ordering switched off in turn:

  dense_stage0   IDC_DENSE_STAGE=0        persistent dense-stage forward (slotted atomics)
  wgbatch0       IDC_WG_BATCH_MAXM=0      batched late-stage weight gradients
  splitk0        IDC_SPLITK=0             split-K tickets of the autotuned convs
  autotune0      IDC_AUTOTUNE=0           fixed default tiles (no split-K, no timing choices)
  all0           all of the above
  det            IDC_DETERMINISTIC=1      every reduction in a fixed order (must be bitwise 0)
  det+perturb    deterministic, but ONE input pixel of ONE image changed by 1/255: the network's own
                 sensitivity to a perturbation far below bf16 resolution, i.e. the spread any
                 rounding-order difference is amplified to

    python tools/spread.py [--model densenet121] [--batch 64] [--md out.md]
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = [
    ("default", {}),
    ("dense_stage0", {"IDC_DENSE_STAGE": "0"}),
    ("wgbatch0", {"IDC_WG_BATCH_MAXM": "0"}),
    ("splitk0", {"IDC_SPLITK": "0"}),
    ("autotune0", {"IDC_AUTOTUNE": "0"}),
    ("all0", {"IDC_DENSE_STAGE": "0", "IDC_WG_BATCH_MAXM": "0", "IDC_SPLITK": "0", "IDC_AUTOTUNE": "0"}),
    ("det", {"IDC_DETERMINISTIC": "1"}),
    ("det+perturb", {"IDC_DETERMINISTIC": "1"}),
]
KEYS = ("IDC_DENSE_STAGE", "IDC_WG_BATCH_MAXM", "IDC_SPLITK", "IDC_AUTOTUNE", "IDC_DETERMINISTIC")


def measure(model: str, batch: int, env: dict, perturb: bool):
    import torch

    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model
    for k in KEYS:
        os.environ.pop(k, None)
    os.environ.update(env)
    dev = torch.device("cuda", 0)
    net = build_model(model, num_outputs=1, seed=0)
    m = Model(net, device=dev)
    m.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="fused")
    g = torch.Generator().manual_seed(1)
    H, W, C = net.input_shape
    x = torch.randint(0, 256, (batch, H, W, C), generator=g, dtype=torch.uint8)
    y = torch.randint(0, 2, (batch,), generator=g)
    x2 = x.clone()
    if perturb:
        x2[0, H // 2, W // 2, 0] = (int(x2[0, H // 2, W // 2, 0]) + 1) % 256
    p = m.impl._prog(batch, True, torch.uint8)
    gs, ls = [], []
    for xi in (x, x, x2):
        p.reset_stats_shift()
        m.impl._stage_inputs(p, xi, y)
        p.run_segment("fwd")
        p.run_segment("bwd")
        torch.cuda.synchronize()
        gs.append(m.arena.grad.double().clone())
        ls.append(float(p.io.loss.item()))
    a, b = gs[0], (gs[2] if perturb else gs[1])
    ar = m.arena
    coss = []
    for i in range(len(ar.params)):
        u, v = ar.view(a, i).reshape(-1), ar.view(b, i).reshape(-1)
        if v.norm() > 0:
            coss.append(float(u @ v / (u.norm() * v.norm() + 1e-300)))
    coss.sort()
    rel = float((a - b).norm() / b.norm())
    m.impl.close()
    return rel, coss[0], coss[len(coss) // 2], bool(torch.equal(a, b)), abs(ls[0] - (ls[2] if perturb else ls[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="densenet121")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--md", default=None)
    args = ap.parse_args()
    lines = [f"# Run-to-run spread of the fused step ({args.model}, batch {args.batch}, tools/spread.py)", "",
             "Two fwd+bwd runs of one program on identical weights and inputs (statistics shifts reset before "
             "each run); `det+perturb` compares a deterministic run with one on an input whose single pixel "
             "moved by 1/255.", "",
             "| config | gradient rel L2 diff | worst param cosine | median param cosine | bitwise equal | loss diff |",
             "|---|---:|---:|---:|---|---:|"]
    for name, env in CONFIGS:
        rel, worst, med, eq, dl = measure(args.model, args.batch, env, name.endswith("perturb"))
        lines.append(f"| {name} | {rel:.3e} | {worst:.6f} | {med:.6f} | {eq} | {dl:.2e} |")
        print(lines[-1], flush=True)
    out = "\n".join(lines) + "\n"
    if args.md:
        with open(args.md, "w") as f:
            f.write(out)


if __name__ == "__main__":
    main()
