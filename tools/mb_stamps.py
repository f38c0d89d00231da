"""Per-phase timing of the persistent MobileNetV2 block chain (csrc/kernels/mb_chain.hip) from the
kernel's own s_memrealtime stamps (IDC_MB_STAMPS=1; 100 MHz clock; persist.h NSTAMP per ticket).

    python tools/mb_stamps.py [--batch 256] [--steps 5] [--md out.md]

Stamp points per tile: 0 ticket | 1 dependency ready | 2 tile done | 3 published (the last tile of
a phase also finalised its statistics and table).  Per phase (us): its end (last publish), the step
from the previous phase's end, the hand-off (first tile past its wait - previous end), the tiles'
median / max work time (2 - 1) and the finalising tile's publish + finalise time (3 - 2).
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NSTAMP = 8
KIND = {1: "TAB", 2: "PW", 3: "DW"}


def analyse(st, phases):
    import numpy as np
    n = sum(t for _, _, t in phases)
    a = st.reshape(-1, NSTAMP)[:n, :4].astype(np.float64)
    a[a == 0] = np.nan
    a = (a - np.nanmin(a[:, 0])) * 0.01
    rows, prev = [], 0.0
    for j, (kind, first, tiles) in enumerate(phases):
        blk = a[first:first + tiles]
        end = float(np.nanmax(blk[:, 3]))
        work = blk[:, 2] - blk[:, 1]
        fin = float(np.nanmax(blk[:, 3] - blk[:, 2]))
        rows.append({"j": j, "kind": KIND.get(kind, str(kind)), "tiles": tiles, "end": end, "step": end - prev,
                     "handoff": float(np.nanmin(blk[:, 1])) - prev, "work_med": float(np.nanmedian(work)),
                     "work_max": float(np.nanmax(work)), "fin": fin,
                     "wait_med": float(np.nanmedian(blk[:, 1] - blk[:, 0]))})
        prev = end
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--md", default=None)
    args = ap.parse_args()
    os.environ["IDC_MB_STAMPS"] = "1"
    import torch

    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model

    dev = torch.device("cuda", 0)
    net = build_model("mobilenetv2", num_outputs=1, seed=1234)
    m = Model(net, device=dev)
    m.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="fused")
    H, W, C = net.input_shape
    x = torch.randint(0, 256, (args.batch, H, W, C), dtype=torch.uint8, device=dev)
    y = torch.randint(0, 2, (args.batch,), device=dev)
    for _ in range(args.steps):
        m.impl.train_step(x, y)
    torch.cuda.synchronize()
    p = m.impl._prog(args.batch, True, torch.uint8)
    out = []
    for si, (stamps, phases) in enumerate(getattr(p.b, "mb_stamps", [])):
        rows = analyse(stamps.cpu().numpy(), phases)
        out += [f"## chain launch {si}: {len(phases)} phases, span {rows[-1]['end']:.1f} us "
                f"(err counter {int(p.b.dense_err[0])})", "",
                "| phase | kind | tiles | end | step | hand-off | wait med | work med | work max | last publish+finalise |",
                "|---|---|---:|---:|---:|---:|---:|---:|---:|---:|"]
        for r in rows:
            out.append(f"| {r['j']} | {r['kind']} | {r['tiles']} | {r['end']:.1f} | {r['step']:.2f} | {r['handoff']:.2f} | "
                       f"{r['wait_med']:.2f} | {r['work_med']:.2f} | {r['work_max']:.2f} | {r['fin']:.2f} |")
        out.append("")
    text = "\n".join(out)
    print(text)
    if args.md:
        with open(args.md, "w") as f:
            f.write(f"# MobileNetV2 block-chain phase timing (batch {args.batch}, in-kernel s_memrealtime stamps, "
                    f"last of {args.steps} steps)\n\n" + text + "\n")


if __name__ == "__main__":
    main()
