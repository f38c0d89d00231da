"""Host issue time vs GPU time of each segment of one training step (is a segment host-bound?).

    python tools/host_issue.py [--model mobilenetv2] [--batch 256] [--steps 20]

For every segment: the host time of issuing it (no synchronisation), and the time until the GPU
finishes it (synchronised right after issue).  A backward whose issue time approaches its GPU time
is bound by kernel-launch overhead: its main lane idles while the host catches up.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mobilenetv2")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model
    dev = torch.device("cuda", 0)
    net = build_model(a.model, num_outputs=1, seed=0)
    m = Model(net, device=dev)
    m.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="fused")
    H, W, C = net.input_shape
    x = torch.randint(0, 256, (a.batch, H, W, C), dtype=torch.uint8, device=dev)
    y = torch.randint(0, 2, (a.batch,), device=dev)
    for _ in range(5):
        m.impl.train_step(x, y)
    torch.cuda.synchronize()
    p = m.impl._prog(a.batch, True, torch.uint8)
    segs = [s for s in ("fwd", "bwd", "opt") if s in p.seg]
    res = {s: [[], []] for s in segs}
    for _ in range(a.steps):
        m.impl._stage_inputs(p, x, y)
        for s in segs:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if s == "bwd":
                p.run_bwd()
            else:
                p.run_segment(s)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            res[s][0].append((t1 - t0) * 1e6)
            res[s][1].append((t2 - t0) * 1e6)
    for s in segs:
        iss, tot = sorted(res[s][0]), sorted(res[s][1])
        n = len(iss) // 2
        lo, hi = p.seg[s]
        print(f"{a.model} {s}: {hi - lo} ops, host issue {iss[n]:.0f} us, issue + GPU {tot[n]:.0f} us")


if __name__ == "__main__":
    main()
