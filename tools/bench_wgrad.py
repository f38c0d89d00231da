"""Isolated device time of the weight-gradient kernels on the VGG16 bs256 50x50 layer shapes:
the general pixel-split kernel (variant 0, conv_wgrad.hip) vs the large-tile LDS-DMA variants
(wgrad_big.hip) at a few pixel splits.  Each timing is 10 launches captured in one HIP graph
(device time per launch, the dependent-kernel boundary included).  Prints achieved TFLOP/s.

    python tools/bench_wgrad.py [--batch 256]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (name, H, Cin, Cout): VGG16 3x3 'same' convolutions after block 1
VGG = [("b1c2", 50, 64, 64), ("b2c1", 25, 64, 128), ("b2c2", 25, 128, 128), ("b3c1", 12, 128, 256),
       ("b3c2", 12, 256, 256), ("b4c1", 6, 256, 512), ("b4c2", 6, 512, 512), ("b5", 3, 512, 512)]


def graph_us(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        g.replay()
    e1.record()
    e1.synchronize()
    del g
    return e0.elapsed_time(e1) / (3 * reps) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--only", default=None, help="LAYER:VARIANT:SPLITS[,...]: plain launches (for --pmc runs)")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    from idc_models_amd.ops import functional as fn
    from idc_models_amd.ops import _native as nat
    ext = nat.require()
    dev = torch.device("cuda", 0)
    N = args.batch
    if args.only:
        shapes = {v[0]: v for v in VGG}
        for spec in args.only.split(","):
            name, v, sp = spec.split(":")
            _, H, Cin, Cout = shapes[name]
            x = (torch.randn(N, H, H, Cin, device=dev) * 0.5).to(torch.bfloat16)
            dy = (torch.randn(N, H, H, Cout, device=dev) * 0.1).to(torch.bfloat16)
            out = torch.zeros(3, 3, Cin, Cout, device=dev)
            for _ in range(args.iters):
                fn.conv2d_wgrad(x, dy, (3, 3), pads=(1, 1), splits=int(sp), out=out, variant=int(v))
            torch.cuda.synchronize()
            print(name, v, sp, "done", flush=True)
        return
    tot0 = totb = 0.0
    for name, H, Cin, Cout in VGG:
        x = (torch.randn(N, H, H, Cin, device=dev) * 0.5).to(torch.bfloat16)
        dy = (torch.randn(N, H, H, Cout, device=dev) * 0.1).to(torch.bfloat16)
        M, K = N * H * H, 9 * Cin
        gflop = 2.0 * M * K * Cout / 1e9
        out = torch.zeros(3, 3, Cin, Cout, device=dev)
        s0 = ext.pick_splits(M, K, Cout)
        ref = fn.conv2d_wgrad(x, dy, (3, 3), pads=(1, 1), splits=s0)
        res = {}
        res[(0, s0)] = graph_us(lambda: fn.conv2d_wgrad(x, dy, (3, 3), pads=(1, 1), splits=s0, out=out))
        for v in range(1, ext.wgrad_num_variants()):
            if not fn.wgrad_big_applies(x, dy, (3, 3), (1, 1), (1, 1), v):
                continue
            sp = ext.wgrad_big_pick_splits(M, K, Cout, v)
            chk = fn.conv2d_wgrad(x, dy, (3, 3), pads=(1, 1), splits=sp, variant=v)
            err = float((chk - ref).norm() / ref.norm())
            if err > 1e-2:
                print(f"  {name} variant {v}: MISMATCH rel {err:.3g}", flush=True)
                continue
            for s in sorted({max(1, sp // 2), sp, sp * 2}):
                res[(v, s)] = graph_us(lambda: fn.conv2d_wgrad(x, dy, (3, 3), pads=(1, 1), splits=s, out=out,
                                                               variant=v))
        best = min(res, key=res.get)
        t0 = res[(0, s0)]
        tot0 += t0
        totb += res[best]
        top = sorted(res.items(), key=lambda kv: kv[1])[:5]
        print(f"{name:5s} M={M:6d} K={K:4d} Co={Cout:3d} {gflop:5.1f} GF | general {t0:7.1f} us "
              f"({gflop / t0:.2f} PF) | best v{best[0]}/s{best[1]} {res[best]:7.1f} us "
              f"({gflop / res[best]:.2f} PF) | " + " ".join(f"v{k[0]}/s{k[1]}:{u:.0f}" for k, u in top),
              flush=True)
    print(f"total general {tot0:.0f} us, best {totb:.0f} us", flush=True)


if __name__ == "__main__":
    main()
