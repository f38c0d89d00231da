"""Isolated device time of the deep-ring tiles (conv_ring.hip) vs the general kernel's tiles on the
DenseNet-121 bs256 forward shapes (pending-BN prologue + statistics epilogue).

    python tools/bench_ring.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from idc_models_amd.ops import _native as nat
    from idc_models_amd.ops import functional as fn
    ext = nat.load()
    dev = torch.device("cuda", 0)
    shapes = [("s1 1x1 K64", 256, 13, 64, 128, 1), ("s1 3x3", 256, 13, 128, 32, 3),
              ("s2 1x1 K480", 256, 6, 480, 128, 1), ("s2 3x3", 256, 6, 128, 32, 3),
              ("s3 1x1 K544", 256, 3, 544, 128, 1), ("s3 1x1 K992", 256, 3, 992, 128, 1),
              ("s3 3x3", 256, 3, 128, 32, 3), ("s4 1x1 K544", 256, 1, 544, 128, 1)]
    for name, N, H, Cin, Cout, k in shapes:
        x = torch.randn(N, H, H, Cin, device=dev).to(torch.bfloat16)
        w = torch.randn(k, k, Cin, Cout, device=dev) * 0.02
        wl = fn.weight_fwd_layout(w, Cin)
        st_in = torch.cat([x.float().sum((0, 1, 2)), (x.float() ** 2).sum((0, 1, 2))])
        bn = fn.BN(stats=st_in, gamma=torch.ones(Cin, device=dev), beta=torch.zeros(Cin, device=dev),
                   count=N * H * H, eps=1e-3, act=1)
        pads = (1, 1) if k == 3 else (0, 0)
        cands = [t for t in range(ext.num_tiles()) if ext.tile_bn(t) <= max(32, Cout)]
        cands += [ext.TILE_RING + v for v in range(ext.TILE_RING_N)]
        res = []
        for t in cands:
            st = torch.zeros(2 * Cout, device=dev)
            try:
                fn.conv2d(x, w, pads=pads, pro=bn, tile=t, stats=st, w_layout=wl)
                torch.cuda.synchronize()
            except Exception:
                continue
            # 20 launches captured in one graph: device time per launch (incl. the ~1.5 us
            # dependent-kernel boundary), free of host issue cost
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(20):
                    fn.conv2d(x, w, pads=pads, pro=bn, tile=t, stats=st, w_layout=wl)
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                g.replay()
            e1.record()
            e1.synchronize()
            res.append((e0.elapsed_time(e1) / 60 * 1e3, t))
            del g
        res.sort()
        ring = sorted(r for r in res if r[1] >= ext.TILE_RING)
        print(f"{name:14s} best {res[0][1]:3d} {res[0][0]:6.2f} us | best ring {ring[0][1]} {ring[0][0]:6.2f} us | "
              + " ".join(f"t{t}:{us:.1f}" for us, t in res[:6]), flush=True)


if __name__ == "__main__":
    main()
