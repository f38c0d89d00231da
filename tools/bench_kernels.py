"""Microbenchmark of the conv kernels on the DenseNet-121 @50x50, bs=256 shapes (per tile).

    python tools/bench_kernels.py            # prints us per launch and TFLOP/s
"""
import sys

import torch

sys.path.insert(0, ".")
from idc_models_amd.ops import functional as fn  # noqa: E402
from idc_models_amd.ops import _native as nat  # noqa: E402

DEV = "cuda"


def timeit(f, reps=20):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ext = nat.require()
    N = 256
    cases = [("1x1 s1 64->128 13x13", 13, 64, 128, 1), ("1x1 s1 224->128 13x13", 13, 224, 128, 1),
             ("3x3 s1 128->32 13x13", 13, 128, 32, 3), ("1x1 s1 480->128 6x6", 6, 480, 128, 1),
             ("3x3 s1 128->32 6x6", 6, 128, 32, 3), ("1x1 992->128 3x3", 3, 992, 128, 1)]
    for name, H, cin, cout, k in cases:
        x = torch.randn(N, H, H, cin, device=DEV).to(torch.bfloat16)
        w = torch.randn(k, k, cin, cout, device=DEV) * 0.05
        st = torch.cat([x.float().sum((0, 1, 2)), (x.float() ** 2).sum((0, 1, 2))])
        bn = fn.BN(stats=st, gamma=torch.ones(cin, device=DEV), beta=torch.zeros(cin, device=DEV),
                   count=N * H * H, eps=1e-3, act=1)
        sout = torch.zeros(2 * cout, device=DEV)
        wl = fn.weight_fwd_layout(w, cin)
        flops = 2.0 * N * H * H * cout * k * k * cin
        res = []
        for t in range(ext.num_tiles()):
            if ext.tile_bn(t) > max(32, cout):
                continue
            us = timeit(lambda: fn.conv2d(x, w, pads=(k // 2, k // 2), pro=bn, stats=sout, tile=t, w_layout=wl))
            us0 = timeit(lambda: fn.conv2d(x, w, pads=(k // 2, k // 2), tile=t, w_layout=wl))
            res.append((us, t, us0))
        res.sort()
        best = res[0]
        print(f"{name:28s} best tile {best[1]:2d}: {best[0]:7.1f} us ({flops / best[0] / 1e6:6.1f} TF/s)"
              f"  plain {best[2]:7.1f} us | " + " ".join(f"t{t}:{u:.0f}/{u0:.0f}" for u, t, u0 in res))
        dy = torch.randn(N, H, H, cout, device=DEV).to(torch.bfloat16)
        for s in (8, 32, 128):
            us = timeit(lambda: fn.conv2d_wgrad(x, dy, (k, k), pads=(k // 2, k // 2), pro=bn, splits=s))
            print(f"    wgrad splits {s:4d}: {us:7.1f} us ({flops / us / 1e6:6.1f} TF/s)")


if __name__ == "__main__":
    main()
