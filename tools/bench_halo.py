"""Halo direct-3x3 kernel vs the best implicit-GEMM tile on the DenseNet growth-conv shapes.

    python tools/bench_halo.py
"""
import sys

import torch

import os  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from idc_models_amd.ops import functional as fn  # noqa: E402
from idc_models_amd.ops import _native as nat  # noqa: E402
from bench_kernels import timeit  # noqa: E402

DEV = "cuda"


def main():
    ext = nat.require()
    N = 256
    for H in (13, 6, 3):
        cin, cout = 128, 32
        x = torch.randn(N, H, H, cin, device=DEV).to(torch.bfloat16)
        w = torch.randn(3, 3, cin, cout, device=DEV) * 0.05
        st = torch.cat([x.float().sum((0, 1, 2)), (x.float() ** 2).sum((0, 1, 2))])
        bn = fn.BN(stats=st, gamma=torch.ones(cin, device=DEV), beta=torch.zeros(cin, device=DEV),
                   count=N * H * H, eps=1e-3, act=1)
        sout = torch.zeros(2 * cout, device=DEV)
        wl = fn.weight_fwd_layout(w, cin)
        flops = 2.0 * N * H * H * cout * 9 * cin
        res = {}
        for t in list(range(ext.num_tiles())) + [ext.TILE_HALO]:
            if t != ext.TILE_HALO and ext.tile_bn(t) > 32:
                continue
            res[t] = timeit(lambda: fn.conv2d(x, w, pads=(1, 1), pro=bn, stats=sout, tile=t, w_layout=wl))
        best = min((v, k) for k, v in res.items() if k != ext.TILE_HALO)
        h = res[ext.TILE_HALO]
        print(f"fwd   {H:2d}x{H:<2d}: halo {h:6.1f} us ({flops / h / 1e6:5.0f} TF/s) | best igemm t{best[1]} {best[0]:6.1f} us")
        # dgrad: fp32 dy (32 ch) -> dz (128 ch) with BN-backward epilogue
        dy = torch.randn(N, H, H, cout, device=DEV)
        mx = x
        gs = torch.zeros(cin, device=DEV)
        gx = torch.zeros(cin, device=DEV)
        res = {}
        for t in [ext.TILE_HALO, -1]:
            res[t] = timeit(lambda: fn.conv2d_dgrad(dy, w, (H, H), pads=(1, 1), mx=mx, mbn=bn, gsum=gs,
                                                      gsumx=gx, tile=t))
        print(f"dgrad {H:2d}x{H:<2d}: halo {res[ext.TILE_HALO]:6.1f} us | default igemm {res[-1]:6.1f} us")


if __name__ == "__main__":
    main()
