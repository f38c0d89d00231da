"""The DenseNet-121 stem max pool at the bench shape (bs 256, 25x25x64 -> 13x13, 3x3 / 2, pad 1),
forward (BN + ReLU prologue, output statistics) and backward (fp32 dy through a pending
BatchNorm backward, BN + ReLU epilogue with gradient sums), a few launches each: run under
`rocprofv3 --kernel-trace --stats` (IDC_POOL_IMG=0/1 selects the row / image-resident kernels)."""
import os
import sys
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from idc_models_amd.ops import functional as fn  # noqa: E402

DEV = torch.device("cuda", 0)


def main():
    fn.nat.require()
    N, H, C, Ho = 256, 25, 64, 13
    g = torch.Generator(device="cpu").manual_seed(3)
    y = torch.randn(N, H, H, C, generator=g).to(DEV)
    st = torch.cat([y.sum((0, 1, 2)), (y * y).sum((0, 1, 2))])
    gam, bet = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.1
    bn = fn.BN(stats=st, gamma=gam, beta=bet, count=N * H * H, eps=1e-3, act=1)
    yb = y.to(torch.bfloat16)
    out_stats = torch.zeros(2 * C, device=DEV)
    for _ in range(5):
        p, am = fn.pool2d(yb, 3, 2, pads=(1, 1), is_max=True, pro=bn, stats=out_stats)
    # the later BatchNorm's pending backward on dy (x = the pool output)
    pst = torch.cat([p.float().sum((0, 1, 2)), (p.float() ** 2).sum((0, 1, 2))])
    pbn = fn.BN(stats=pst, gamma=gam, beta=bet, count=N * Ho * Ho, eps=1e-3, act=1)
    gs, gx = torch.randn(C, device=DEV), torch.randn(C, device=DEV)
    aff = fn.bwd_aff(p, pbn, gs, gx, unit_alpha=True)
    dy = torch.randn(N, Ho, Ho, C, device=DEV)
    s1, s2 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    for _ in range(5):
        fn.pool2d_bwd(dy, (N, H, H, C), 3, 2, pads=(1, 1), is_max=True, argmax=am, x=yb, bn=bn, gsum=s1,
                      gsumx=s2, dyaff=aff)
    torch.cuda.synchronize()
    print("ok", float(s1.sum()))


if __name__ == "__main__":
    main()
