"""Timing of the stem kernels (conv_stem.hip, wgrad_stem.hip) against the implicit GEMM on the
DenseNet-121 stem shape (bs 256, 50x50x8 -> 25x25x64, 7x7 / 2): with and without statistics."""
import os
import sys
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from idc_models_amd.ops import functional as fn  # noqa: E402

DEV = torch.device("cuda", 0)


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
    ext = fn.nat.require()
    only = len(sys.argv) > 1 and sys.argv[1] == "--stem-only"
    if only:  # (PMC runs: the DenseNet stem shape, the stem kernel only, a few launches)
        x = torch.zeros(256, 50, 50, 8, device=DEV)
        x[..., :3] = torch.rand(256, 50, 50, 3, device=DEV)
        x = x.to(torch.bfloat16)
        w = torch.randn(7, 7, 8, 64, device=DEV) * 0.05
        for _ in range(3):
            fn.conv2d(x, w, stride=(2, 2), pads=(3, 3), out_hw=(25, 25), tile=ext.TILE_STEM)
        torch.cuda.synchronize()
        return
    for (N, H, k, s, p, ho, C) in ((256, 50, 7, 2, 3, 25, 64), (256, 50, 3, 1, 1, 50, 64), (256, 50, 3, 2, 0, 25, 32)):
        x = torch.zeros(N, H, H, 8, device=DEV)
        x[..., :3] = torch.rand(N, H, H, 3, device=DEV)
        x = x.to(torch.bfloat16)
        w = torch.randn(k, k, 8, C, device=DEV) * 0.05
        st = torch.zeros(2 * C * 16, device=DEV)
        for tile in (ext.TILE_STEM, 2, 7):
            for stats in (None, st):
                t = timeit(lambda: fn.conv2d(x, w, stride=(s, s), pads=(p, p), out_hw=(ho, ho), tile=tile, stats=stats))
                print(f"fwd k{k} s{s} C{C} tile {tile} stats {stats is not None}: {t:.1f} us", flush=True)
        dy = torch.randn(N, ho, ho, C, device=DEV).to(torch.bfloat16)
        for part in (False, True):
            n = k * k * 3 * C
            slab = torch.zeros(2048 * n, device=DEV) if part else None
            t = timeit(lambda: fn.conv2d_wgrad(x, dy, (k, k), stride=(s, s), pads=(p, p), cin_real=3, part=slab,
                                               splits=2048 if part else -1))
            print(f"wgrad k{k} s{s} C{C} part {part}: {t:.1f} us", flush=True)


if __name__ == "__main__":
    main()
