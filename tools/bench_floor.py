"""Per-launch floor and small-conv latency: back-to-back launches of one op, events around 200.

    python tools/bench_floor.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from idc_models_amd.ops import _native as nat  # noqa: E402
from idc_models_amd.ops import functional as fn  # noqa: E402


def per_launch(plan, i, sh, reps=200, graph=False):
    st = torch.cuda.current_stream()  # a side stream (main() runs under torch.cuda.stream(S))
    if graph:
        g = plan.capture(i, i + 1, sh)
    plan.run(i, i + 1, sh)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        if graph:
            plan.launch(g, sh)
        else:
            plan.run(i, i + 1, sh)
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    with torch.cuda.stream(torch.cuda.Stream()):
        _main()


def _main():
    ext = nat.require()
    sh = torch.cuda.current_stream().cuda_stream
    buf = torch.zeros(1 << 20, device="cuda")
    plan = ext.Plan()
    plan.add(nat.OP_MEMSET, b"", [], [], [16], [buf.data_ptr()], 0)
    plan.add(nat.OP_MEMSET, b"", [], [], [4 << 20], [buf.data_ptr()], 0)
    print(f"zero_fill 16 B   : {per_launch(plan, 0, sh):6.2f} us/launch (direct)  "
          f"{per_launch(plan, 0, sh, graph=True):6.2f} us (graph replay of 1 node)")
    print(f"zero_fill 4 MiB  : {per_launch(plan, 1, sh):6.2f} us/launch")
    # a 10-node graph of tiny kernels: per-node cost inside a graph
    p10 = ext.Plan()
    for _ in range(10):
        p10.add(nat.OP_MEMSET, b"", [], [], [16], [buf.data_ptr()], 0)
    g = p10.capture(0, 10, sh)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(torch.cuda.current_stream())
    for _ in range(50):
        p10.launch(g, sh)
    e1.record(torch.cuda.current_stream())
    torch.cuda.synchronize()
    print(f"graph of 10 tiny kernels: {e0.elapsed_time(e1) / 500 * 1e3:6.2f} us per node")
    N = 256
    for (H, cin, cout, k) in [(3, 512, 128, 1), (3, 992, 128, 1), (1, 992, 128, 1), (6, 480, 128, 1),
                              (13, 224, 128, 1), (3, 128, 32, 3), (6, 128, 32, 3), (13, 128, 32, 3)]:
        x = torch.randn(N, H, H, cin, device="cuda").to(torch.bfloat16)
        w = torch.randn(k, k, cin, cout, device="cuda") * 0.05
        wl = fn.weight_fwd_layout(w, cin)
        y = torch.empty(N, H, H, cout, device="cuda", dtype=torch.bfloat16)
        a = nat.ConvArgs()
        a.x, a.N, a.H, a.W, a.Cin, a.ldx = x.data_ptr(), N, H, H, cin, cin
        a.Ho, a.Wo, a.Cout, a.y, a.ldy = H, H, cout, y.data_ptr(), cout
        a.w = wl.data_ptr()
        a.KH, a.KW, a.SH, a.SW, a.PT, a.PL = k, k, 1, 1, k // 2, k // 2
        a.pro, a.mbn = nat.bn_args(), nat.bn_args()
        best = None
        for t in range(ext.num_tiles()):
            if ext.tile_bn(t) > max(32, cout):
                continue
            pl = ext.Plan()
            for _ in range(40):
                pl.add(nat.OP_CONV, nat.raw(a), [t, 0], [], [], [], 0)
            gid = pl.capture(0, 40, sh)
            pl.launch(gid, sh)
            torch.cuda.synchronize()
            e0.record(torch.cuda.current_stream())
            for _ in range(5):
                pl.launch(gid, sh)
            e1.record(torch.cuda.current_stream())
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 200 * 1e3
            if best is None or us < best[0]:
                best = (us, t)
        flops = 2.0 * N * H * H * cout * k * k * cin
        print(f"conv {k}x{k} {cin:4d}->{cout:3d} {H:2d}x{H:<2d} M={N * H * H:6d}: best tile {best[1]:2d} "
              f"{best[0]:6.1f} us  ({flops / best[0] / 1e6:6.1f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
