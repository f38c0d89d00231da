"""Isolated device time of the depthwise kernels on the MobileNetV2 bs256 50x50 layer shapes:
forward (pending BN + ReLU6 prologue, statistics epilogue), backward data (BN-backward epilogue)
and the two-stage weight gradient.  Each timing is 20 launches captured in one HIP graph.

    python tools/bench_dw.py [--batch 256]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (input H, C, stride, (PT, PL)) of the 17 depthwise layers (Keras correct_pad on stride 2)
MBV2 = [(25, 32, 1, (1, 1)), (25, 96, 2, (1, 1)), (13, 144, 1, (1, 1)), (13, 144, 2, (1, 1)),
        (7, 192, 1, (1, 1)), (7, 192, 2, (1, 1)), (4, 384, 1, (1, 1)), (4, 576, 1, (1, 1)),
        (4, 576, 2, (0, 0)), (2, 960, 1, (1, 1))]


def graph_us(fn, reps=20):
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
    args = ap.parse_args()
    from idc_models_amd.ops import _native as nat
    from idc_models_amd.ops import functional as fn
    ext = nat.require()
    dev = torch.device("cuda", 0)
    N = args.batch
    for H, C, S, pads in MBV2:
        Ho = (H + 2 * pads[0] - 3) // S + 1 if pads[0] else (H + 1 - 3) // S + 1
        x = (torch.randn(N, H, H, C, device=dev)).to(torch.bfloat16)
        k = torch.randn(3, 3, C, 1, device=dev) * 0.3
        st_in = torch.cat([x.float().sum((0, 1, 2)), (x.float() ** 2).sum((0, 1, 2))])
        bn = fn.BN(stats=st_in, gamma=torch.ones(C, device=dev), beta=torch.zeros(C, device=dev),
                   count=N * H * H, eps=1e-3, act=2)
        stats = torch.zeros(2 * C, device=dev)
        y = torch.empty(N, Ho, Ho, C, dtype=torch.bfloat16, device=dev)
        a = fn._dw_args(x, k, S, pads, Ho, Ho, bn)
        a.y, a.ldy = y.data_ptr(), C
        a.stats, a.stats_ld = stats.data_ptr(), C
        pf = ext.Plan()
        pf.add(nat.OP_DW_FWD, nat.raw(a), [], [], [], [])
        dy = torch.randn(N, Ho, Ho, C, device=dev).to(torch.bfloat16)
        dx = torch.empty_like(x)
        dw = torch.zeros(3, 3, C, 1, device=dev)
        gs, gx = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        b = fn._dw_args(x, k, S, pads, Ho, Ho, bn)
        b.dy, b.lddy, b.dx, b.lddx = dy.data_ptr(), C, dx.data_ptr(), C
        b.gsum, b.gsumx, b.dw = gs.data_ptr(), gx.data_ptr(), dw.data_ptr()
        ws = torch.empty(int(ext.dw_wgrad_ws_floats(N * Ho * Ho, C, 9)), device=dev)
        b.ws = ws.data_ptr()
        pb = ext.Plan()
        pb.add(nat.OP_DW_BWD_DATA, nat.raw(b), [], [], [], [])
        pw = ext.Plan()
        pw.add(nat.OP_DW_WGRAD, nat.raw(b), [], [], [], [])
        sh = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
        tf = graph_us(lambda: pf.run(0, -1, sh()))
        # the same forward without the statistics epilogue, and with 16 statistics slots
        a.stats = 0
        pn = ext.Plan()
        pn.add(nat.OP_DW_FWD, nat.raw(a), [], [], [], [])
        tn = graph_us(lambda: pn.run(0, -1, sh()))
        st16 = torch.zeros(16 * 2 * C, device=dev)
        a.stats, a.stats_slots = st16.data_ptr(), 16
        p16 = ext.Plan()
        p16.add(nat.OP_DW_FWD, nat.raw(a), [], [], [], [])
        t16 = graph_us(lambda: p16.run(0, -1, sh()))
        tb = graph_us(lambda: pb.run(0, -1, sh()))
        tw = graph_us(lambda: pw.run(0, -1, sh()))
        mb_in, mb_out = N * H * H * C * 2 / 1e6, N * Ho * Ho * C * 2 / 1e6
        print(f"H={H:2d} C={C:3d} s{S}: fwd {tf:6.1f} us ({(mb_in + mb_out) / tf:.2f} TB/s) "
              f"[no stats {tn:5.1f}, 16 slots {t16:5.1f}] | "
              f"bwd-data {tb:6.1f} us ({(2 * mb_in + mb_out) / tb:.2f} TB/s) | wgrad {tw:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
