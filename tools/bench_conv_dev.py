"""Device-time microbenchmark of the conv kernels on the DenseNet-121 @50x50, bs=256 shapes.

Each measurement captures R back-to-back launches of ONE kernel configuration into a HIP graph
(through the native Plan) and times the replay with events, so the numbers are GPU time per
launch (including the ~1.5 us dependent-launch boundary), not host launch overhead.

    python tools/bench_conv_dev.py [--reps 40]
"""
import argparse
import sys

import torch

sys.path.insert(0, ".")
from idc_models_amd.ops import _native as nat  # noqa: E402
from idc_models_amd.ops import functional as fn  # noqa: E402

DEV = "cuda"


def time_plan(adds, reps):
    ext = nat.require()
    p = ext.Plan()
    for _ in range(reps):
        for a in adds:
            p.add(*a)
    s = torch.cuda.Stream()
    g = p.capture(0, -1, s.cuda_stream)
    p.launch(g, s.cuda_stream)
    s.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(3):
        p.launch(g, s.cuda_stream)
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / (3 * reps) * 1e3


_WS = {}


def conv_op(x, w_layout, N, H, W, Cin, Cout, k, pads, pro, stats, tile, y, ks=1):
    a = nat.ConvArgs()
    a.x = x.data_ptr()
    a.N, a.H, a.W, a.Cin, a.ldx = N, H, W, Cin, Cin
    a.Ho, a.Wo, a.Cout = H, W, Cout
    a.y, a.ldy = y.data_ptr(), Cout
    a.w = w_layout.data_ptr()
    a.KH, a.KW, a.SH, a.SW = k, k, 1, 1
    a.PT, a.PL = pads
    a.pro = pro.args() if pro is not None else nat.bn_args(mode=0, act=0)
    a.epi_mode = 0
    a.bias = 0
    a.epi_act = 0
    a.out_mode = nat.OUT_BF16
    if stats is not None:
        a.stats_out, a.stats_ld, a.stats_off = stats.data_ptr(), Cout, 0
    a.mbn = nat.bn_args(mode=0, act=0)
    if ks > 1:
        if "slab" not in _WS:
            _WS["slab"] = torch.empty(1 << 24, device=DEV)
        t = torch.zeros(1 << 16, dtype=torch.int32, device=DEV)
        _WS.setdefault("t", []).append(t)
        a.slab, a.tickets = _WS["slab"].data_ptr(), t.data_ptr()
        a.slab_floats, a.tickets_n = _WS["slab"].numel(), t.numel()
    return (nat.OP_CONV, nat.raw(a), [tile, 0, ks], [], [], [], 0)


def wgrad_op(x, dy, N, H, W, Cin, Cout, k, pads, pro, dw, splits):
    a = nat.WgradArgs()
    a.x = x.data_ptr()
    a.N, a.H, a.W, a.Cin, a.ldx = N, H, W, Cin, Cin
    a.g, a.ldg = dy.data_ptr(), Cout
    a.Ho, a.Wo, a.Cout = H, W, Cout
    a.KH, a.KW, a.SH, a.SW = k, k, 1, 1
    a.PT, a.PL = pads
    a.pro = pro.args() if pro is not None else nat.bn_args(mode=0, act=0)
    a.dw = dw.data_ptr()
    a.scale = 1.0
    a.cin_real = 0
    return (nat.OP_WGRAD, nat.raw(a), [splits, 0], [], [], [], 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--wgrad", action="store_true")
    args = ap.parse_args()
    ext = nat.require()
    N = 256
    cases = [("1x1 64->128 13x13", 13, 64, 128, 1), ("1x1 224->128 13x13", 13, 224, 128, 1),
             ("3x3 128->32 13x13", 13, 128, 32, 3), ("1x1 480->128 6x6", 6, 480, 128, 1),
             ("3x3 128->32 6x6", 6, 128, 32, 3), ("1x1 992->128 3x3", 3, 992, 128, 1),
             ("3x3 128->32 3x3", 3, 128, 32, 3), ("1x1 1000->128 1x1", 1, 1000, 128, 1),
             ("3x3 128->32 1x1", 1, 128, 32, 3)]
    for name, H, cin, cout, k in cases:
        cin = (cin + 7) // 8 * 8
        x = torch.randn(N, H, H, cin, device=DEV).to(torch.bfloat16)
        w = torch.randn(k, k, cin, cout, device=DEV) * 0.05
        st = torch.cat([x.float().sum((0, 1, 2)), (x.float() ** 2).sum((0, 1, 2))])
        bn = fn.BN(stats=st, gamma=torch.ones(cin, device=DEV), beta=torch.zeros(cin, device=DEV),
                   count=N * H * H, eps=1e-3, act=1)
        sout = torch.zeros(2 * cout, device=DEV)
        y = torch.empty(N, H, H, cout, device=DEV, dtype=torch.bfloat16)
        wl = fn.weight_fwd_layout(w, cin)
        pads = (k // 2, k // 2)
        flops = 2.0 * N * H * H * cout * k * k * cin
        res = []
        for t in range(ext.num_tiles()):
            if ext.tile_bn(t) > max(32, cout):
                continue
            us = time_plan([conv_op(x, wl, N, H, H, cin, cout, k, pads, bn, sout, t, y)], args.reps)
            us0 = time_plan([conv_op(x, wl, N, H, H, cin, cout, k, pads, None, None, t, y)], args.reps)
            us1 = time_plan([conv_op(x, wl, N, H, H, cin, cout, k, pads, bn, None, t, y)], args.reps)
            us2 = time_plan([conv_op(x, wl, N, H, H, cin, cout, k, pads, None, sout, t, y)], args.reps)
            res.append((us, t, us0, us1, us2))
        res.sort()
        b = res[0]
        print(f"{name:22s} M={N * H * H:6d} best t{b[1]:2d}: {b[0]:6.1f} us ({flops / b[0] / 1e6:6.1f} TF/s) "
              f"plain {b[2]:6.1f} pro-only {b[3]:6.1f} stats-only {b[4]:6.1f} | " +
              " ".join(f"t{t}:{u:.1f}/{u0:.1f}/{u1:.1f}/{u2:.1f}" for u, t, u0, u1, u2 in res[:6]), flush=True)
        for t in sorted({b[1], 4, 9, 12, 17}):
            if ext.tile_bn(t) > max(32, cout):
                continue
            row = []
            tiles = -(-(N * H * H) // ext.tile_bm(t)) * -(-cout // ext.tile_bn(t))
            for ks in (1, 2, 4, 8):
                if ks > 1 and tiles * ks * ext.tile_bm(t) * ext.tile_bn(t) > (1 << 24):
                    continue
                us = time_plan([conv_op(x, wl, N, H, H, cin, cout, k, pads, None, None, t, y, ks)], args.reps)
                us2 = time_plan([conv_op(x, wl, N, H, H, cin, cout, k, pads, bn, sout, t, y, ks)], args.reps)
                row.append(f"ks{ks}:{us:.1f}/{us2:.1f}")
            print(f"    split-K t{t:2d} plain/full " + " ".join(row), flush=True)
        if args.wgrad:
            dy = torch.randn(N, H, H, cout, device=DEV).to(torch.bfloat16)
            dw = torch.zeros(k * k * cin * cout, device=DEV)
            out = []
            for s in (1, 4, 16, 64, 256):
                us = time_plan([wgrad_op(x, dy, N, H, H, cin, cout, k, pads, bn, dw, s)], args.reps)
                out.append(f"s{s}:{us:.1f}")
            print("    wgrad " + " ".join(out), flush=True)


if __name__ == "__main__":
    main()
