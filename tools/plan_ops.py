"""Isolated device time of every op of a built training plan (one HIP graph of R launches of the
op, timed with events), with its shape, tile / split choice and lane.  Complements the rocprof
timeline: that shows the critical path in situ, this shows what each launch costs on its own.

    python tools/plan_ops.py [--model densenet121] [--batch 256] [--reps 20] [--seg bwd]
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from idc_models_amd.ops import _native as nat  # noqa: E402


def describe(plan, i):
    k = plan.kind(i)
    name = plan.describe(i)
    if k == nat.OP_CONV:
        a = nat.ConvArgs.from_buffer_copy(plan.payload(i))
        M = a.N * a.Ho * a.Wo
        pro = 2 if a.bpro.mode else int(a.pro.mode != 0 or a.pro.act != 0)
        return (f"{name} {a.KH}x{a.KW} M={M} K={a.KH * a.KW * a.Cin} N={a.Cout} pro={pro} epi={a.epi_mode} "
                f"f32={plan.get_int(i, 1)} tile={plan.get_int(i, 0)} ks={plan.get_int(i, 2)}")
    if k == nat.OP_WGRAD:
        a = nat.WgradArgs.from_buffer_copy(plan.payload(i))
        M = a.N * a.Ho * a.Wo
        return (f"{name} {a.KH}x{a.KW} P={M} K={a.KH * a.KW * a.Cin} N={a.Cout} gpro={int(a.gpro.mode != 0)} "
                f"f32={plan.get_int(i, 1)} splits={plan.get_int(i, 0)}")
    return name


def time_op(plan, i, stream, reps):
    """Back-to-back direct issue of the op (a one-node graph replay pays ~10 us of host floor per
    launch, more than most of these kernels): device time per launch incl. the ~1.5 us boundary;
    ops shorter than the ~3.5 us host issue cost read as that cost."""
    sh = stream.cuda_stream
    plan.run(i, i + 1, sh)
    stream.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        plan.run(i, i + 1, sh)
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="densenet121")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--seg", default="fwd,bwd,opt")
    ap.add_argument("--alt", default="", help="comma list of extra conv tiles to time on every eligible op "
                                             "(img, rows): printed beside the tuned choice")
    a = ap.parse_args()
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model
    dev = torch.device("cuda", 0)
    net = build_model(a.model, num_outputs=1, seed=0)
    m = Model(net, device=dev)
    m.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="fused")
    H, W, C = net.input_shape
    x = torch.randint(0, 256, (a.batch, H, W, C), dtype=torch.uint8, device=dev)
    y = torch.randint(0, 2, (a.batch,), device=dev)
    m.impl.train_step(x, y)
    torch.cuda.synchronize()
    p = m.impl._prog(a.batch, True, torch.uint8)
    plan, st = p.plan, p.stream
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for seg in a.seg.split(","):
        if seg not in p.seg:
            continue
        lo, hi = p.seg[seg]
        print(f"== {seg} ops {lo}..{hi}")
        for i in range(lo, hi):
            us = time_op(plan, i, st, a.reps)
            lane = plan.lane(i)
            d = describe(plan, i)
            alt = ""
            if a.alt and plan.kind(i) == nat.OP_CONV:
                ext = nat.load()
                t0, f32 = plan.get_int(i, 0), plan.get_int(i, 1)
                for name in a.alt.split(","):
                    tile, ok = {"img": (ext.TILE_IMG, ext.img_ok)}[name]
                    if ok(plan.payload(i), f32) and t0 != tile:
                        plan.set_int(i, 0, tile)
                        p.b.reset_tickets()
                        alt += f"  [{name} {time_op(plan, i, st, a.reps):.2f} us]"
                        plan.set_int(i, 0, t0)
                p.b.reset_tickets()
            print(f"{i:4d} {seg} L{lane} {us:8.2f} us  {d}{alt}", flush=True)
            key = (seg, lane, d.split(" ")[0] + (" " + " ".join(w for w in d.split(" ") if w.startswith(("pro=", "epi=", "gpro="))) if d.startswith(("conv", "wgrad")) else ""))
            tot[key] += us
            cnt[key] += 1
    print("== totals (isolated, includes ~1.5 us launch boundary each)")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"{k[0]} L{k[1]} {v:9.1f} us {cnt[k]:4d}x  {k[2]}")


if __name__ == "__main__":
    main()
