"""Row-resident dense stage (dense_rows.hip) vs the work-queue launch on small shapes: per-row max
error of each layer's slice (debugging aid).  usage: python tools/dense_rows_debug.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from idc_models_amd.ops import functional as fn  # noqa: E402

DEV = torch.device("cuda", 0)


def run(N, H, c0, L, rb, rows):
    os.environ["IDC_DS_ROWS_RB"] = str(rb)
    g = torch.Generator().manual_seed(5)
    ld = c0 + 32 * L
    buf = torch.zeros(N, H, H, ld)
    buf[..., :c0] = torch.randn(N, H, H, c0, generator=g)
    buf = buf.to(torch.bfloat16).to(DEV)
    x0 = buf[..., :c0].float().reshape(-1, c0)
    sst = torch.zeros(2 * ld, device=DEV)
    sst[:c0], sst[ld:ld + c0] = x0.sum(0), (x0 * x0).sum(0)
    k2 = 1 if H == 1 else 3
    lays = []
    for i in range(L):
        cin = c0 + 32 * i
        w1 = (torch.randn(1, 1, cin, 128, generator=g) * (2.0 / cin) ** 0.5).to(DEV)
        w2 = (torch.randn(3, 3, 128, 32, generator=g) * (2.0 / 1152) ** 0.5).to(DEV)
        lays.append(dict(w1=fn.weight_fwd_layout(w1, cin), w2=fn.weight_fwd_layout(w2[1:2, 1:2] if k2 == 1 else w2, 128),
                         g1=torch.ones(cin, device=DEV), b1=torch.zeros(cin, device=DEV),
                         g2=torch.ones(128, device=DEV), b2=torch.zeros(128, device=DEV),
                         t=torch.zeros(N, H, H, 128, dtype=torch.bfloat16, device=DEV),
                         tstats=torch.zeros(256, device=DEV), tshift=None, eps1=1e-5, eps2=1e-5, cin=cin))
    sync, err, _ = fn.dense_stage(buf, sst, lays, grid=256, k2=k2, rows=rows)
    return buf.float(), [d["t"].float() for d in lays], int(err[0]), [d["tstats"].clone() for d in lays], sst.clone(), lays


for (N, H, c0, L) in [(1, 5, 32, 1), (3, 5, 32, 2), (2, 4, 32, 1), (4, 3, 64, 2), (2, 5, 64, 1)]:
    for rb in (1, 2):
        ok, r, ipg, G = fn.nat.require().dense_rows_geometry(N, H, H, c0 + 32 * L, c0 + 32 * (L - 1)) \
            if (os.environ.__setitem__("IDC_DS_ROWS_RB", str(rb)) or True) else None
        if not ok:
            print(f"N{N} H{H} c0 {c0} L{L} rb{rb}: geometry refused")
            continue
        b0, t0, e0, ts0, ss0, l0 = run(N, H, c0, L, rb, 0)
        b1, t1, e1, ts1, ss1, l1 = run(N, H, c0, L, rb, 1)
        # torch: slice 0 from the kernel's own t with BN2 from its batch statistics
        t = t1[0].reshape(-1, 128)
        mu, var = t.mean(0), t.var(0, unbiased=False)
        a2 = torch.relu((t - mu) * torch.rsqrt(var + 1e-5)).reshape(N, H, H, 128).to(torch.bfloat16).float()
        w2 = l1[0]["w2"].float().reshape(32, 3 if H > 1 else 1, 3 if H > 1 else 1, 128).permute(0, 3, 1, 2)
        y = torch.nn.functional.conv2d(a2.permute(0, 3, 1, 2), w2, padding=1 if H > 1 else 0).permute(0, 2, 3, 1)
        ye = lambda b: float((b[..., c0:c0 + 32] - y).abs().max())
        print(f"   tstats diff {float((ts1[0] - ts0[0]).abs().max()):.4g} (vs torch {float((ts1[0][:128] - t.sum(0)).abs().max()):.4g}); "
              f"slice0 vs torch: rows {ye(b1):.4g} queue {ye(b0):.4g}", flush=True)
        d = (b1 - b0).abs().reshape(N * H * H, -1)
        rows_bad = [int(i) for i in torch.nonzero(d.amax(1) > 0.05).flatten()[:40]]
        cols_bad = [int(i) for i in torch.nonzero(d.amax(0) > 0.05).flatten()[:40]]
        terr = [float((a - b).abs().max()) for a, b in zip(t1, t0)]
        print(f"N{N} H{H} c0 {c0} L{L} rb{rb} ipg{ipg} G{G}: err {e0},{e1} t maxdiff {terr} bad rows {rows_bad} "
              f"bad cols {cols_bad}", flush=True)
