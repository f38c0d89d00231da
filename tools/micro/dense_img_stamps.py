"""Phase stamps of the per-image training launch (csrc/kernels/dense_infer.hip dense_img_fwd) at
DenseNet-121's stage-1 / stage-2 bench shapes: median microseconds per layer phase over workgroups.
Phases: 0->1 GEMM1 (+ t moments), 1->2 t store + publish, 2->3 barrier 1, 3->4 BN2 table + pass,
4->5 GEMM2, 5->6 slice moments + publish, 6->7 barrier 2 + next BN1 table, 7->next 0 loop."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from idc_models_amd.ops import functional as fn  # noqa: E402


def run(N, H, c0, L):
    dev = "cuda"
    ld = c0 + 32 * L
    g = torch.Generator().manual_seed(1)
    buf = torch.zeros(N, H, H, ld)
    buf[..., :c0] = torch.randn(N, H, H, c0, generator=g)
    buf = buf.to(torch.bfloat16).to(dev)
    x0 = buf[..., :c0].float().reshape(-1, c0)
    sst = torch.zeros(2 * ld, device=dev)
    sst[:c0], sst[ld:ld + c0] = x0.sum(0), (x0 * x0).sum(0)
    lays = []
    for i in range(L):
        cin = c0 + 32 * i
        lays.append(dict(w1=(torch.randn(128, cin, generator=g) * 0.05).to(torch.bfloat16).to(dev),
                         w2=(torch.randn(32, 9 * 128, generator=g) * 0.03).to(torch.bfloat16).to(dev),
                         g1=torch.ones(cin, device=dev), b1=torch.zeros(cin, device=dev),
                         g2=torch.ones(128, device=dev), b2=torch.zeros(128, device=dev),
                         t=torch.zeros(N, H, H, 128, dtype=torch.bfloat16, device=dev),
                         tstats=torch.zeros(256, device=dev), eps1=1e-5, eps2=1e-5, cin=cin))
    for _ in range(3):
        sst2 = sst.clone()
        _, err, st = fn.dense_stage(buf, sst2, lays, rows=2, stamps=True)
    G = -(-N // -(-N // 256))
    st = st.reshape(L, 256, 8)[:, :G].double() / 100.0  # 100 MHz -> us
    names = ["gemm1", "t-store+pub", "barrier1", "bn2", "gemm2", "mom+pub", "barrier2+bn1", "loop"]
    print(f"N={N} H={H} c0={c0} L={L} grid={G} err={int(err[0])}")
    tot = (st[-1, :, 5] - st[0, :, 0]).median().item()
    print(f"  layer 0 start -> last layer GEMM2 end: {tot:.1f} us (median over workgroups)")
    for k in range(7):
        d = (st[:-1, :, k + 1] - st[:-1, :, k]).median().item()
        print(f"  {names[k]:14s} {d:7.2f} us")
    d = (st[1:, :, 0] - st[:-1, :, 7]).median().item()
    print(f"  {names[7]:14s} {d:7.2f} us")
    skew = (st[:, :, 2].max(1).values - st[:, :, 2].min(1).values).median().item()
    print(f"  publish-1 spread across workgroups: {skew:.2f} us")


run(256, 13, 64, 6)
run(256, 6, 128, 12)
