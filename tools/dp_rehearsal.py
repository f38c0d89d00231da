"""Rehearse the fused data-parallel path on ONE GPU: N gloo ranks share cuda:0.

    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 tools/dp_rehearsal.py [ARCH] [B] [mirrored|central]

Each rank trains the fused program on its half of a fixed global batch with bucketed
all-reduces issued between backward segments; rank 0 then runs the single-process reference on
the whole batch.  Checks: replicas stay bit-identical, and the DP update equals the
single-process update (VGG16 has no BatchNorm, so the two are the same computation up to bf16
rounding / summation order).  Prints one JSON line.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    arch = sys.argv[1] if len(sys.argv) > 1 else "vgg16"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    kind = sys.argv[3] if len(sys.argv) > 3 else "mirrored"
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model
    from idc_models_amd.parallel import CentralStorageStrategy, MirroredStrategy, OneDeviceStrategy
    import torch.distributed as dist
    cls = CentralStorageStrategy if kind == "central" else MirroredStrategy
    st = cls(backend="gloo", device="cuda:0", bucket_bytes=4 << 20)
    rank, world = st.rank, st.world
    net = build_model(arch, None, 1, seed=7)
    w0 = [t.detach().clone() for t in net.trainable_weights]
    m = Model(net, st)
    m.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="fused")
    g = torch.Generator().manual_seed(3)
    H, W, C = net.input_shape
    x = torch.randint(0, 256, (B, H, W, C), generator=g, dtype=torch.uint8)
    y = torch.randint(0, 2, (B,), generator=g)
    per = B // world
    xs, ys = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]
    steps = 2
    for _ in range(steps):
        m.impl.train_step(xs, ys)
    torch.cuda.synchronize()
    flat = torch.cat([t.detach().reshape(-1) for t in m.net.trainable_weights])
    gathered = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    same = max(float((gg - flat).abs().max()) for gg in gathered)
    bk = m.strategy.bucketer(m.arena)
    out = {"world": world, "arch": arch, "strategy": kind, "replica_max_diff": same,
           "buckets": len(bk.buckets) if bk is not None else 0, "bwd_marks": None}
    if rank == 0:
        p = m.impl._prog(per, True, torch.uint8)
        out["bwd_marks"] = len(p.bwd_marks)
        ref_net = build_model(arch, None, 1, seed=7)
        ref = Model(ref_net, OneDeviceStrategy("cuda:0"))
        ref.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="fused")
        for _ in range(steps):
            ref.impl.train_step(x, y)
        torch.cuda.synchronize()
        rflat = torch.cat([t.detach().reshape(-1) for t in ref.net.trainable_weights])
        base = torch.cat([t.reshape(-1) for t in w0]).to(rflat.device)
        du, dr = (flat - base).double(), (rflat - base).double()
        out["update_cosine"] = float(du @ dr / (du.norm() * dr.norm() + 1e-30))
        out["update_rel_err"] = float((du - dr).norm() / (dr.norm() + 1e-30))
        out["ok"] = bool(same == 0.0 and out["update_cosine"] > 0.98)
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
