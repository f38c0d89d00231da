"""Worker for tests/test_dp_gpu.py (launched by torch.distributed.run, 2+ ranks sharing cuda:0
over gloo: RCCL refuses two ranks on one device, so this is how the fused data-parallel path runs
on a one-GPU box; the collectives, bucket boundaries, comm stream and side-lane hand-offs are the
same code the nccl backend runs).

For each (arch, strategy) it checks, on the fused MI355X program:
  * the reduced gradient after one DP step equals the sum of the single-process fused gradients of
    the per-rank shards (local-batch BatchNorm, as MirroredStrategy: each replica normalises its
    own shard) — so bucketing, marks and the all-reduce feed the optimizer the right thing;
  * after two steps every replica holds bit-identical trainable weights.
Rank 0 prints one JSON line per configuration.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def flat(ts):
    return torch.cat([t.detach().reshape(-1).float() for t in ts])


def run_case(arch, kind, per=None):
    # DenseNet at 8 images per rank normalises its last stage over 8 rows: two runs of the SAME
    # program then differ by float-atomic summation order amplified through 120 BatchNorms, so
    # the comparison uses 32 per rank (as the fine-tune GPU test does)
    per = per or (32 if arch.startswith("densenet") else 8)
    # (under IDC_DETERMINISTIC=1 the comparison is exact at any batch)
    import torch.distributed as dist
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model
    from idc_models_amd.parallel import CentralStorageStrategy, MirroredStrategy, OneDeviceStrategy
    from idc_models_amd.parallel.strategy import current_replica_weight
    cls = CentralStorageStrategy if kind == "central" else MirroredStrategy
    st = cls(backend="gloo", device="cuda:0", bucket_bytes=2 << 20)
    rank, world = st.rank, st.world
    net = build_model(arch, None, 1, seed=7)
    m = Model(net, st)
    m.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="fused")
    g = torch.Generator().manual_seed(3)
    H, W, C = net.input_shape
    # "uneven": a global batch of world * per + 1 rows, rank 0 holding the extra one (the split
    # strategy._ShardedBatches makes); each rank's local gradient is weighted n_r * world / b
    sizes = [per + (1 if (kind == "uneven" and r == 0) else 0) for r in range(world)]
    offs = [sum(sizes[:r]) for r in range(world + 1)]
    gb = offs[-1]
    wts = [n * world / gb for n in sizes]
    x = torch.randint(0, 256, (gb, H, W, C), generator=g, dtype=torch.uint8)
    y = torch.randint(0, 2, (gb,), generator=g)
    xs, ys = x[offs[rank]:offs[rank + 1]], y[offs[rank]:offs[rank + 1]]
    current_replica_weight[0] = wts[rank]
    try:
        m.impl.train_step(xs, ys)
        torch.cuda.synchronize()
        red = m.arena.grad.detach().clone()  # the SUM the optimizer consumed (rank 0 for central)
        m.impl.train_step(xs, ys)
        torch.cuda.synchronize()
    finally:
        current_replica_weight[0] = 1.0
    w = flat(m.net.trainable_weights)
    gathered = [torch.empty_like(w) for _ in range(world)]
    dist.all_gather(gathered, w)
    same = max(float((gg - w).abs().max()) for gg in gathered)
    out = {"arch": arch, "strategy": kind, "world": world, "replica_max_diff": same,
           "buckets": len(st.bucketer(m.arena).buckets) if st.bucketer(m.arena) else 0}
    if rank == 0:
        ref = Model(build_model(arch, None, 1, seed=7), OneDeviceStrategy("cuda:0"))
        ref.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="fused")
        tot = torch.zeros_like(red)
        tot_plain = torch.zeros_like(red, dtype=torch.float64)
        for r in range(world):
            # the reference shard gradient carries the same seed weight (the weight
            # enters BEFORE the reduction), so the DP sum is exactly the shard sum in det mode
            current_replica_weight[0] = wts[r]
            try:
                p = ref.impl._prog(sizes[r], True, torch.uint8)
            finally:
                current_replica_weight[0] = 1.0
            p.reset_stats_shift()  # each rank's shard as a first step (statistics shift K = 0)
            ref.impl._stage_inputs(p, x[offs[r]:offs[r + 1]], y[offs[r]:offs[r + 1]])
            p.run_segment("fwd")
            p.run_segment("bwd")
            torch.cuda.current_stream().wait_stream(p.stream)
            torch.cuda.synchronize()
            tot += ref.arena.grad
            tot_plain += ref.arena.grad.double() / wts[r]
        d, e = red.double(), tot.double()
        out["grad_cos"] = float(d @ e / (d.norm() * e.norm() + 1e-30))
        out["grad_rel_err"] = float((d - e).norm() / (e.norm() + 1e-30))
        if kind == "uneven":
            # the replicas stay bit-identical (before, each rank scaled the same reduced
            # sum by its own weight), the reduced gradient is exactly the sum of the seed-weighted
            # shard gradients, and those differ from the unweighted sum (the weights are applied)
            out["weights"] = wts
            out["rel_err_unweighted"] = float((d - tot_plain).norm() / (tot_plain.norm() + 1e-30))
            out["ok"] = bool(same == 0.0 and out["grad_rel_err"] == 0.0 and out["rel_err_unweighted"] > 1e-3)
        elif os.environ.get("IDC_DETERMINISTIC") == "1":
            # fixed-order reductions: each rank's shard gradient is the single-process one to the
            # bit, and a two-rank sum is exactly g0 + g1
            out["ok"] = bool(same == 0.0 and out["grad_rel_err"] == 0.0)
        else:
            tol = (0.999, 0.05) if arch.startswith("vgg") else (0.99, 0.15)
            out["ok"] = bool(same == 0.0 and out["grad_cos"] > tol[0] and out["grad_rel_err"] < tol[1])
        print("DPCASE " + json.dumps(out), flush=True)
    m.impl.close()
    dist.barrier()


def main():
    cases = [c.split(":") for c in (sys.argv[1] if len(sys.argv) > 1 else
                                    "vgg16:mirrored,densenet121:mirrored,densenet121:central").split(",")]
    for arch, kind in cases:
        run_case(arch, kind)
    import torch.distributed as dist
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
