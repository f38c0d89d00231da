#!/usr/bin/env python3
"""Headline benchmark: DenseNet-121 50x50x3 training, bs=256 per GPU, bf16, data-parallel.

Metric (BASELINE.json): images/sec for the WHOLE job (all ranks), DenseNet-121 at 50x50x3,
batch 256 per GPU, weak scaling over 1/2/4/8 MI355X.  Synthetic uint8 patches of that shape and
random-init weights (no network on the box).  The timed region is the complete training step:
input staging, forward, loss, backward, bucketed RCCL gradient all-reduce (N>1), fused RMSprop
update and bf16 weight re-cast — nothing skipped.

    python bench.py                     # 1 GPU, defaults
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8

``vs_baseline`` is relative to the in-situ stock PyTorch-ROCm measurement recorded in
BASELINE.md (the reference publishes no number): 9,379 img/s per GPU x N.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

STOCK_PYTORCH_IMG_S_PER_GPU = {"densenet121": 9379.3, "vgg16": 58586.2, "mobilenetv2": 19653.8}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="densenet121")
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--backend", default="fused")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model
    from idc_models_amd.parallel import MirroredStrategy, OneDeviceStrategy
    from idc_models_amd.parallel.comm import all_reduce_max, barrier

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and os.environ.get("IDC_BENCH_REHEARSE") == "1":
        # rehearsal of the N>1 path on a one-GPU box: every rank on cuda:0, gloo collectives
        # (RCCL refuses two ranks on one device); numbers from this mode are not throughput
        strategy = MirroredStrategy(backend="gloo", device="cuda:0")
    elif world > 1:
        strategy = MirroredStrategy()
    else:
        strategy = OneDeviceStrategy("cuda:0")
    rank = strategy.rank
    dev = strategy.device
    torch.manual_seed(1234)

    with strategy.scope():
        net = build_model(args.model, num_outputs=1, seed=1234)
        model = Model(net, strategy)
        model.compile(RMSprop(args.lr), "binary_crossentropy", ["accuracy"], backend=args.backend,
                      **({"use_graphs": False} if args.no_graphs and args.backend == "fused" else {}))
    H, W, C = net.input_shape
    g = torch.Generator(device="cpu").manual_seed(1000 + rank)
    x = torch.randint(0, 256, (args.batch, H, W, C), generator=g, dtype=torch.uint8).to(dev)
    y = torch.randint(0, 2, (args.batch,), generator=g).to(dev)

    step = model.impl.train_step
    for _ in range(args.warmup):
        loss, _ = step(x, y)
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss, _ = step(x, y)
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    dt = all_reduce_max(dt, dev) if world > 1 else dt
    ms = dt / args.steps * 1e3
    total_imgs = args.batch * world * args.steps
    value = total_imgs / dt
    base = STOCK_PYTORCH_IMG_S_PER_GPU.get(args.model)
    lossv = float(loss.item())
    if rank == 0:
        print(json.dumps({
            "metric": "images/sec (whole node) DenseNet-121 50x50x3 bs=256 at 1/2/4/8 MI355X"
            if args.model == "densenet121" else f"images/sec (whole node) {args.model} 50x50x3",
            "value": round(value, 1),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / (base * world), 3) if base else None,
            "dtype": "bf16",
            "data": "synthetic uint8 50x50x3 patches, random-init weights",
            "config": {"model": "DenseNet-121" if args.model == "densenet121" else args.model,
                       "global_batch": args.batch * world, "seq_len": None,
                       "input": [H, W, C], "per_gpu_batch": args.batch,
                       "parallelism": f"dp{world}", "optimizer": "RMSprop(lr=%g)" % args.lr,
                       "loss": "BCE(from_logits)", "final_loss": round(lossv, 5),
                       "backend": args.backend},
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
