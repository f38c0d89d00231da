#!/usr/bin/env python3
"""Headline benchmark: DenseNet-121 50x50x3 training, bs=256 per GPU, bf16, data-parallel.

Metric (BASELINE.json): images/sec for the WHOLE job (all ranks), DenseNet-121 at 50x50x3,
batch 256 per GPU, weak scaling over 1/2/4/8 MI355X; plus validation AUC.  Synthetic uint8
patches of that shape and random-init weights (no network on the box).

* ``value`` — the timed region is the complete training step on a device-resident batch: input
  staging, forward, loss, backward, bucketed RCCL gradient all-reduce (N>1), fused RMSprop update
  and bf16 weight re-cast — nothing skipped.  W warm-up steps, then exactly K steps between
  barrier + synchronize on both sides, max over ranks.
* ``fit_images_per_sec`` — after the timed region: ``Model.fit`` throughput on a host-resident
  learnable synthetic dataset (pinned-memory prefetcher, per-rank index sharding, metrics),
  training epochs only.
* ``val_auc`` — exact (Mann-Whitney) AUC of ``Model.evaluate`` on a held-out synthetic set after
  that fit (``secure_fed_model.py:81-82`` reports AUC; here over the whole set, not per batch).

    python bench.py                     # 1 GPU, defaults
    python bench.py --gpus 8            # starts 8 rank processes itself (torch.distributed.run)
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8

With ``--gpus N`` (N > 1) and no launcher environment (``WORLD_SIZE`` unset), bench.py starts the N
rank processes itself through ``torch.distributed.run`` before anything touches the GPU and exits
with their status; every rank refuses to run (exit 3) when the world it joined is not N.  On a GPU
the ranks talk over RCCL: the fused step's gradient buckets are all-reduced by the native
communicator from inside the C++ plan (``parallel/native_comm.py``).

``vs_baseline`` is relative to the in-situ stock PyTorch-ROCm measurement committed in
``benchmarks/stock_baseline.json`` (the reference publishes no number): the faster of
its eager and HIP-graph-captured steps, per GPU, times N.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n: int) -> int:
    """Start ``n`` rank processes of this script (one per GPU) and return their exit status.  The
    parent never initialises the GPU; the children are started as new processes (no exec)."""
    import subprocess
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def check_world(expected: int, got: int):
    if got != expected:
        print(json.dumps({"error": f"--gpus {expected} but the job has {got} rank(s)"}), flush=True)
        sys.exit(3)


def rccl_version_of(strategy):
    nc = getattr(strategy, "native_comm", None)
    if nc is not None:
        return nc.version()
    try:
        import torch
        return ".".join(str(v) for v in torch.cuda.nccl.version())
    except Exception:  # pragma: no cover - version query unsupported
        return "unknown"


def stock_img_s_per_gpu(model: str, size: int = 50, classes: int = 1, phase: str = "full"):
    """Best stock PyTorch-ROCm images/sec on one GPU for ``model`` at this input size / class
    count / training phase (benchmarks/stock_baseline.json; entries without those keys are the
    default 50x50x3, 1 logit, every layer trained)."""
    p = os.path.join(ROOT, "benchmarks", "stock_baseline.json")
    try:
        with open(p) as f:
            runs = json.load(f)
    except (OSError, ValueError):
        return None
    vals = [r["images_per_sec"] for r in runs.get("results", []) if r.get("model") == model
            and r.get("input", [50])[0] == size and r.get("classes", 1) == classes
            and r.get("phase", "full") == phase]
    return max(vals) if vals else None


def fed_bench(args):
    """Configs #4 / #5: FedAvg rounds (MobileNetV2) or secure-aggregation FedAvg rounds (DenseNet-121)
    with ``--clients`` simulated clients spread over the ranks (one process per GPU), each holding
    ``--client-size`` synthetic 50x50x3 patches trained for one local epoch at ``--client-batch``
    (``fed_model.py:47-61``: 3,000 examples per client, batch 32).  One untimed warm-up round, then
    ``--rounds`` timed rounds between barrier + synchronize; max over ranks."""
    import torch
    import torch.distributed as dist

    from idc_models_amd.data import contiguous_clients, synthetic_dataset
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.fed import build_federated_averaging_process
    from idc_models_amd.models import build_model
    from idc_models_amd.parallel import OneDeviceStrategy, comm

    rank, world, local = comm.init_process_group()
    check_world(args.gpus, world)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    # config #4 backbone MobileNetV2, config #5 DenseNet-121 (--model overrides for fedavg only)
    arch = "densenet121" if args.mode == "secure" else (
        "mobilenetv2" if args.model == "densenet121" else args.model)
    base = build_model(arch, None, 1, seed=1234)
    mine = [k for k in range(args.clients) if k % world == rank]
    ds = synthetic_dataset(args.client_size * len(mine), (50, 50, 3), 2, seed=100 + rank)
    parts = contiguous_clients(ds, len(mine), args.client_size)
    clients = [None] * args.clients  # only this rank's clients are materialised
    for k, c in zip(mine, parts):
        clients[k] = c.batch(args.client_batch, True, 1000, True, seed=k)

    import copy

    def model_fn():
        return Model(copy.deepcopy(base), OneDeviceStrategy(dev))

    proc = build_federated_averaging_process(
        model_fn, lambda: RMSprop(1e-4), average_bn_stats=True, backend=args.backend,
        secure_aggregation="mask" if args.mode == "secure" else None,
        concurrent_clients=args.concurrent_clients, client_batching=bool(args.client_batching))
    state = proc.initialize()
    state, _ = proc.next(state, clients)  # warm-up: builds and tunes the client program
    torch.cuda.synchronize(dev)
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(args.rounds):
        state, metrics = proc.next(state, clients)
    torch.cuda.synchronize(dev)
    comm.barrier()
    dt = time.perf_counter() - t0
    dt = comm.all_reduce_max(dt, dev) if world > 1 else dt
    spr = dt / args.rounds
    imgs = args.clients * (args.client_size // args.client_batch) * args.client_batch
    if rank == 0:
        print(json.dumps({
            "metric": ("seconds/round FedAvg MobileNetV2" if args.mode == "fedavg"
                       else "seconds/round secure-aggregation FedAvg DenseNet-121") +
                      f" 50x50x3, {args.clients} clients x {args.client_size} examples, batch {args.client_batch}",
            "value": round(spr, 4), "unit": "seconds/round", "n_gpus": world, "steps": args.rounds,
            "warmup": 1, "higher_is_better": False, "scaling": "strong", "vs_baseline": None,
            "dtype": "bf16", "data": "synthetic uint8 50x50x3 patches, random-init weights",
            "client_images_per_sec": round(imgs / spr, 1),
            "train_loss": round(float(metrics["loss"]), 5),
            "train_metrics": {k: float(v) for k, v in metrics.items()},
            "config": {"model": arch, "clients": args.clients, "concurrent_clients": args.concurrent_clients,
                       "client_batching": bool(args.client_batching and proc._grouped is not None),
                       "client_size": args.client_size,
                       "client_batch": args.client_batch, "local_epochs": 1,
                       "client_optimizer": "RMSprop(lr=1e-4)", "server_optimizer": "SGD(lr=1.0)",
                       "aggregation": "DH-keyed additive masks, int32 all-reduce" if args.mode == "secure"
                       else "example-weighted mean, packed all-reduce",
                       "parallelism": f"clients over {world} rank(s)", "backend": args.backend,
                       "comm_backend": dist.get_backend() if world > 1 else None,
                       "world_size": world},
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="densenet121")
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--input", type=int, default=None, help="square input size (default: the model's, 50)")
    ap.add_argument("--classes", type=int, default=1,
                    help="logits: 1 = binary IDC head (BCE); >1 = softmax head (categorical CE), "
                         "e.g. --model densenet201 --input 32 --classes 10 (dist_model_tf_dense.py)")
    ap.add_argument("--phase", default="full", choices=["full", "frozen", "finetune"],
                    help="frozen: reference phase 1 (base_model.trainable = False, head only); "
                         "finetune: phase 2 (layers[:fine_tune_at] frozen, 150 DenseNet / 100 "
                         "MobileNetV2 / 15 VGG16, lr/10); full: every layer trains (the headline)")
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--backend", default="fused")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: config #1 (MobileNetV2 on CPU, world_size 1, eager backend)")
    # ~320 fit steps: Keras BatchNorm momentum 0.99 leaves the inference-mode moving statistics
    # mostly at their init after a few dozen steps (0.99^36 = 0.70), so a short fit evaluates stale
    # statistics; 0.99^320 = 0.04
    ap.add_argument("--fit-steps", type=int, default=20, help="global batches per fit epoch (0: skip fit/AUC)")
    ap.add_argument("--fit-epochs", type=int, default=None,
                    help="default: enough epochs for the BatchNorm moving statistics to forget their "
                         "Keras init (momentum^updates < 1e-2), at least 48")
    ap.add_argument("--mode", default="train", choices=["train", "fedavg", "secure"],
                    help="train: the headline DP step; fedavg / secure: north-star configs #4 / #5")
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--client-size", type=int, default=3000)
    ap.add_argument("--client-batch", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--concurrent-clients", type=int, default=2,
                    help="without client batching: clients a rank trains at once, each on its own "
                         "worker model and stream")
    ap.add_argument("--client-batching", type=int, default=1,
                    help="1: a rank's clients run in lockstep through ONE grouped program "
                         "(fed/grouped.py); 0: one client program at a time")
    ap.add_argument("--force-collectives", action="store_true",
                    help="run the RCCL data-parallel path (native bucket all-reduces) even on one GPU")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    if args.force_collectives:
        os.environ["IDC_FORCE_COLLECTIVES"] = "1"
    if args.mode != "train":
        return fed_bench(args)

    import torch
    import torch.distributed as dist

    from idc_models_amd.data import synthetic_dataset
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.engine.callbacks import ThroughputMeter
    from idc_models_amd.models import build_model
    from idc_models_amd.parallel import MirroredStrategy, OneDeviceStrategy
    from idc_models_amd.parallel.comm import all_reduce_max, barrier

    world = int(os.environ.get("WORLD_SIZE", "1"))
    check_world(args.gpus, world)
    forced = os.environ.get("IDC_FORCE_COLLECTIVES", "0") == "1"
    if world > 1 and os.environ.get("IDC_BENCH_REHEARSE") == "1":
        # rehearsal of the N>1 path on a one-GPU box: every rank on cuda:0, gloo collectives
        # (RCCL refuses two ranks on one device); numbers from this mode are not throughput
        strategy = MirroredStrategy(backend="gloo", device="cuda:0")
    elif args.device == "cpu" and world > 1:
        strategy = MirroredStrategy(backend="gloo", device="cpu")
        args.backend = "eager"
    elif world > 1 or (forced and args.device == "cuda"):
        strategy = MirroredStrategy(force_collectives=forced)
    elif args.device == "cpu":
        strategy = OneDeviceStrategy("cpu")
        args.backend = "eager"
    else:
        strategy = OneDeviceStrategy("cuda:0")
    rank = strategy.rank
    dev = strategy.device
    comm_backend = dist.get_backend() if strategy.active else None
    world = strategy.num_replicas_in_sync
    check_world(args.gpus, world)
    rccl = rccl_version_of(strategy) if comm_backend == "nccl" else None
    torch.manual_seed(1234)

    size = args.input or 50
    if args.phase == "finetune":
        args.lr /= 10  # the reference recompiles phase 2 with base_learning_rate / 10
    with strategy.scope():
        net = build_model(args.model, (size, size, 3) if args.input else None, num_outputs=args.classes, seed=1234)
        if args.phase == "frozen":
            net.base.trainable = False
        elif args.phase == "finetune":
            from idc_models_amd.recipes.transfer import fine_tune_at_for
            net.base.trainable = True
            for layer in net.base.layers[:fine_tune_at_for(args.model)]:  # VGG16 15, MBv2 100, DN 150
                layer.trainable = False
        model = Model(net, strategy)
        binary = args.classes == 1
        model.compile(RMSprop(args.lr), "binary_crossentropy" if binary else "categorical_crossentropy",
                      ["accuracy", "auc"] if binary else ["accuracy"], backend=args.backend,
                      **({"use_graphs": False} if args.no_graphs and args.backend == "fused" else {}))
    H, W, C = net.input_shape
    g = torch.Generator(device="cpu").manual_seed(1000 + rank)
    x = torch.randint(0, 256, (args.batch, H, W, C), generator=g, dtype=torch.uint8).to(dev)
    y = torch.randint(0, max(2, args.classes), (args.batch,), generator=g).to(dev)

    step = model.impl.train_step

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        loss, _ = step(x, y)
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss, _ = step(x, y)
    sync()
    barrier()
    sync()
    dt = time.perf_counter() - t0
    dt = all_reduce_max(dt, dev) if strategy.active else dt
    ms = dt / args.steps * 1e3
    total_imgs = args.batch * world * args.steps
    value = total_imgs / dt
    lossv = float(loss.item())

    # ---- after the timed region: fit() throughput and held-out validation AUC ----------------
    fit_ips = val_auc = val_acc = None
    if args.fit_epochs is None:
        # evaluate() uses the moving statistics (Keras inference BN): with MobileNetV2's momentum
        # 0.999 they keep 38% of their init after 960 updates and the held-out output collapses to
        # a constant, in the eager reference backend as much as in the fused one
        moms = [l.momentum for l in net.base.layers if getattr(l, "keras_class", "") == "BatchNormalization"]
        need = math.ceil(math.log(1e-2) / math.log(max(moms))) if moms else 0
        args.fit_epochs = max(48, math.ceil(need / max(args.fit_steps, 1)))
    if args.fit_steps > 0 and args.fit_epochs > 0:
        gb = args.batch * world
        # weak class signal and 20 % re-drawn labels: the held-out AUC ceiling is 0.90, so the
        # number says how well the fit learned rather than saturating at 1.0
        nc = max(2, args.classes)
        train = synthetic_dataset(gb * args.fit_steps, (H, W, C), nc, seed=11, signal=6.0, label_noise=0.2)
        held = synthetic_dataset(max(gb * 2, 1024), (H, W, C), nc, seed=12, signal=6.0, label_noise=0.2)
        meter = ThroughputMeter()
        model.fit(train.batch(gb, True, 1000, True, seed=5), epochs=args.fit_epochs, callbacks=[meter],
                  verbose=0)
        k = 1 if len(meter.epoch_seconds) > 1 else 0
        t_ep = max(sum(meter.epoch_seconds[k:]) / len(meter.epoch_seconds[k:]), 1e-9)
        t_ep = all_reduce_max(t_ep, dev) if strategy.active else t_ep  # slowest rank sets the pace
        fit_ips = gb * args.fit_steps / t_ep
        logs = model.evaluate(held.batch(gb, False, 1000, False), return_dict=True)
        val_auc, val_acc = (float(logs["auc"]) if "auc" in logs else None), float(logs["accuracy"])

    base = stock_img_s_per_gpu(args.model, size, args.classes, args.phase)
    headline = args.model == "densenet121" and size == 50 and args.classes == 1 and args.phase == "full"
    if rank == 0:
        print(json.dumps({
            "metric": "images/sec (whole node) DenseNet-121 50x50x3 bs=256 at 1/2/4/8 MI355X; val AUC"
            if headline else (f"images/sec (whole node) {args.model} {size}x{size}x3"
                              + (f" {args.classes}-class" if args.classes > 1 else "")
                              + (f" phase={args.phase}" if args.phase != "full" else "")),
            "value": round(value, 1),
            "unit": "images/sec",
            "n_gpus": world if dev.type == "cuda" else 0,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / (base * world), 3) if base and dev.type == "cuda" else None,
            "dtype": "bf16" if dev.type == "cuda" else "fp32",
            "data": f"synthetic uint8 {size}x{size}x3 images, random-init weights",
            "val_auc": round(val_auc, 4) if val_auc is not None else None,
            "val_accuracy": round(val_acc, 4) if val_acc is not None else None,
            "fit_images_per_sec": round(fit_ips, 1) if fit_ips is not None else None,
            "config": {"model": "DenseNet-121" if args.model == "densenet121" else args.model,
                       "global_batch": args.batch * world, "seq_len": None,
                       "input": [H, W, C], "per_gpu_batch": args.batch, "classes": args.classes,
                       "phase": args.phase, "trainable_params": sum(int(t.numel()) for t in model.arena.params)
                       if hasattr(model, "arena") else None,
                       "parallelism": f"dp{world}", "optimizer": "RMSprop(lr=%g)" % args.lr,
                       "loss": "BCE(from_logits)" if args.classes == 1 else "CategoricalCE(from_logits)",
                       "final_loss": round(lossv, 5),
                       "backend": args.backend, "comm_backend": comm_backend, "rccl_version": rccl,
                       "world_size": world,
                       "grad_allreduce": ("native RCCL communicator, bucket ops in the C++ plan"
                                          if getattr(strategy, "native_comm", None) is not None
                                          else "torch.distributed" if strategy.active else None),
                       "stock_baseline_img_s_per_gpu": base,
                       "val": ("exact AUC on a held-out synthetic set (weak signal, 20%% re-drawn labels: "
                               "AUC ceiling 0.90) after %d fit epochs of %d global batches"
                               % (args.fit_epochs, args.fit_steps)) if val_auc is not None else None},
        }), flush=True)
    if strategy.active:
        strategy.close()


if __name__ == "__main__":
    main()
