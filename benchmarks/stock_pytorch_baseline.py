"""In-situ comparison point: stock PyTorch-ROCm DenseNet-121/201 / VGG16 / MobileNetV2 training step.

BASELINE.md: the reference publishes no numbers, so the point to beat is "stock PyTorch-ROCm
(MIOpen convolutions, bf16 autocast, channels_last)" on the same MI355X and config.  This is a
plain ``torch.nn`` implementation (torchvision is not installed) — NOT part of the framework's
hot path; it exists only to produce that number.

    python benchmarks/stock_pytorch_baseline.py --model densenet121 --batch 256 --steps 20
    python benchmarks/stock_pytorch_baseline.py --model densenet201 --input 32 --classes 10 --phase finetune

``--phase``: ``full`` (every layer trains), ``frozen`` (reference phase 1, ``base_model.trainable =
False``: only the head trains, frozen BatchNorms in inference mode) or ``finetune`` (reference
phase 2, ``fine_tune_at`` = 150 for DenseNet / 100 for MobileNetV2 / 15 for VGG16 Keras layers
frozen (recipes/transfer.py fine_tune_at_for): the same
number of leading weighted layers -- Keras order = this module order -- is frozen here).
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class DenseLayer(nn.Module):
    def __init__(self, cin, growth=32):
        super().__init__()
        self.bn1 = nn.BatchNorm2d(cin, eps=1.001e-5, momentum=0.01)
        self.conv1 = nn.Conv2d(cin, 4 * growth, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(4 * growth, eps=1.001e-5, momentum=0.01)
        self.conv2 = nn.Conv2d(4 * growth, growth, 3, padding=1, bias=False)

    def forward(self, x):
        y = self.conv1(F.relu(self.bn1(x)))
        y = self.conv2(F.relu(self.bn2(y)))
        return torch.cat([x, y], 1)


class DenseNet121(nn.Module):
    def __init__(self, blocks=(6, 12, 24, 16), classes=1):
        super().__init__()
        layers = [nn.ZeroPad2d(3), nn.Conv2d(3, 64, 7, 2, bias=False),
                  nn.BatchNorm2d(64, eps=1.001e-5, momentum=0.01), nn.ReLU(), nn.ZeroPad2d(1),
                  nn.MaxPool2d(3, 2)]
        ch = 64
        for i, nb in enumerate(blocks):
            for _ in range(nb):
                layers.append(DenseLayer(ch))
                ch += 32
            if i < len(blocks) - 1:
                layers += [nn.BatchNorm2d(ch, eps=1.001e-5, momentum=0.01), nn.ReLU(),
                           nn.Conv2d(ch, ch // 2, 1, bias=False), nn.AvgPool2d(2, 2)]
                ch //= 2
        layers += [nn.BatchNorm2d(ch, eps=1.001e-5, momentum=0.01), nn.ReLU(),
                   nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(ch, classes)]
        self.net = nn.Sequential(*layers)

    def forward(self, x):
        return self.net(x)


def densenet201(classes=1):
    return DenseNet121((6, 12, 48, 32), classes)


def vgg16(classes=1):
    cfg = [(64, 2), (128, 2), (256, 3), (512, 3), (512, 3)]
    layers, cin = [], 3
    for c, n in cfg:
        for _ in range(n):
            layers += [nn.Conv2d(cin, c, 3, padding=1), nn.ReLU()]
            cin = c
        layers.append(nn.MaxPool2d(2, 2))
    layers += [nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(512, classes)]
    return nn.Sequential(*layers)


def _div8(v):
    n = max(8, int(v + 4) // 8 * 8)
    return n + 8 if n < 0.9 * v else n


class InvRes(nn.Module):
    def __init__(self, cin, cout, stride, t):
        super().__init__()
        ch = cin * t
        layers = []
        if t != 1:
            layers += [nn.Conv2d(cin, ch, 1, bias=False), nn.BatchNorm2d(ch, eps=1e-3, momentum=1e-3), nn.ReLU6()]
        pad = (1, 1, 1, 1) if stride == 1 else (0, 1, 0, 1)
        layers += [nn.ZeroPad2d(pad), nn.Conv2d(ch, ch, 3, stride, groups=ch, bias=False),
                   nn.BatchNorm2d(ch, eps=1e-3, momentum=1e-3), nn.ReLU6(),
                   nn.Conv2d(ch, cout, 1, bias=False), nn.BatchNorm2d(cout, eps=1e-3, momentum=1e-3)]
        self.body = nn.Sequential(*layers)
        self.res = stride == 1 and cin == cout

    def forward(self, x):
        y = self.body(x)
        return x + y if self.res else y


def mobilenetv2(classes=1):
    cfg = [(16, 1, 1), (24, 2, 6), (24, 1, 6), (32, 2, 6), (32, 1, 6), (32, 1, 6), (64, 2, 6), (64, 1, 6),
           (64, 1, 6), (64, 1, 6), (96, 1, 6), (96, 1, 6), (96, 1, 6), (160, 2, 6), (160, 1, 6),
           (160, 1, 6), (320, 1, 6)]
    layers = [nn.ZeroPad2d((0, 1, 0, 1)), nn.Conv2d(3, 32, 3, 2, bias=False),
              nn.BatchNorm2d(32, eps=1e-3, momentum=1e-3), nn.ReLU6()]
    cin = 32
    for c, s, t in cfg:
        layers.append(InvRes(cin, _div8(c), s, t))
        cin = _div8(c)
    layers += [nn.Conv2d(cin, 1280, 1, bias=False), nn.BatchNorm2d(1280, eps=1e-3, momentum=1e-3),
               nn.ReLU6(), nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(1280, classes)]
    return nn.Sequential(*layers)


def _keras_frozen_weighted(model_name: str, phase: str, size: int, classes: int):
    """How many leading weighted (conv / BN) layers the reference freezes in ``phase``: counted on
    the framework's Keras-order layer list, so both sides freeze the same layers."""
    if phase == "full":
        return 0
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from idc_models_amd.models import build_model
    from idc_models_amd.recipes.transfer import fine_tune_at_for
    net = build_model(model_name, (size, size, 3), classes, seed=0)
    layers = net.base.layers
    if phase == "finetune":  # the reference's cut: VGG16 15, MobileNetV2 100, DenseNets 150
        layers = layers[:fine_tune_at_for(model_name)]
    return sum(1 for l in layers if l.keras_class in ("Conv2D", "BatchNormalization", "DepthwiseConv2D"))


def _heartbeat(stop):
    """MIOpen compiles (and with benchmark mode searches) every new conv shape on first use: a
    201-layer network on a fresh box stays inside its first step for minutes.  Say so."""
    t0 = time.time()
    while not stop.wait(30):
        print(f"# still in MIOpen first-use compilation / search after {time.time() - t0:.0f} s",
              file=sys.stderr, flush=True)


def run(model_name: str, batch: int, steps: int, warmup: int, graph: bool, channels_last: bool = True,
        size: int = 50, classes: int = 1, phase: str = "full", benchmark: bool = True) -> dict:
    """Time one stock training step (bf16 autocast forward, fp32 loss, backward, RMSprop).
    ``graph``: the whole step captured once into a HIP graph (torch.cuda.graphs, capturable
    RMSprop) and replayed — the strongest stock configuration (no per-kernel host launches)."""
    import threading
    dev = torch.device("cuda")
    torch.backends.cudnn.benchmark = benchmark
    stop = threading.Event()
    threading.Thread(target=_heartbeat, args=(stop,), daemon=True).start()
    torch.manual_seed(0)
    ctor = {"densenet121": DenseNet121, "densenet201": densenet201, "vgg16": vgg16, "mobilenetv2": mobilenetv2}
    model = ctor[model_name](classes=classes).to(dev)
    nfreeze = _keras_frozen_weighted(model_name, phase, size, classes)
    weighted = [mod for mod in model.modules() if isinstance(mod, (nn.Conv2d, nn.BatchNorm2d))]
    for mod in weighted[:nfreeze]:
        for prm in mod.parameters():
            prm.requires_grad_(False)
    frozen_bn = [mod for mod in weighted[:nfreeze] if isinstance(mod, nn.BatchNorm2d)]
    fmt = torch.channels_last if channels_last else torch.contiguous_format
    model = model.to(memory_format=fmt)
    model.train()
    for mod in frozen_bn:  # Keras: a non-trainable BatchNormalization runs in inference mode
        mod.eval()
    opt = torch.optim.RMSprop([q for q in model.parameters() if q.requires_grad], lr=1e-4, alpha=0.9,
                              eps=1e-7, capturable=graph)
    x = torch.rand(batch, 3, size, size, device=dev).to(memory_format=fmt)
    if classes == 1:
        y = torch.randint(0, 2, (batch, 1), device=dev).float()
    else:
        y = torch.randint(0, classes, (batch,), device=dev)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(x)
        loss = (F.binary_cross_entropy_with_logits(out.float(), y) if classes == 1
                else F.cross_entropy(out.float(), y))
        loss.backward()
        opt.step()
        return loss

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for i in range(warmup):
            opt.zero_grad(set_to_none=True)
            step()
            torch.cuda.synchronize()  # MIOpen's first-call searches can take minutes: show progress
            print(f"# warmup step {i} done", file=sys.stderr, flush=True)
    torch.cuda.current_stream().wait_stream(side)
    if graph:
        g = torch.cuda.CUDAGraph()
        opt.zero_grad(set_to_none=True)
        with torch.cuda.graph(g):
            step()
        run_step = g.replay
    else:
        def run_step():
            opt.zero_grad(set_to_none=True)
            step()
    for _ in range(3):
        run_step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        run_step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    stop.set()
    return {"baseline": "stock_pytorch_%s_bf16_autocast" % ("hipgraph" if graph else "eager"),
            "model": model_name, "batch": batch, "input": [size, size, 3], "classes": classes, "phase": phase,
            "frozen_weighted_layers": nfreeze, "miopen_benchmark": benchmark, "ms_per_step": round(dt * 1e3, 3),
            "images_per_sec": round(batch / dt, 1), "channels_last": channels_last,
            "torch": torch.__version__, "device": torch.cuda.get_device_name()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="densenet121")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-channels-last", action="store_true")
    ap.add_argument("--graph", action="store_true", help="HIP-graph-captured step")
    ap.add_argument("--input", type=int, default=50, help="square input size")
    ap.add_argument("--classes", type=int, default=1)
    ap.add_argument("--phase", default="full", choices=["full", "frozen", "finetune"])
    ap.add_argument("--no-benchmark", action="store_true",
                    help="MIOpen immediate mode (PyTorch's default) instead of benchmark-mode search")
    ap.add_argument("--all", metavar="OUT_JSON", help="every model, eager and graph; write JSON")
    ap.add_argument("--append", metavar="JSON", help="append this run's eager and graph results to JSON")
    args = ap.parse_args()
    if args.append:
        with open(args.append) as f:
            doc = json.load(f)
        for graph in (False, True):
            r = run(args.model, args.batch, args.steps, args.warmup, graph, not args.no_channels_last,
                    args.input, args.classes, args.phase, not args.no_benchmark)
            print(json.dumps(r), flush=True)
            doc["results"].append(r)
        with open(args.append, "w") as f:
            json.dump(doc, f, indent=1)
        return
    if args.all:
        results = []
        for m in ("densenet121", "vgg16", "mobilenetv2"):
            for graph in (False, True):
                try:
                    r = run(m, args.batch, args.steps, args.warmup, graph, not args.no_channels_last)
                except Exception as e:  # a stock configuration that cannot be captured is recorded
                    r = {"model": m, "baseline": "stock_pytorch_%s" % ("hipgraph" if graph else "eager"),
                         "error": repr(e)[:300], "images_per_sec": 0.0}
                print(json.dumps(r), flush=True)
                results.append(r)
        with open(args.all, "w") as f:
            json.dump({"note": "in-situ comparison point (BASELINE.md): stock PyTorch-ROCm, MIOpen "
                               "convolutions, bf16 autocast, channels_last, RMSprop; one MI355X; "
                               "synthetic 50x50x3, per-GPU batch %d" % args.batch,
                       "results": results}, f, indent=1)
        return
    print(json.dumps(run(args.model, args.batch, args.steps, args.warmup, args.graph,
                         not args.no_channels_last, args.input, args.classes, args.phase,
                         not args.no_benchmark)))


if __name__ == "__main__":
    main()
