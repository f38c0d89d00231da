"""In-situ comparison point: stock PyTorch-ROCm DenseNet-121 / VGG16 / MobileNetV2 training step.

BASELINE.md: the reference publishes no numbers, so the point to beat is "stock PyTorch-ROCm
(MIOpen convolutions, bf16 autocast, channels_last)" on the same MI355X and config.  This is a
plain ``torch.nn`` implementation (torchvision is not installed) — NOT part of the framework's
hot path; it exists only to produce that number.

    python benchmarks/stock_pytorch_baseline.py --model densenet121 --batch 256 --steps 20
"""
from __future__ import annotations

import argparse
import json
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
    def __init__(self, blocks=(6, 12, 24, 16)):
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
                   nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(ch, 1)]
        self.net = nn.Sequential(*layers)

    def forward(self, x):
        return self.net(x)


def vgg16():
    cfg = [(64, 2), (128, 2), (256, 3), (512, 3), (512, 3)]
    layers, cin = [], 3
    for c, n in cfg:
        for _ in range(n):
            layers += [nn.Conv2d(cin, c, 3, padding=1), nn.ReLU()]
            cin = c
        layers.append(nn.MaxPool2d(2, 2))
    layers += [nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(512, 1)]
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


def mobilenetv2():
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
               nn.ReLU6(), nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(1280, 1)]
    return nn.Sequential(*layers)


def run(model_name: str, batch: int, steps: int, warmup: int, graph: bool, channels_last: bool = True) -> dict:
    """Time one stock training step (bf16 autocast forward, fp32 loss, backward, RMSprop).
    ``graph``: the whole step captured once into a HIP graph (torch.cuda.graphs, capturable
    RMSprop) and replayed — the strongest stock configuration (no per-kernel host launches)."""
    dev = torch.device("cuda")
    torch.backends.cudnn.benchmark = True
    torch.manual_seed(0)
    model = {"densenet121": DenseNet121, "vgg16": vgg16, "mobilenetv2": mobilenetv2}[model_name]().to(dev)
    fmt = torch.channels_last if channels_last else torch.contiguous_format
    model = model.to(memory_format=fmt)
    opt = torch.optim.RMSprop(model.parameters(), lr=1e-4, alpha=0.9, eps=1e-7, capturable=graph)
    x = torch.rand(batch, 3, 50, 50, device=dev).to(memory_format=fmt)
    y = torch.randint(0, 2, (batch, 1), device=dev).float()

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(x)
        loss = F.binary_cross_entropy_with_logits(out.float(), y)
        loss.backward()
        opt.step()
        return loss

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(warmup):
            opt.zero_grad(set_to_none=True)
            step()
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
    return {"baseline": "stock_pytorch_%s_bf16_autocast" % ("hipgraph" if graph else "eager"),
            "model": model_name, "batch": batch, "ms_per_step": round(dt * 1e3, 3),
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
    ap.add_argument("--all", metavar="OUT_JSON", help="every model, eager and graph; write JSON")
    args = ap.parse_args()
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
                         not args.no_channels_last)))


if __name__ == "__main__":
    main()
