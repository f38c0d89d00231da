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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="densenet121")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-channels-last", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda")
    torch.backends.cudnn.benchmark = True
    model = {"densenet121": DenseNet121, "vgg16": vgg16, "mobilenetv2": mobilenetv2}[args.model]().to(dev)
    fmt = torch.contiguous_format if args.no_channels_last else torch.channels_last
    model = model.to(memory_format=fmt)
    opt = torch.optim.RMSprop(model.parameters(), lr=1e-4, alpha=0.9, eps=1e-7)
    x = torch.rand(args.batch, 3, 50, 50, device=dev).to(memory_format=fmt)
    y = torch.randint(0, 2, (args.batch, 1), device=dev).float()

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(x)
        loss = F.binary_cross_entropy_with_logits(out.float(), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / args.steps
    print(json.dumps({"baseline": "stock_pytorch_eager_bf16_autocast", "model": args.model,
                      "batch": args.batch, "ms_per_step": dt * 1e3,
                      "images_per_sec": args.batch / dt,
                      "channels_last": not args.no_channels_last}))


if __name__ == "__main__":
    main()
