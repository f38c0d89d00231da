"""Run N fused training steps on a fixed batch and print the loss per step (race / blow-up hunt).

usage: python tools/stress_steps.py ARCH B STEPS [REPEATS] [LR]
"""
import sys

import torch

sys.path.insert(0, ".")
from idc_models_amd.engine import Model, RMSprop  # noqa: E402
from idc_models_amd.models import build_model  # noqa: E402


def main():
    arch, B, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    lr = float(sys.argv[5]) if len(sys.argv) > 5 else 1e-4
    dev = torch.device("cuda", 0)
    for r in range(reps):
        net = build_model(arch, None, 1, seed=0)
        m = Model(net, device=dev)
        m.compile(RMSprop(lr), "binary_crossentropy", [], backend="fused")
        H, W, C = net.input_shape
        g = torch.Generator().manual_seed(1)
        x = torch.randint(0, 256, (B, H, W, C), generator=g, dtype=torch.uint8)
        y = torch.randint(0, 2, (B,), generator=g)
        losses = []
        for _ in range(steps):
            loss, logits = m.impl.train_step(x, y)
            losses.append(loss.item())
        amax = logits.abs().max().item()
        print(f"rep {r}: " + " ".join(f"{v:.4f}" for v in losses) + f" | max|logit| {amax:.3g}", flush=True)
        m._release_impl()


if __name__ == "__main__":
    main()
