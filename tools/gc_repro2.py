"""Deterministic version of the flaky fused-test sequence: garbage from a previous test is
collected right before the eager reference forward that sits between two fused train steps."""
import copy
import gc
import importlib.util
import sys

import torch

sys.path.insert(0, ".")
spec = importlib.util.spec_from_file_location("t", "tests/test_fused_gpu.py")
T = importlib.util.module_from_spec(spec)
spec.loader.exec_module(T)
DEV = T.DEV


def main():
    gc.disable()
    T.test_densenet121_fused_matches_eager()
    m, ref, x, y = T._setup("densenet121", 16)
    from idc_models_amd.engine import RMSprop
    if "--once" not in sys.argv:
        m.compile(RMSprop(1e-4), "binary_crossentropy", ["accuracy"], backend="fused")
    loss0, _ = m.impl.train_step(x, y)
    torch.cuda.synchronize()
    print("collected", gc.collect())
    ref.train()
    ref(x.to(DEV).float() / 255.0)
    losses = [loss0.item()]
    for _ in range(3):
        loss, _ = m.impl.train_step(x, y)
        losses.append(loss.item())
    print("losses", losses, "BAD" if losses[-1] > losses[0] else "ok")


if __name__ == "__main__":
    main()
