"""Fused vs eager: fit a fresh model on a learnable synthetic set, then compare evaluate()
(inference-mode BatchNorm, exact AUC) and the eval logits of both backends on the same weights.

    python tools/check_eval.py [--model densenet121] [--batch 64] [--epochs 3]
"""
import argparse
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="densenet121")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--train-backend", default="fused", choices=["fused", "eager"])
    a = ap.parse_args()
    from idc_models_amd.data import synthetic_dataset
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model
    dev = torch.device("cuda", 0)
    net = build_model(a.model, num_outputs=1, seed=0)
    m = Model(net, device=dev)
    m.compile(RMSprop(a.lr), "binary_crossentropy", ["accuracy", "auc"], backend=a.train_backend)
    tr = synthetic_dataset(a.batch * 16, net.input_shape, 2, seed=11)
    te = synthetic_dataset(512, net.input_shape, 2, seed=12)
    h = m.fit(tr.batch(a.batch, True, 1000, True, seed=1), epochs=a.epochs, verbose=1,
              validation_data=te.batch(a.batch, False))
    print("fused fit history", {k: [round(v, 4) for v in vs] for k, vs in h.history.items()})
    print("fused evaluate", m.evaluate(te.batch(a.batch, False), return_dict=True))
    ref = Model(copy.deepcopy(m.net), device=dev)
    ref.compile(RMSprop(a.lr), "binary_crossentropy", ["accuracy", "auc"], backend="eager")
    print("eager evaluate (same weights)", ref.evaluate(te.batch(a.batch, False), return_dict=True))
    xb, yb = next(iter(te.batch(a.batch, False)))
    _, lf = m.impl.eval_step(xb, yb)
    _, le = ref.impl.eval_step(xb, yb)
    print("eval logits fused", lf.reshape(-1)[:8].tolist())
    print("eval logits eager", le.reshape(-1)[:8].tolist())
    # run-to-run variability of the fused training step at this batch: the same program, the same
    # weights and inputs, gradients of two back-to-back fwd+bwd runs
    if a.train_backend != "fused":
        return
    p = m.impl._prog(xb.shape[0], True, torch.uint8)
    gs = []
    for _ in range(2):
        m.impl._stage_inputs(p, xb, yb)
        p.run_segment("fwd")
        p.run_segment("bwd")
        torch.cuda.synchronize()
        gs.append(m.arena.grad.double().clone())
    cos = float(gs[0] @ gs[1] / (gs[0].norm() * gs[1].norm()))
    print("fused run-to-run grad cosine at batch", xb.shape[0], cos, "rel", float((gs[0] - gs[1]).norm() / gs[0].norm()))
    bn = [l for l in m.net.base.layers if l.__class__.__name__ == "BatchNormalization"]
    for l in bn[:3] + bn[-2:]:
        print(l.name, "mm", float(l.moving_mean.abs().mean()), "mv", float(l.moving_variance.mean()))


if __name__ == "__main__":
    main()
