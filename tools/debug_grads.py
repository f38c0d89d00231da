"""Per-parameter gradient agreement of the fused program vs the eager fp32 reference, and of a
bf16-rounded eager reference vs fp32 (the noise floor), printed from head to stem."""
import copy
import sys

import torch

sys.path.insert(0, ".")
from idc_models_amd.engine import Model, RMSprop  # noqa: E402
from idc_models_amd.models import build_model  # noqa: E402


def cos(a, b):
    a, b = a.reshape(-1).double(), b.reshape(-1).double()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


def grads_eager(net, x, y, dtype):
    net.train()
    xx = x.float() / 255.0
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype == torch.bfloat16):
        logits = net(xx)
    loss = torch.nn.functional.binary_cross_entropy_with_logits(logits.float().reshape(-1), y.float())
    params = [p for p in net.trainable_weights if isinstance(p, torch.nn.Parameter)]
    return loss.item(), logits.detach().float(), torch.autograd.grad(loss, params)


def main():
    arch = sys.argv[1] if len(sys.argv) > 1 else "vgg16"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    dev = torch.device("cuda", 0)
    shape = tuple(int(v) for v in sys.argv[3].split(",")) if len(sys.argv) > 3 else (50, 50, 3)
    net = build_model(arch, shape, num_outputs=1, seed=0)
    ref = copy.deepcopy(net).to(dev)
    ref16 = copy.deepcopy(net).to(dev)
    m = Model(net, device=dev)
    m.compile(RMSprop(1e-3), "binary_crossentropy", [], backend="fused")
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, 256, (B,) + shape, generator=g, dtype=torch.uint8).to(dev)
    y = torch.randint(0, 2, (B,), generator=g).to(dev)
    p = m.impl._prog(B, True, torch.uint8)
    m.impl._stage_inputs(p, x, y)
    p.run_segment("fwd")
    p.run_segment("bwd")
    torch.cuda.synchronize()
    l32, lg32, g32 = grads_eager(ref, x, y, torch.float32)
    l16, lg16, g16 = grads_eager(ref16, x, y, torch.bfloat16)
    print(f"loss fused {p.io.loss.item():.5f} fp32 {l32:.5f} autocast-bf16 {l16:.5f}")
    print("logit maxdiff fused", (p.io.logits - lg32).abs().max().item(), "bf16", (lg16 - lg32).abs().max().item())
    names = []
    for l in ref.base.layers + [ref.head]:
        for n in l.weight_names():
            t = getattr(l, n)
            if isinstance(t, torch.nn.Parameter) and t.requires_grad:
                names.append(f"{l.name}/{n}")
    ar = m.arena
    rows = []
    for i, (a, b) in enumerate(zip(g32, g16)):
        gf = ar.view(ar.grad, i)
        rows.append((names[i] if i < len(names) else str(i), cos(gf, a), cos(b, a),
                     (gf.norm() / (a.norm() + 1e-30)).item()))
    for r in reversed(rows):
        print(f"{r[0]:40s} fused-cos {r[1]:.5f}  autocast-cos {r[2]:.5f}  norm-ratio {r[3]:.4f}")


if __name__ == "__main__":
    main()
