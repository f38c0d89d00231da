"""Layer-by-layer comparison of the lowered DenseNet forward (training mode) with the eager
reference: stem output, stats, every stage buffer and bottleneck tensor."""
import copy
import sys

import torch

sys.path.insert(0, ".")
from idc_models_amd.engine import Model, RMSprop  # noqa: E402
from idc_models_amd.models import build_model  # noqa: E402


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def folded(st):
    """[sum | sumsq] of a Stats view with its slot copies added up."""
    return st.t[:2 * st.ld * st.slots].view(st.slots, 2 * st.ld).sum(0)


def main():
    dev = torch.device("cuda", 0)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    arch = sys.argv[2] if len(sys.argv) > 2 else "densenet121"
    shape = tuple(int(v) for v in sys.argv[3].split(",")) if len(sys.argv) > 3 else (50, 50, 3)
    net = build_model(arch, shape, num_outputs=1, seed=0)
    ref = copy.deepcopy(net).to(dev)
    m = Model(net, device=dev)
    m.compile(RMSprop(1e-3), "binary_crossentropy", [], backend="fused")
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, 256, (B,) + shape, generator=g, dtype=torch.uint8)
    y = torch.randint(0, 2, (B,), generator=g)
    p = m.impl._prog(B, True, torch.uint8)
    m.impl._stage_inputs(p, x, y)
    p.run_segment("fwd")
    torch.cuda.synchronize()
    dbg = p.b.debug
    # reference activations, hooking the eager graph
    base = ref.base
    ref.train()
    acts = {}
    xx = x.to(dev).float() / 255.0
    saved = []
    h = xx
    for kind, layer in base.graph:
        if kind == "seq":
            h = layer(h)
            acts[layer.name] = h
        elif kind == "save":
            saved.append(h)
        elif kind == "concat":
            h = layer(saved.pop(), h)
            acts[layer.name] = h
    ys = dbg["ys"].t.float()
    print("stem conv", rel(ys, acts["conv1/conv"]))
    ss = folded(dbg["ss"])
    yr = acts["conv1/conv"]
    print("stem stats sum", rel(ss[:64], yr.sum((0, 1, 2))), "sq", rel(ss[64:128], (yr * yr).sum((0, 1, 2))))
    for si, st in enumerate(dbg["stages"]):
        buf = st["buf"].t.float()
        c0 = st["c0"]
        print(f"stage {si}: first {c0} ch vs", end=" ")
        if si == 0:
            print(rel(buf[..., :64], acts["pool1"]))
        else:
            print(rel(buf[..., :c0], acts[f"pool{si + 1}_pool"]))
        stt = folded(st["stats"])
        ctot = st["ctot"]
        for li, lay in enumerate(st["layers"]):
            name = f"conv{si + 2}_block{li + 1}"
            t = lay["t"].t.float()
            e_t = rel(t, acts[name + "_1_conv"])
            new = buf[..., lay["cin"]:lay["cin"] + 32]
            e_n = rel(new, acts[name + "_2_conv"])
            cin = lay["cin"]
            cat_in = acts[name + "_concat"][..., :cin] if li else None
            if li < 2 or e_t > 0.15 or e_n > 0.15:
                print(f"  {name}: T {e_t:.4f}  new {e_n:.4f}")
        full = acts[f"conv{si + 2}_block{len(st['layers'])}_concat"]
        print(f"  stage buffer vs concat: {rel(buf, full):.4f}")
        print(f"  stats sum {rel(stt[:ctot], full.sum((0, 1, 2))):.5f} sq {rel(stt[ctot:2 * ctot], (full * full).sum((0, 1, 2))):.5f}")
    print("logits", p.io.logits.reshape(-1)[:8].tolist())
    print("ref   ", ref.head(ref.gap(h)).reshape(-1)[:8].tolist())


if __name__ == "__main__":
    main()
