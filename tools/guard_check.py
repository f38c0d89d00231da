"""Out-of-bounds hunt: lower a model with NaN-guarded buffers (IDC_GUARD=1), run the plan op by
op and report (a) the first op after which any guard region changed (OOB write) and (b) the
first op whose buffers turned non-finite (OOB read of a NaN guard, or a real overflow).

usage: python tools/guard_check.py ARCH B [H,W,C]
"""
import os
import sys

os.environ["IDC_GUARD"] = "1"
os.environ["IDC_AUTOTUNE"] = "0"
os.environ["IDC_NO_GRAPHS"] = "1"

import torch  # noqa: E402

sys.path.insert(0, ".")
from idc_models_amd.engine import Model, RMSprop  # noqa: E402
from idc_models_amd.models import build_model  # noqa: E402


def main():
    arch, B = sys.argv[1], int(sys.argv[2])
    shape = tuple(int(v) for v in sys.argv[3].split(",")) if len(sys.argv) > 3 else None
    dev = torch.device("cuda", 0)
    net = build_model(arch, shape, 1, seed=0)
    m = Model(net, device=dev)
    m.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="fused")
    H, W, C = net.input_shape
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, 256, (B, H, W, C), generator=g, dtype=torch.uint8)
    y = torch.randint(0, 2, (B,), generator=g)
    p = m.impl._prog(B, True, torch.uint8)
    m.impl._stage_inputs(p, x, y)
    b = p.b
    plan, sh = p.plan, p.stream.cuda_stream
    torch.cuda.synchronize()
    flo = [(base, gd, n) for base, gd, n in b.guards if base.dtype.is_floating_point]
    print(f"{plan.size()} ops, {len(flo)} guarded float buffers", flush=True)

    def guards_ok():
        bad = [i for i, (base, gd, n) in enumerate(flo)
               if not (bool(torch.isnan(base[:gd]).all()) and bool(torch.isnan(base[gd + n:]).all()))]
        return bad

    def nonfinite():
        return [i for i, (base, gd, n) in enumerate(flo) if not bool(torch.isfinite(base[gd:gd + n]).all())]

    seen_nf = set()
    for step in range(2):
        for i in range(plan.size()):
            plan.run(i, i + 1, sh)
            torch.cuda.synchronize()
            bad = guards_ok()
            if bad:
                base, gd, n = flo[bad[0]]
                print(f"step {step} op {i} ({plan.describe(i)}): guard overwritten on buffers {bad[:8]} "
                      f"(shape numel {n}, dtype {base.dtype})", flush=True)
                return
            nf = [j for j in nonfinite() if j not in seen_nf]
            if nf:
                print(f"step {step} op {i} ({plan.describe(i)}): new non-finite buffers {nf[:8]}", flush=True)
                seen_nf.update(nf)
    print("done; non-finite buffers:", sorted(seen_nf)[:20])


if __name__ == "__main__":
    main()
