"""Reproduce the 'stale memory after GC' corruption deterministically and find the first bad op.

1. build model A + fused program, run fwd+bwd, drop it WITHOUT collecting (reference cycles);
2. build model B + program, run one full train step (captures graphs);
3. gc.collect() and fill the freed memory with 1e30;
4. run step 2 op by op (no graphs) and report the first op after which any program buffer holds
   values > 1e20, plus that op's pointer fields checked against the live tensors.

usage: python tools/gc_repro.py [B]
"""
import ctypes as C
import gc
import os
import sys

import torch

sys.path.insert(0, ".")
os.environ.setdefault("IDC_AUTOTUNE", "0")
from idc_models_amd.engine import Model, RMSprop  # noqa: E402
from idc_models_amd.models import build_model  # noqa: E402
from idc_models_amd.ops import _native as nat  # noqa: E402

DEV = torch.device("cuda", 0)


def make(B, seed, twice=False):
    net = build_model("densenet121", None, 1, seed=seed)
    m = Model(net, device=DEV)
    if twice:
        m.compile(RMSprop(1e-3), "binary_crossentropy", [], backend="fused")
    m.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="fused")
    g = torch.Generator().manual_seed(1)
    H, W, Cc = net.input_shape
    x = torch.randint(0, 256, (B, H, W, Cc), generator=g, dtype=torch.uint8)
    y = torch.randint(0, 2, (B,), generator=g)
    return m, x, y


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    gc.disable()
    a, xa, ya = make(8, 0)
    pa = a.impl._prog(8, True, torch.uint8)
    a.impl._stage_inputs(pa, xa, ya)
    pa.run_segment("fwd")
    pa.run_segment("bwd")
    torch.cuda.synchronize()
    del a, pa
    m, x, y = make(B, 0, twice=os.environ.get("TWICE") == "1")
    loss0, _ = m.impl.train_step(x, y)
    torch.cuda.synchronize()
    print("loss0", loss0.item(), flush=True)
    n = gc.collect()
    junk = []
    free, total = torch.cuda.mem_get_info()
    for _ in range(64):
        try:
            junk.append(torch.full((1 << 20,), 1e30, device=DEV))
        except RuntimeError:
            break
    torch.cuda.synchronize()
    print("collected", n, "objects; junk tensors", len(junk), flush=True)
    p = m.impl._prog(B, True, torch.uint8)
    if os.environ.get("GRAPH") == "1":
        for k in range(3):
            loss, _ = m.impl.train_step(x, y)
            print("graph step", k + 1, "loss", loss.item(), flush=True)
        return
    m.impl._stage_inputs(p, x, y)
    plan, sh = p.plan, p.stream.cuda_stream
    bufs = [t for t in p.b.keep if t.is_floating_point()]
    live = []
    for t in p.b.keep + [p.b.stats_arena, m.arena.data, m.arena.grad, m.optimizer.ms]:
        live.append((t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()))
    for t in list(m.net.parameters()) + list(m.net.buffers()):
        live.append((t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()))
    jr = [(t.data_ptr(), t.data_ptr() + t.numel() * 4) for t in junk]
    torch.cuda.synchronize()
    for i in range(plan.size()):
        plan.run(i, i + 1, sh)
        torch.cuda.synchronize()
        bad = [j for j, t in enumerate(bufs) if t.float().abs().max().item() > 1e20]
        if bad:
            print(f"op {i} ({plan.describe(i)}) -> huge values in buffers {bad[:6]}", flush=True)
            raw = plan.payload(i)
            print("ints", [plan.get_int(i, k) for k in range(4)])
            for nm, st in [("ConvArgs", nat.ConvArgs), ("WgradArgs", nat.WgradArgs), ("PoolArgs", nat.PoolArgs),
                           ("BnBwdApplyArgs", nat.BnBwdApplyArgs), ("HeadArgs", nat.HeadArgs)]:
                if len(raw) == C.sizeof(st):
                    s = st.from_buffer_copy(raw)
                    print(nm)
                    _dump(s, "", live, jr)
            return
    print("no corruption found; loss", p.io.loss.item())


def _dump(s, pre, live, jr):
    for f in s._fields_:
        v = getattr(s, f[0])
        if isinstance(v, C.Structure):
            _dump(v, pre + f[0] + ".", live, jr)
        elif f[1] is C.c_void_p:
            v = v or 0
            where = "null" if not v else ("live" if any(lo <= v < hi for lo, hi in live) else
                                          ("JUNK" if any(lo <= v < hi for lo, hi in jr) else "unknown"))
            print(f"  {pre}{f[0]} = {hex(v)} [{where}]")
        else:
            print(f"  {pre}{f[0]} = {v}")


if __name__ == "__main__":
    main()
