"""Host-side issue time of each program segment vs its GPU time (is the step CPU-bound?).

usage: python tools/host_overhead.py [ARCH] [B]
"""
import sys
import time

import torch

sys.path.insert(0, ".")
from idc_models_amd.engine import Model, RMSprop  # noqa: E402
from idc_models_amd.models import build_model  # noqa: E402


def main():
    arch = sys.argv[1] if len(sys.argv) > 1 else "densenet121"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    dev = torch.device("cuda", 0)
    net = build_model(arch, None, 1, seed=0)
    m = Model(net, device=dev)
    m.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="fused")
    H, W, C = net.input_shape
    x = torch.randint(0, 256, (B, H, W, C), dtype=torch.uint8)
    y = torch.randint(0, 2, (B,))
    for _ in range(5):
        m.impl.train_step(x, y)
    torch.cuda.synchronize()
    p = m.impl._prog(B, True, torch.uint8)
    m.impl._stage_inputs(p, x, y)
    for seg in ("fwd", "bwd", "opt"):
        lo, hi = p.seg[seg]
        for graph in (True, False):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(p.stream)
            t0 = time.perf_counter()
            for _ in range(10):
                p.run_range(lo, hi, graph=graph)
            t1 = time.perf_counter()
            e1.record(p.stream)
            torch.cuda.synchronize()
            print(f"{seg:4s} graph={graph!s:5s} ops={hi - lo:4d} host issue {1e3 * (t1 - t0) / 10:7.3f} ms "
                  f"GPU {e0.elapsed_time(e1) / 10:7.3f} ms", flush=True)


if __name__ == "__main__":
    main()
