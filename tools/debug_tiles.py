"""Find conv ops whose result depends on the tile choice: for every OP_CONV / OP_WGRAD op of a
lowered program, run it with every candidate tile / split and compare outputs bitwise-ish."""
import sys

import torch

sys.path.insert(0, ".")
from idc_models_amd.engine import Model, RMSprop  # noqa: E402
from idc_models_amd.models import build_model  # noqa: E402
from idc_models_amd.ops import _native as nat  # noqa: E402


def main():
    arch = sys.argv[1]
    B = int(sys.argv[2])
    shape = tuple(int(v) for v in sys.argv[3].split(",")) if len(sys.argv) > 3 else None
    dev = torch.device("cuda", 0)
    import os
    os.environ["IDC_AUTOTUNE"] = "0"
    net = build_model(arch, shape, 1, seed=0)
    m = Model(net, device=dev)
    m.compile(RMSprop(1e-3), "binary_crossentropy", [], backend="fused")
    H, W, C = net.input_shape
    x = torch.randint(0, 256, (B, H, W, C), dtype=torch.uint8)
    y = torch.randint(0, 2, (B,))
    p = m.impl._prog(B, True, torch.uint8)
    m.impl._stage_inputs(p, x, y)
    plan = p.plan
    sh = p.stream.cuda_stream
    ext = nat.load()
    # run everything once so every buffer holds real data
    plan.run(0, -1, sh)
    torch.cuda.synchronize()
    bad = 0
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    for i in range(plan.size()):
        if plan.kind(i) == nat.OP_WGRAD:
            a = nat.WgradArgs.from_buffer_copy(plan.payload(i))
            creal = a.cin_real or a.Cin
            n = a.KH * a.KW * creal * a.Cout
            M = a.N * a.Ho * a.Wo
            res = {}
            for s in (1, 2, 4, 16, 64, 256):
                if (M + s - 1) // s < 1:
                    continue
                hip.hipMemset(ctypes.c_void_p(a.dw), 0, ctypes.c_size_t(n * 4))
                torch.cuda.synchronize()
                plan.set_int(i, 0, s)
                plan.run(i, i + 1, sh)
                torch.cuda.synchronize()
                t_ = torch.empty(n, dtype=torch.float32, device=dev)
                hip.hipMemcpy(ctypes.c_void_p(t_.data_ptr()), ctypes.c_void_p(a.dw), ctypes.c_size_t(n * 4), 3)
                res[s] = t_
            ref = res[1]
            for s, v in res.items():
                err = ((v - ref).norm() / (ref.norm() + 1e-12)).item()
                if err > 1e-3 or not torch.isfinite(v).all():
                    bad += 1
                    print(f"wgrad op {i} M={M} Cin={a.Cin} Cout={a.Cout} k={a.KH} f32={plan.get_int(i,1)} "
                          f"splits {s}: rel {err:.3g}")
            continue
        if plan.kind(i) != nat.OP_CONV:
            continue
        a = nat.ConvArgs.from_buffer_copy(plan.payload(i))
        M = a.N * a.Ho * a.Wo
        nbytes = 4 if (a.epi_mode == 0 and a.out_mode) else 2
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")

        def grab(ptr, n, dt):
            t_ = torch.empty(n, dtype=dt, device=dev)
            hip.hipMemcpy(ctypes.c_void_p(t_.data_ptr()), ctypes.c_void_p(ptr), ctypes.c_size_t(n * t_.element_size()), 3)
            return t_

        def zero(ptr, n):
            if ptr:
                hip.hipMemset(ctypes.c_void_p(ptr), 0, ctypes.c_size_t(n * 4))

        acc_ptrs = []
        if a.epi_mode == 0 and a.stats_out:
            acc_ptrs = [a.stats_out + 4 * a.stats_off, a.stats_out + 4 * (a.stats_ld + a.stats_off)]
        elif a.epi_mode == 1:
            acc_ptrs = [a.gsum, a.gsumx]
        outs = {}
        for t in range(ext.num_tiles()):
            if ext.tile_bn(t) > max(32, a.Cout):
                continue
            for q in acc_ptrs:
                zero(q, a.Cout)
            torch.cuda.synchronize()
            plan.set_int(i, 0, t)
            plan.run(i, i + 1, sh)
            torch.cuda.synchronize()
            buf = grab(a.y, M * a.ldy, torch.bfloat16 if nbytes == 2 else torch.float32)
            v = buf.view(M, a.ldy)[:, :a.Cout].float().clone()
            accs = [grab(q, a.Cout, torch.float32) for q in acc_ptrs if q]
            outs[t] = (v, accs)
        ref = outs[min(outs)]
        for t, (v, accs) in outs.items():
            err = ((v - ref[0]).norm() / (ref[0].norm() + 1e-12)).item()
            aerr = max([((x_ - r_).norm() / (r_.norm() + 1e-12)).item() for x_, r_ in zip(accs, ref[1])] or [0])
            if err > 1e-2 or aerr > 1e-2 or not torch.isfinite(v).all():
                bad += 1
                print(f"op {i} M={M} Cin={a.Cin} Cout={a.Cout} k={a.KH} epi={a.epi_mode} f32={plan.get_int(i,1)} "
                      f"tile {t}: out {err:.3g} acc {aerr:.3g}")
    print("bad", bad)


if __name__ == "__main__":
    main()
