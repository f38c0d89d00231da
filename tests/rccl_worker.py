"""Worker for tests/test_rccl_gpu.py: one rank on cuda:0 over the ``nccl`` (= RCCL) backend with
collectives forced on in a world of one (``IDC_FORCE_COLLECTIVES=1``), launched by
``torch.distributed.run``.  Every data-parallel / federated collective the framework issues then
really runs through RCCL on the MI355X:

* ``native``   — the C++ communicator: f32 / int32 / bf16 all-reduce, reduce, broadcast,
                 all-gather, exact (a world of one is the identity, extreme int32 values included);
* ``dp_det``   — DenseNet-121 fused training steps through MirroredStrategy with the native
                 bucketed all-reduce ops inside the plan (comm stream, per-bucket ncclAllReduce,
                 join) under IDC_DETERMINISTIC=1: bit-identical to the single-device program;
* ``dp_tuned`` — the same with autotuned split-K tiles and float-atomic statistics (what ships):
                 every parameter's gradient checked against an fp32 eager reference of the same
                 step (per-parameter cosine against the bf16-autocast floor, as
                 tests/test_fused_gpu.py::_check), for the data-parallel AND the single-device
                 program;
* ``central``  — CentralStorageStrategy (``dist_model_tf_dense.py:18,21-24``): reduce to rank 0,
                 RMSprop on rank 0 only, broadcast of the parameters, all through the native
                 communicator inside the fused step, under IDC_DETERMINISTIC=1: bit-identical
                 gradients and updated weights to the single-device program;
* ``masked``   — MaskedAggregator's masked SUM (one ncclUint32 all-reduce) and decode;
* ``nonblocking`` — a communicator created non-blocking with an init timeout (the world > 1
                 form), the uint32 ring sum and the watchdog's progress marks;
* ``fedavg``   — the FedAvg packed all-reduce and the server-state broadcast helpers.
Prints ``RCCLCASE {json}`` per case.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def emit(d):
    print("RCCLCASE " + json.dumps(d), flush=True)


def case_native(st):
    nc = st.native_comm
    dev = st.device
    before = nc.collectives
    x = torch.randn(1 << 16, device=dev)
    y = x.clone()
    nc.all_reduce_(y)
    i = torch.tensor([-(2 ** 31), 2 ** 31 - 1, -1, 0, 12345], dtype=torch.int32, device=dev)
    j = i.clone()
    nc.all_reduce_(j)
    b = torch.randn(999, device=dev).bfloat16()
    bb = b.clone()
    nc.all_reduce_(bb, "max")
    r = x.clone()
    nc.reduce_(r, 0)
    c = x.clone()
    nc.broadcast_(c, 0)
    g = nc.all_gather(i)
    torch.cuda.synchronize()
    ok = (torch.equal(x, y) and torch.equal(i, j) and torch.equal(b, bb) and torch.equal(r, x)
          and torch.equal(c, x) and tuple(g.shape) == (1, 5) and torch.equal(g[0], i)
          and nc.collectives - before == 6)
    nc.check()
    emit({"case": "native", "ok": bool(ok), "rccl": nc.version(), "collectives": nc.collectives - before})


def _step_models(arch, per, det, bucket_bytes):
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model
    from idc_models_amd.parallel import MirroredStrategy, OneDeviceStrategy
    os.environ["IDC_DETERMINISTIC"] = "1" if det else "0"
    st = MirroredStrategy(bucket_bytes=bucket_bytes, force_collectives=True)
    m = Model(build_model(arch, None, 1, seed=7), st)
    m.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="fused")
    ref = Model(build_model(arch, None, 1, seed=7), OneDeviceStrategy("cuda:0"))
    ref.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="fused")
    ref2 = None
    if not det:  # a second single-device run gives the run-to-run noise floor of the float atomics
        ref2 = Model(build_model(arch, None, 1, seed=7), OneDeviceStrategy("cuda:0"))
        ref2.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="fused")
    g = torch.Generator().manual_seed(3)
    H, W, C = m.net.input_shape
    x = torch.randint(0, 256, (per, H, W, C), generator=g, dtype=torch.uint8)
    y = torch.randint(0, 2, (per,), generator=g)
    return st, m, ref, ref2, x, y


def _fp32_check(net0, arena, grad, x, y):
    """Parameters of a fused program's gradient ``grad`` (flat, ``arena`` layout) further from the
    fp32 eager gradient of the pre-step network ``net0`` than 1.5x bf16 autocast's relative error
    + 0.02 (idc_models_amd/utils/fidelity.py).  Returns (number of failures, worst failure)."""
    import copy

    from idc_models_amd.utils.fidelity import eager_grads, grad_failures
    ref = copy.deepcopy(net0).to(grad.device)
    g32, g16 = eager_grads(ref, x, y, "fp32"), eager_grads(ref, x, y, "autocast")
    bad = grad_failures(arena, grad, g32, g16)
    worst = max(bad, key=lambda r: r["rel"] / max(r["rel_autocast"], 1e-12)) if bad else None
    return len(bad), worst


def case_nonblocking(st):
    """A second communicator created NON-blocking (ncclCommInitRankConfig, blocking = 0, init
    timeout) as every world > 1 is: its collectives settle through ncclInProgress, the uint32 ring
    sum, the watchdog's progress marks and its poll on a healthy communicator."""
    from idc_models_amd.parallel.native_comm import NativeCommunicator
    from idc_models_amd.parallel.watchdog import CommWatchdog
    dev = st.device
    nc = NativeCommunicator(0, 1, dev, init_timeout_s=60.0, watchdog=False)
    x = torch.randn(4097, device=dev)
    y = x.clone()
    nc.all_reduce_(y)
    u = torch.tensor([-1, -(2 ** 31), 2 ** 31 - 1, 7], dtype=torch.int32, device=dev)
    v = u.clone()
    nc.all_reduce_u32_(v)
    wd = CommWatchdog(nc.c, timeout_s=30.0)
    wd.mark()
    torch.cuda.synchronize()
    age = nc.c.mark_age()
    polled = wd.poll_once()
    nc.close()
    ok = torch.equal(x, y) and torch.equal(u, v) and age == 0.0 and polled is None
    emit({"case": "nonblocking", "ok": bool(ok), "age": age, "polled": polled})


def case_dp(det):
    from idc_models_amd.parallel import comm
    import copy
    st, m, ref, ref2, x, y = _step_models("densenet121", 64, det, 2 << 20)
    net0 = copy.deepcopy(m.net) if not det else None  # the weights the first step starts from
    nc = st.native_comm
    c0 = nc.collectives
    m.impl.train_step(x, y)
    ref.impl.train_step(x, y)
    torch.cuda.synchronize()
    p = m.impl._prog(x.shape[0], True, torch.uint8)
    g_dp, g_ref = m.arena.grad.detach().clone(), ref.arena.grad.detach().clone()
    rel = float((g_dp - g_ref).norm() / g_ref.norm().clamp_min(1e-30))
    floor = 0.0
    bad_dp = bad_ref = None
    if ref2 is not None:
        ref2.impl.train_step(x, y)
        torch.cuda.synchronize()
        floor = float((ref2.arena.grad - g_ref).norm() / g_ref.norm().clamp_min(1e-30))
        ref2.impl.close()
        # falsifiable bound: both programs' first-step gradients against fp32 (the weights the
        # step started from are the seed's, identical in m, ref and the eager copies)
        bad_dp, info_dp = _fp32_check(net0, m.arena, g_dp, x, y)
        bad_ref, info_ref = _fp32_check(net0, ref.arena, g_ref, x, y)
    m.impl.train_step(x, y)
    ref.impl.train_step(x, y)
    torch.cuda.synchronize()
    wdp, wref = m.arena.data.detach(), ref.arena.data.detach()
    wdiff = float((wdp - wref).abs().max())
    n_ops = p.n_comm_ops
    ran = nc.collectives - c0
    out = {"case": "dp_det" if det else "dp_tuned", "backend": comm.backend(), "comm_ops_per_step": n_ops,
           "collectives": ran, "grad_rel": rel, "noise_floor_rel": floor, "weight_max_diff": wdiff,
           "native": p.native_comm is not None, "fp32_failures_dp": bad_dp, "fp32_failures_single": bad_ref}
    if not det:
        out["worst_dp"], out["worst_single"] = info_dp, info_ref
    if det:
        ok = n_ops >= 2 and ran == 2 * n_ops and rel == 0.0 and wdiff == 0.0
    else:
        # what ships (autotuned split-K, float-atomic statistics): every parameter's gradient of
        # the data-parallel step within the bf16 floor of the fp32 reference (and the
        # single-device program's too, which validates the reference itself)
        ok = n_ops >= 2 and ran == 2 * n_ops and bad_dp == 0 and bad_ref == 0
    out["ok"] = bool(ok and comm.backend() == "nccl" and p.native_comm is not None)
    emit(out)
    m.impl.close()
    ref.impl.close()
    st.native_comm.close()


def case_central():
    """Fused DenseNet-121 steps through CentralStorageStrategy with the native reduce /
    broadcast (world of one) vs the single-device program, deterministic reductions."""
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model
    from idc_models_amd.parallel import CentralStorageStrategy, OneDeviceStrategy
    os.environ["IDC_DETERMINISTIC"] = "1"
    st = CentralStorageStrategy(force_collectives=True)
    m = Model(build_model("densenet121", None, 1, seed=9), st)
    m.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="fused")
    ref = Model(build_model("densenet121", None, 1, seed=9), OneDeviceStrategy("cuda:0"))
    ref.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="fused")
    g = torch.Generator().manual_seed(4)
    x = torch.randint(0, 256, (32, 50, 50, 3), generator=g, dtype=torch.uint8)
    y = torch.randint(0, 2, (32,), generator=g)
    nc = st.native_comm
    c0 = nc.collectives if nc is not None else 0
    for _ in range(2):
        m.impl.train_step(x, y)
        ref.impl.train_step(x, y)
    torch.cuda.synchronize()
    gdiff = float((m.arena.grad - ref.arena.grad).abs().max())
    wdiff = float((m.arena.data - ref.arena.data).abs().max())
    ran = (nc.collectives - c0) if nc is not None else 0
    ok = nc is not None and gdiff == 0.0 and wdiff == 0.0 and ran == 4  # reduce + broadcast per step
    emit({"case": "central", "ok": bool(ok), "grad_max_diff": gdiff, "weight_max_diff": wdiff,
          "collectives": ran})
    m.impl.close()
    ref.impl.close()
    st.native_comm.close()
    os.environ["IDC_DETERMINISTIC"] = "0"


def case_masked(dev):
    from idc_models_amd.fed.secagg import MaskedAggregator
    from idc_models_amd.parallel import comm
    agg = MaskedAggregator(2, [0, 1], dev)
    gen = torch.Generator(device="cpu").manual_seed(5)
    sizes = [1000, 37, 4096]
    v0 = torch.randn(sum(sizes), generator=gen).to(dev)
    v1 = torch.randn(sum(sizes), generator=gen).to(dev) * 3
    tot = agg.masked_sum({0: v0, 1: v1}, sizes, round_=1)
    ref = v0 + v1
    # per element: one quantum of rounding per client, plus the float32 rounding of the decoded
    # sum (the int32 fixed-point total converts to float32 with a 24-bit mantissa)
    q = float(1.0 / min(agg.last_scales))
    err = float(((tot - ref).abs() - ref.abs() * 2.0 ** -22).max())
    tol = 2 * q
    emit({"case": "masked", "ok": bool(err <= tol and comm.backend() == "nccl"), "err": err, "tol": tol})


def case_fedavg(dev):
    import torch.distributed as dist
    from idc_models_amd.parallel import comm
    a = torch.randn(333, device=dev)
    b = torch.arange(7, dtype=torch.float64, device=dev)
    ra, rb = comm.pack_all_reduce([a, b])
    c = torch.randn(55, device=dev)
    d = c.clone()
    comm.broadcast_(d, 0)
    mx = comm.all_reduce_max(3.5, dev)
    torch.cuda.synchronize()
    ok = (torch.allclose(ra, a) and torch.equal(rb, b) and torch.equal(c, d) and mx == 3.5
          and comm.is_dist() and dist.get_backend() == "nccl")
    emit({"case": "fedavg", "ok": bool(ok)})


def main():
    os.environ["IDC_FORCE_COLLECTIVES"] = "1"
    from idc_models_amd.parallel import MirroredStrategy
    cases = sys.argv[1].split(",") if len(sys.argv) > 1 else ["native", "nonblocking", "dp_det", "dp_tuned",
                                                              "central", "masked", "fedavg"]
    st = MirroredStrategy(force_collectives=True)
    assert st.native_comm is not None, "no native communicator on a nccl GPU rank"
    for c in cases:
        if c == "native":
            case_native(st)
        elif c == "nonblocking":
            case_nonblocking(st)
        elif c == "dp_det":
            case_dp(True)
        elif c == "dp_tuned":
            case_dp(False)
        elif c == "central":
            case_central()
        elif c == "masked":
            case_masked(st.device)
        elif c == "fedavg":
            case_fedavg(st.device)
    st.close()


if __name__ == "__main__":
    main()
