"""Numerics of every HIP kernel vs a plain PyTorch fp32 reference of the same op.

Shapes are the shape classes of SURVEY §2.4: 1x1 with K-tails (Cin = 64+32k), 3x3 s1 'same'
with N=32 outputs, the 7x7 s2 stem on a channel-padded image, 3x3 s2 with Keras' asymmetric
correct_pad, M tails, fp32 gradient operands, pending-BN prologues and BN-backward epilogues.
bf16 tolerances: inputs are rounded to bf16 before the reference so only accumulation differs.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def bf(x):
    return x.to(torch.bfloat16).float()


def relerr(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def ref_conv(x_nhwc, w_hwio, stride, pads_tblr, bias=None, act=0):
    x = x_nhwc.permute(0, 3, 1, 2)
    t, bo, l, r = pads_tblr
    x = F.pad(x, (l, r, t, bo))
    y = F.conv2d(x, w_hwio.permute(3, 2, 0, 1), bias, stride=stride)
    if act == 1:
        y = F.relu(y)
    return y.permute(0, 2, 3, 1)


def bn_ref(x, stats, gamma, beta, count, eps, act):
    C = x.shape[-1]
    mean = stats[:C] / count
    var = (stats[C:] / count - mean * mean).clamp_min(0)
    z = (x - mean) * torch.rsqrt(var + eps) * gamma + beta
    if act == 1:
        z = F.relu(z)
    elif act == 2:
        z = z.clamp(0, 6)
    return z


@pytest.fixture(scope="module")
def fn():
    from idc_models_amd.ops import functional as fn
    fn.nat.require()
    return fn


@pytest.mark.parametrize("N,H,Cin,Cout,k,s,pads,outhw", [
    (2, 13, 96, 128, 1, 1, (0, 0, 0, 0), None),     # DenseNet 1x1, K tail (96 = 64+32)
    (2, 13, 128, 32, 3, 1, (1, 1, 1, 1), None),     # DenseNet 3x3 growth conv
    (3, 7, 224, 128, 1, 1, (0, 0, 0, 0), None),     # M tail
    (2, 50, 8, 64, 7, 2, (3, 3, 3, 3), None),       # stem 7x7 s2 on padded image
    (2, 50, 8, 32, 3, 2, (0, 1, 0, 1), (25, 25)),   # MobileNetV2 Conv1 correct_pad
    (2, 25, 64, 128, 3, 1, (1, 1, 1, 1), None),     # VGG block2_conv1
    (1, 3, 512, 512, 3, 1, (1, 1, 1, 1), None),     # VGG block5 tiny M
])
def test_conv_fwd(fn, N, H, Cin, Cout, k, s, pads, outhw):
    x = bf(torch.randn(N, H, H, Cin, device=DEV))
    w = bf(torch.randn(k, k, Cin, Cout, device=DEV) * (2.0 / (k * k * Cin)) ** 0.5)
    bias = torch.randn(Cout, device=DEV) * 0.1
    ho = outhw or ((H + pads[0] + pads[1] - k) // s + 1,) * 2
    y = fn.conv2d(x.to(torch.bfloat16), w, stride=(s, s), pads=(pads[0], pads[2]), out_hw=ho,
                  bias=bias, act=1, out_f32=True)
    ref = ref_conv(x, w, s, pads, bias, act=1)
    assert y.shape == ref.shape
    assert relerr(y, ref) < 1e-2


@pytest.mark.parametrize("tile", list(range(23)))
def test_conv_every_tile_large_m_odd_ktiles(fn, tile):
    """Every tile config at scale: M = 40000 with an odd K-tile count (K = 392 -> 7 / 13 tiles)
    exercises the pipeline tail + epilogue LDS aliasing (a missing barrier once raced here)."""
    N, H, Cin, Cout = 64, 50, 8, 64
    x = bf(torch.randn(N, H, H, Cin, device=DEV))
    w = bf(torch.randn(7, 7, Cin, Cout, device=DEV) * 0.05)
    st = torch.zeros(2 * Cout, device=DEV)
    y = fn.conv2d(x.to(torch.bfloat16), w, stride=(2, 2), pads=(3, 3), out_f32=True, tile=tile, stats=st)
    ref = ref_conv(x, w, 2, (3, 3, 3, 3))
    assert relerr(y, ref) < 1e-2
    assert relerr(st[:Cout], ref.sum((0, 1, 2))) < 1e-2


@pytest.mark.parametrize("N,H,k,s,pads,cout,bias", [
    (64, 50, 7, 2, (3, 3, 3, 3), 64, False),   # DenseNet-121 conv1/conv (ZeroPadding2D(3))
    (37, 50, 3, 2, (0, 1, 0, 1), 32, False),   # MobileNetV2 Conv1 (correct_pad), odd batch
    (8, 50, 3, 1, (1, 1, 1, 1), 64, True),     # VGG16 block1_conv1 (bias + ReLU)
    (3, 32, 3, 1, (1, 1, 1, 1), 16, True),     # one column fragment, CIFAR-sized maps
])
def test_conv_stem_matches_reference(fn, N, H, k, s, pads, cout, bias):
    """Image-resident stem conv (conv_stem.hip, tile TILE_STEM): 8-channel staged images (RGB +
    zero channels, as the input op stores them), the band's input rows in LDS, bf16 output with
    bias + activation and shifted output statistics, vs fp32 PyTorch on the same bf16 operands."""
    ext = fn.nat.require()
    g = torch.Generator(device="cpu").manual_seed(N + k)
    x = torch.zeros(N, H, H, 8)
    x[..., :3] = torch.rand(N, H, H, 3, generator=g)
    x = bf(x.to(DEV))
    w = torch.zeros(k, k, 8, cout)
    w[:, :, :3] = torch.randn(k, k, 3, cout, generator=g) * (2.0 / (k * k * 3)) ** 0.5
    w = bf(w.to(DEV))
    b = (torch.randn(cout, generator=g) * 0.1).to(DEV) if bias else None
    ho = (H + pads[0] + pads[1] - k) // s + 1
    K = (torch.randn(cout, generator=g) * 0.1).to(DEV)
    st = torch.zeros(2 * cout, device=DEV)
    y = fn.conv2d(x.to(torch.bfloat16), w, stride=(s, s), pads=(pads[0], pads[2]), out_hw=(ho, ho), bias=b,
                  act=1 if bias else 0, tile=ext.TILE_STEM, stats=st, stats_shift=K)
    ref = ref_conv(x, w, s, pads, b, act=1 if bias else 0)
    assert y.shape == ref.shape
    assert relerr(y.float(), ref) < 1e-2
    yk = y.float().reshape(-1, cout) - K
    assert relerr(st[:cout], yk.sum(0)) < 1e-3 and relerr(st[cout:], (yk * yk).sum(0)) < 1e-3


@pytest.mark.parametrize("tile,ks", [(4, 2), (9, 4), (12, 2), (17, 2), (18, 4), (8, 8), (7, 3), (19, 4), (22, 2)])
def test_conv_split_k_matches_reference(fn, tile, ks):
    """Split-K (in-launch last-arriver reduction) on a small-M deep-K layer with the BN prologue
    and output statistics; launched three times to check the modulo tickets realign."""
    N, H, Cin, Cout = 16, 6, 480, 128
    x = bf(torch.randn(N, H, H, Cin, device=DEV))
    w = bf(torch.randn(1, 1, Cin, Cout, device=DEV) * 0.05)
    st_in = torch.cat([x.sum((0, 1, 2)), (x * x).sum((0, 1, 2))])
    g = torch.rand(Cin, device=DEV) + 0.5
    be = torch.randn(Cin, device=DEV) * 0.1
    bn = fn.BN(stats=st_in, gamma=g, beta=be, count=N * H * H, eps=1e-3, act=1)
    mean = x.mean((0, 1, 2))
    var = (x * x).mean((0, 1, 2)) - mean * mean
    xa = torch.relu((x - mean) / torch.sqrt(var + 1e-3) * g + be)
    ref = ref_conv(xa, w, 1, (0, 0, 0, 0))
    for _ in range(3):
        st = torch.zeros(2 * Cout, device=DEV)
        y = fn.conv2d(x.to(torch.bfloat16), w, pro=bn, out_f32=True, tile=tile, stats=st, ksplit=ks)
        assert relerr(y, ref) < 1e-2
        assert relerr(st[:Cout], ref.sum((0, 1, 2))) < 1e-2


def test_conv_dgrad_split_k(fn):
    N, H, Cin, Cout = 16, 3, 128, 32
    dy = bf(torch.randn(N, H, H, Cout, device=DEV))
    w = bf(torch.randn(3, 3, Cin, Cout, device=DEV) * 0.05)
    ref = torch.nn.grad.conv2d_input((N, Cin, H, H), w.permute(3, 2, 0, 1), dy.permute(0, 3, 1, 2),
                                     padding=1).permute(0, 2, 3, 1)
    dx = fn.conv2d_dgrad(dy.to(torch.bfloat16), w, (H, H), pads=(1, 1), out_f32=True, tile=9, ksplit=4)
    assert relerr(dx, ref) < 1e-2


def test_conv_fwd_asymmetric_B(fn):
    """A = identity-like input, asymmetric B: catches a transposed C write (guide §3)."""
    N, H, C = 1, 4, 16
    x = torch.zeros(N, H, H, C, device=DEV)
    for i in range(16):
        x[0, i // 4, i % 4, i] = 1.0
    w = torch.arange(C * 32, device=DEV, dtype=torch.float32).reshape(1, 1, C, 32) / 64.0
    y = fn.conv2d(x.to(torch.bfloat16), w, out_f32=True)
    ref = ref_conv(x, bf(w), 1, (0, 0, 0, 0))
    assert torch.allclose(y, ref, atol=1e-2)


def test_conv_prologue_bn_relu_and_stats(fn):
    N, H, Cin, Cout = 4, 13, 160, 128
    x = bf(torch.randn(N, H, H, Cin, device=DEV) * 2 + 0.5)
    st = torch.cat([x.sum((0, 1, 2)), (x * x).sum((0, 1, 2))])
    gamma = torch.rand(Cin, device=DEV) + 0.5
    beta = torch.randn(Cin, device=DEV) * 0.1
    w = bf(torch.randn(1, 1, Cin, Cout, device=DEV) * 0.1)
    stats_out = torch.zeros(2 * Cout, device=DEV)
    cnt = N * H * H
    y = fn.conv2d(x.to(torch.bfloat16), w, pro=fn.BN(stats=st, gamma=gamma, beta=beta, count=cnt,
                  eps=1.001e-5, act=1), stats=stats_out)
    a = bn_ref(x, st, gamma, beta, cnt, 1.001e-5, 1)
    ref = ref_conv(bf(a), w, 1, (0, 0, 0, 0))
    assert relerr(y, ref) < 1e-2
    yf = y.float()
    assert relerr(stats_out[:Cout], yf.sum((0, 1, 2))) < 1e-3
    assert relerr(stats_out[Cout:], (yf * yf).sum((0, 1, 2))) < 1e-3


def test_conv_fp32_operand(fn):
    N, H, Cin, Cout = 2, 13, 32, 128
    x = torch.randn(N, H, H, Cin, device=DEV)
    w = bf(torch.randn(3, 3, Cin, Cout, device=DEV) * 0.1)
    y = fn.conv2d(x, w, pads=(1, 1), out_f32=True)
    ref = ref_conv(bf(x), w, 1, (1, 1, 1, 1))
    assert relerr(y, ref) < 1e-2


@pytest.mark.parametrize("N,H,Cin,Cout,k", [(2, 13, 128, 32, 3), (2, 13, 96, 128, 1), (3, 6, 64, 64, 3)])
def test_conv_dgrad(fn, N, H, Cin, Cout, k):
    p = k // 2
    dy = bf(torch.randn(N, H, H, Cout, device=DEV))
    w = bf(torch.randn(k, k, Cin, Cout, device=DEV) * 0.1)
    dx = fn.conv2d_dgrad(dy.to(torch.bfloat16), w, (H, H), pads=(p, p), out_f32=True)
    ref = torch.nn.grad.conv2d_input((N, Cin, H, H), w.permute(3, 2, 0, 1), dy.permute(0, 3, 1, 2),
                                     padding=p).permute(0, 2, 3, 1)
    assert relerr(dx, ref) < 1e-2


def test_conv_dgrad_bn_epilogue(fn):
    N, H, Cin, Cout = 4, 6, 128, 32
    mx = bf(torch.randn(N, H, H, Cin, device=DEV))
    st = torch.cat([mx.sum((0, 1, 2)), (mx * mx).sum((0, 1, 2))])
    gamma = torch.rand(Cin, device=DEV) + 0.5
    beta = torch.randn(Cin, device=DEV) * 0.1
    cnt = N * H * H
    dy = bf(torch.randn(N, H, H, Cout, device=DEV))
    w = bf(torch.randn(3, 3, Cin, Cout, device=DEV) * 0.1)
    gsum = torch.zeros(Cin, device=DEV)
    gsumx = torch.zeros(Cin, device=DEV)
    dz = fn.conv2d_dgrad(dy.to(torch.bfloat16), w, (H, H), pads=(1, 1), mx=mx.to(torch.bfloat16),
                         mbn=fn.BN(stats=st, gamma=gamma, beta=beta, count=cnt, eps=1e-3, act=1),
                         gsum=gsum, gsumx=gsumx)
    dA = torch.nn.grad.conv2d_input((N, Cin, H, H), w.permute(3, 2, 0, 1), dy.permute(0, 3, 1, 2),
                                    padding=1).permute(0, 2, 3, 1)
    mean = st[:Cin] / cnt
    var = st[Cin:] / cnt - mean ** 2
    xhat = (mx - mean) * torch.rsqrt(var + 1e-3)
    z = xhat * gamma + beta
    dZ = dA * (z > 0).float()
    assert relerr(dz, dZ) < 1e-2
    assert relerr(gsum, dZ.sum((0, 1, 2))) < 2e-2
    assert relerr(gsumx, (dZ * xhat).sum((0, 1, 2))) < 2e-2


@pytest.mark.parametrize("N,H,Cin,Cout,k,s,pads,gf32", [
    (4, 13, 128, 32, 3, 1, (1, 1), True),     # DenseNet 3x3 (fp32 concat grads)
    (4, 13, 96, 128, 1, 1, (0, 0), False),    # DenseNet 1x1
    (2, 25, 64, 128, 3, 1, (1, 1), False),    # VGG
    (2, 50, 8, 64, 7, 2, (3, 3), False),      # stem (padded channels)
])
def test_conv_wgrad(fn, N, H, Cin, Cout, k, s, pads, gf32):
    x = bf(torch.randn(N, H, H, Cin, device=DEV))
    Ho = (H + 2 * pads[0] - k) // s + 1
    dy = torch.randn(N, Ho, Ho, Cout, device=DEV)
    dyb = dy if gf32 else dy.to(torch.bfloat16)
    dw = fn.conv2d_wgrad(x.to(torch.bfloat16), dyb, (k, k), stride=(s, s), pads=pads)
    ref = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2), (Cout, Cin, k, k), bf(dy).permute(0, 3, 1, 2),
                                      stride=s, padding=pads[0]).permute(2, 3, 1, 0)
    assert relerr(dw, ref) < 1e-2


def test_conv_wgrad_prologue_and_cin_real(fn):
    N, H, Cin, Cout = 2, 50, 8, 64
    x = torch.zeros(N, H, H, Cin, device=DEV)
    x[..., :3] = torch.rand(N, H, H, 3, device=DEV)
    x = bf(x)
    dy = bf(torch.randn(N, 25, 25, Cout, device=DEV))
    dw = fn.conv2d_wgrad(x.to(torch.bfloat16), dy.to(torch.bfloat16), (7, 7), stride=(2, 2), pads=(3, 3),
                         cin_real=3)
    ref = torch.nn.grad.conv2d_weight(x[..., :3].permute(0, 3, 1, 2), (Cout, 3, 7, 7), dy.permute(0, 3, 1, 2),
                                      stride=2, padding=3).permute(2, 3, 1, 0)
    assert dw.shape == (7, 7, 3, 64)
    assert relerr(dw, ref) < 1e-2


@pytest.mark.parametrize("N,H,k,s,pads,ho,cout,aff", [
    (64, 50, 7, 2, (3, 3), 25, 64, True),    # DenseNet-121 stem, G through the stem BN's backward
    (37, 50, 3, 2, (0, 0), 25, 32, False),   # MobileNetV2 Conv1 (correct_pad: bottom/right implicit)
    (8, 50, 3, 1, (1, 1), 50, 64, False),    # VGG16 block1_conv1
    (3, 32, 3, 1, (1, 1), 32, 16, True),
])
def test_wgrad_stem_matches_reference(fn, N, H, k, s, pads, ho, cout, aff):
    """Image-resident stem weight gradient (wgrad_stem.hip, taken by conv_wgrad whenever it
    applies): 8-channel staged images with 3 real channels, dW over the real channels only; with
    ``aff`` the gradient is the stem BatchNorm's pending backward A*g + B*x + C."""
    g = torch.Generator(device="cpu").manual_seed(N * 3 + k)
    x = torch.zeros(N, H, H, 8)
    x[..., :3] = torch.rand(N, H, H, 3, generator=g)
    x = bf(x.to(DEV))
    if aff:
        kc = _bn_case(N, ho, cout, seed=N + 1)
        gin = kc["dZ"].to(torch.bfloat16)
        gp = fn.bwd_aff(kc["x"].to(torch.bfloat16), kc["bn"], kc["gsum"], kc["gsumx"])
        dy = bf(kc["dX"])
    else:
        dy = bf(torch.randn(N, ho, ho, cout, generator=g).to(DEV))
        gin, gp = dy.to(torch.bfloat16), None
    dw = fn.conv2d_wgrad(x.to(torch.bfloat16), gin, (k, k), stride=(s, s), pads=pads, cin_real=3, gpro=gp)
    L = (ho - 1) * s + k  # the padded extent the output reads (top/left pad, implicit bottom/right)
    xr = F.pad(x[..., :3].permute(0, 3, 1, 2), (pads[1], L, pads[0], L))[:, :, :L, :L]
    ref = torch.nn.grad.conv2d_weight(xr, (cout, 3, k, k), dy.permute(0, 3, 1, 2), stride=s)
    ref = ref.permute(2, 3, 1, 0)
    assert dw.shape == (k, k, 3, cout)
    assert relerr(dw, ref) < 2e-2


def test_wgrad_with_bn_prologue(fn):
    N, H, Cin, Cout = 4, 13, 128, 32
    t = bf(torch.randn(N, H, H, Cin, device=DEV))
    st = torch.cat([t.sum((0, 1, 2)), (t * t).sum((0, 1, 2))])
    g, b = torch.rand(Cin, device=DEV) + 0.5, torch.randn(Cin, device=DEV) * 0.1
    dy = bf(torch.randn(N, H, H, Cout, device=DEV))
    cnt = N * H * H
    dw = fn.conv2d_wgrad(t.to(torch.bfloat16), dy.to(torch.bfloat16), (3, 3), pads=(1, 1),
                         pro=fn.BN(stats=st, gamma=g, beta=b, count=cnt, eps=1e-3, act=1))
    a = bf(bn_ref(t, st, g, b, cnt, 1e-3, 1))
    ref = torch.nn.grad.conv2d_weight(a.permute(0, 3, 1, 2), (Cout, Cin, 3, 3), dy.permute(0, 3, 1, 2),
                                      padding=1).permute(2, 3, 1, 0)
    assert relerr(dw, ref) < 1.5e-2


def test_maxpool_fwd_bwd_stem(fn):
    N, H, C = 2, 25, 64
    y = bf(torch.randn(N, H, H, C, device=DEV))
    st = torch.cat([y.sum((0, 1, 2)), (y * y).sum((0, 1, 2))])
    g, b = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.1
    cnt = N * H * H
    bn = fn.BN(stats=st, gamma=g, beta=b, count=cnt, eps=1.001e-5, act=1)
    out_stats = torch.zeros(2 * C, device=DEV)
    p, am = fn.pool2d(y.to(torch.bfloat16), 3, 2, pads=(1, 1), is_max=True, pro=bn, stats=out_stats)
    a = bn_ref(y, st, g, b, cnt, 1.001e-5, 1).requires_grad_(True)
    ap = F.pad(a.permute(0, 3, 1, 2), (1, 1, 1, 1))
    ref = F.max_pool2d(ap, 3, 2).permute(0, 2, 3, 1)
    assert relerr(p, ref) < 1e-2
    assert relerr(out_stats[:C], p.float().sum((0, 1, 2))) < 1e-3
    dp = torch.randn_like(ref)
    ref.backward(dp)
    gsum = torch.zeros(C, device=DEV)
    gsumx = torch.zeros(C, device=DEV)
    dz = fn.pool2d_bwd(dp.contiguous(), (N, H, H, C), 3, 2, pads=(1, 1), is_max=True, argmax=am,
                       x=y.to(torch.bfloat16), bn=bn, gsum=gsum, gsumx=gsumx)
    # reference dZ (grad wrt BN pre-activation)
    z = bn_ref(y, st, g, b, cnt, 1.001e-5, 0)
    dZ = a.grad * (z > 0).float()
    assert relerr(dz, dZ) < 2e-2


def test_avgpool_fwd_bwd(fn):
    N, H, C = 2, 13, 256
    x = bf(torch.randn(N, H, H, C, device=DEV))
    p, _ = fn.pool2d(x.to(torch.bfloat16), 2, 2, is_max=False)
    ref = F.avg_pool2d(x.permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1)
    assert p.shape == ref.shape == (N, 6, 6, C)
    assert relerr(p, ref) < 1e-2
    dp = torch.randn(N, 6, 6, C, device=DEV)
    dx = fn.pool2d_bwd(dp.to(torch.bfloat16), (N, H, H, C), 2, 2, is_max=False)
    xr = x.clone().requires_grad_(True)
    F.avg_pool2d(xr.permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1).backward(bf(dp))
    assert relerr(dx, xr.grad) < 1e-2


def test_bn_backward_pair_matches_autograd(fn):
    N, H, C = 4, 6, 64
    x = bf(torch.randn(N, H, H, C, device=DEV) * 3 + 1)
    st = torch.cat([x.sum((0, 1, 2)), (x * x).sum((0, 1, 2))])
    g, b = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.1
    cnt = N * H * H
    xr = x.clone().requires_grad_(True)
    mean = xr.mean((0, 1, 2))
    var = xr.var((0, 1, 2), unbiased=False)
    gr, br = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    y = F.relu((xr - mean) * torch.rsqrt(var + 1e-3) * gr + br)
    dy = torch.randn_like(y)
    y.backward(dy)
    bn = fn.BN(stats=st, gamma=g, beta=b, count=cnt, eps=1e-3, act=1)
    gsum = torch.zeros(C, device=DEV)
    gsumx = torch.zeros(C, device=DEV)
    dz = fn.bn_bwd_reduce(dy, x.to(torch.bfloat16), bn, gsum, gsumx)
    dx = fn.bn_bwd_apply(dz, x.to(torch.bfloat16), bn, gsum, gsumx, out_f32=True)
    assert relerr(gsum, br.grad) < 2e-2
    assert relerr(gsumx, gr.grad) < 2e-2
    assert relerr(dx, xr.grad) < 3e-2


def test_bn_stats(fn):
    x = bf(torch.randn(3, 7, 7, 96, device=DEV))
    st = fn.bn_stats(x.to(torch.bfloat16))
    assert relerr(st[:96], x.sum((0, 1, 2))) < 1e-4
    assert relerr(st[96:], (x * x).sum((0, 1, 2))) < 1e-4


@pytest.mark.parametrize("s,H,pads,ho,C", [(1, 13, (1, 1), 13, 96), (2, 26, (0, 0), 13, 96), (2, 13, (1, 1), 7, 96),
                                            (1, 4, (1, 1), 4, 384), (2, 4, (0, 0), 2, 960),
                                            (1, 25, (1, 1), 25, 32), (1, 13, (1, 1), 13, 144)])
def test_dwconv(fn, s, H, pads, ho, C):
    N = 2
    x = bf(torch.randn(N, H, H, C, device=DEV))
    k = torch.randn(3, 3, C, 1, device=DEV) * 0.3
    y = fn.dwconv(x.to(torch.bfloat16), k, stride=s, pads=pads, out_hw=(ho, ho))
    # Keras: stride-2 uses explicit correct_pad (top/left pads[0], bottom/right enough for ho).
    # The fp32 reference runs on the CPU: with MIOpen off (tests/conftest.py) PyTorch-ROCm's own
    # grouped-conv backward returned a wrong input gradient here (rel 1.41 against our kernel)
    xr = x.cpu().clone().requires_grad_(True)
    xp = F.pad(xr.permute(0, 3, 1, 2), (pads[1], 2, pads[0], 2))
    kr = k.cpu().clone().requires_grad_(True)
    ref = F.conv2d(xp, kr.permute(2, 3, 0, 1), stride=s, groups=C)[:, :, :ho, :ho].permute(0, 2, 3, 1)
    assert relerr(y.cpu(), ref) < 1e-2
    dy = bf(torch.randn_like(ref))
    ref.backward(dy)
    dx, dw = fn.dwconv_bwd(x.to(torch.bfloat16), k, dy.to(DEV).to(torch.bfloat16), stride=s, pads=pads)
    assert relerr(dx.cpu(), xr.grad) < 1e-2
    assert relerr(dw.cpu(), kr.grad) < 1e-2


@pytest.mark.parametrize("H,C,pro", [(13, 144, False), (13, 144, True), (25, 32, True), (7, 192, True),
                                     (4, 384, True), (2, 960, True), (5, 24, True)])
def test_dwconv_bwd_fused_matches_separate_kernels(fn, H, C, pro):
    """The one-pass stride-1 depthwise backward (dw_bwd3_fused_kernel: data gradient through the
    pending BN + ReLU6 and its BatchNorm-backward sums, weight-gradient partials + column sums) vs
    the data-gradient and weight-gradient kernels it replaces (themselves checked against fp32
    autograd in test_dwconv), and without a prologue vs fp32 autograd on the CPU directly."""
    N = 3
    torch.manual_seed(H * 10 + C)
    x = bf(torch.randn(N, H, H, C, device=DEV) * 2 + 0.3)
    k = torch.randn(3, 3, C, 1, device=DEV) * 0.3
    dy = bf(torch.randn(N, H, H, C, device=DEV))
    bn = None
    if pro:
        st = torch.cat([x.sum((0, 1, 2)), (x * x).sum((0, 1, 2))])
        bn = fn.BN(stats=st, gamma=torch.rand(C, device=DEV) + 0.5, beta=torch.randn(C, device=DEV) * 0.1,
                   count=N * H * H, eps=1e-3, act=2)
    xb, dyb = x.to(torch.bfloat16), dy.to(torch.bfloat16)
    sums = [torch.zeros(C, device=DEV) for _ in range(4)]
    dx0, dw0 = fn.dwconv_bwd(xb, k, dyb, stride=1, pads=(1, 1), pro=bn, gsum=sums[0] if pro else None,
                             gsumx=sums[1] if pro else None)
    dx1, dw1 = fn.dwconv_bwd_fused(xb, k, dyb, pads=(1, 1), pro=bn, gsum=sums[2] if pro else None,
                                   gsumx=sums[3] if pro else None)
    assert relerr(dx1, dx0) < 4e-3, relerr(dx1, dx0)
    assert relerr(dw1, dw0) < 1e-4, relerr(dw1, dw0)
    if pro:
        assert relerr(sums[2], sums[0]) < 4e-3 and relerr(sums[3], sums[1]) < 4e-3
    else:
        xr = x.cpu().clone()
        kr = k.cpu().clone().requires_grad_(True)
        xr.requires_grad_(True)
        ref = F.conv2d(F.pad(xr.permute(0, 3, 1, 2), (1, 1, 1, 1)), kr.permute(2, 3, 0, 1), groups=C)
        ref.backward(dy.cpu().permute(0, 3, 1, 2))
        assert relerr(dx1.cpu(), xr.grad) < 1e-2
        assert relerr(dw1.cpu(), kr.grad) < 1e-2


def test_rmsprop_kernel_matches_keras_formula():
    from idc_models_amd.ops.optim import rmsprop_
    n = 4096
    w = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV)
    ms = torch.rand(n, device=DEV)
    w0, ms0 = w.clone(), ms.clone()
    rmsprop_(w, g, ms, 1e-3, 0.9, 1e-7, 0.5)
    gs = g * 0.5
    ms_ref = 0.9 * ms0 + 0.1 * gs * gs
    w_ref = w0 - 1e-3 * gs / (ms_ref.sqrt() + 1e-7)
    assert torch.allclose(ms, ms_ref, rtol=1e-5, atol=1e-7)
    assert torch.allclose(w, w_ref, rtol=1e-5, atol=1e-6)


def test_secagg_masks_cancel_exactly():
    from idc_models_amd.fed.keyagree import ClientKeys
    from idc_models_amd.fed.secagg import mask_quantize, segment_ends, unmask
    K, sizes = 5, [10000, 7]
    n = sum(sizes)
    seg = segment_ends(sizes)
    scales = [2.0 ** 16, 2.0 ** 10]
    ks = {k: ClientKeys(k) for k in range(K)}
    pubs = {k: ks[k].public for k in range(K)}
    rk = {k: ks[k].round_keys(pubs, 7, range(K)) for k in range(K)}
    xs = [torch.randn(n, device=DEV) for _ in range(K)]
    masked = [mask_quantize(x, scales, seg, K, r, rk[r], round_=7) for r, x in enumerate(xs)]
    total = torch.zeros(n, dtype=torch.int64, device=DEV)
    for m in masked:
        total = (total + m.to(torch.int64)) % (1 << 32)
    s32 = torch.where(total >= (1 << 31), total - (1 << 32), total).to(torch.int32)
    sc = torch.tensor([scales[0]] * sizes[0] + [scales[1]] * sizes[1], device=DEV)
    plain = sum(torch.round(x * sc).to(torch.int64) for x in xs)
    assert torch.equal(s32.to(torch.int64), plain)
    mean = unmask(s32, scales, seg, K)
    assert torch.allclose(mean, sum(xs) / K, atol=K / min(scales))
    # CPU numpy Philox produces the same bits as the GPU kernel
    cpu = mask_quantize(xs[1].cpu(), scales, seg, K, 1, rk[1], round_=7)
    assert torch.equal(cpu, masked[1].cpu())


# ---------------------------------------------------------------------------------------------
# Backward pending affine (csrc/kernels/common.h BwdAff): BatchNorm backward applied by consumers
def _bn_case(N, H, C, x=None, seed=0, act=0):
    """raw x, BN descriptor, upstream dZ (grad wrt the BN output), reductions and autograd dX."""
    from idc_models_amd.ops import functional as fn
    g0 = torch.Generator(device=DEV).manual_seed(seed)
    if x is None:
        x = bf(torch.randn(N, H, H, C, device=DEV, generator=g0) * 2 + 0.5)
    st = torch.cat([x.sum((0, 1, 2)), (x * x).sum((0, 1, 2))])
    g = torch.rand(C, device=DEV, generator=g0) + 0.5
    b = torch.randn(C, device=DEV, generator=g0) * 0.1
    cnt = N * H * H
    dZ = bf(torch.randn(N, H, H, C, device=DEV, generator=g0))
    xr = x.clone().requires_grad_(True)
    mean, var = xr.mean((0, 1, 2)), xr.var((0, 1, 2), unbiased=False)
    ((xr - mean) * torch.rsqrt(var + 1e-3) * g + b).backward(dZ)
    rstd = torch.rsqrt(x.var((0, 1, 2), unbiased=False) + 1e-3)
    xhat = (x - x.mean((0, 1, 2))) * rstd
    gsum, gsumx = dZ.sum((0, 1, 2)), (dZ * xhat).sum((0, 1, 2))
    bn = fn.BN(stats=st, gamma=g, beta=b, count=cnt, eps=1e-3, act=act)
    return dict(x=x, bn=bn, dZ=dZ, gsum=gsum, gsumx=gsumx, dX=xr.grad, A=g * rstd, xhat=xhat)


def test_dgrad_bwd_affine_prologue_1x1(fn):
    """DenseNet dgrad cv1: the operand is z2 = dZ of bn2, staged as A*z2 + B*t + C (= dt)."""
    N, H, C, cin = 4, 13, 128, 96
    k = _bn_case(N, H, C)
    w = bf(torch.randn(1, 1, cin, C, device=DEV) * 0.1)
    x16 = k["x"].to(torch.bfloat16)
    aff = fn.bwd_aff(x16, k["bn"], k["gsum"], k["gsumx"])
    out = fn.conv2d_dgrad(k["dZ"].to(torch.bfloat16), w, (H, H), bpro=aff, out_f32=True)
    ref = torch.nn.grad.conv2d_input((N, cin, H, H), w.permute(3, 2, 0, 1),
                                     bf(k["dX"]).permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
    assert relerr(out, ref) < 2e-2


@pytest.mark.parametrize("ksplit,tile", [(1, -1), (2, 9), (4, 12)])
def test_dgrad_bwd_affine_unit_alpha_3x3_fp32_and_fold(fn, ksplit, tile):
    """DenseNet dgrad cv2: fp32 concat-gradient operand already holding A*dZ; B*x + C of the
    pending BatchNorm added while staging; block 0 folds the reductions into d beta / d gamma."""
    N, H, C, cin = 4, 6, 32, 128
    k = _bn_case(N, H, C, seed=1)
    v = (k["dZ"] * k["A"]).contiguous()
    w = bf(torch.randn(3, 3, cin, C, device=DEV) * 0.1)
    db, dg = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    x16 = k["x"].to(torch.bfloat16)
    aff = fn.bwd_aff(x16, k["bn"], k["gsum"], k["gsumx"], unit_alpha=True, fold=(db, dg))
    staged = torch.zeros(N, H, H, C, dtype=torch.bfloat16, device=DEV)
    out = fn.conv2d_dgrad(v, w, (H, H), pads=(1, 1), bpro=aff, out_f32=True, ksplit=ksplit, tile=tile,
                          aout=staged)
    ref = torch.nn.grad.conv2d_input((N, cin, H, H), w.permute(3, 2, 0, 1),
                                     bf(k["dX"]).permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    assert relerr(out, ref) < 2e-2
    assert relerr(staged, k["dX"]) < 1e-2  # the staged operand, for the side-lane wgrad
    torch.cuda.synchronize()
    assert torch.equal(db, k["gsum"]) and torch.equal(dg, k["gsumx"])


@pytest.mark.parametrize("unit,Cout,k_", [(False, 128, 1), (True, 32, 3)])
def test_wgrad_bwd_affine_on_g(fn, unit, Cout, k_):
    """wgrad cv1 (G = A*z2 + B*t + C, bf16) and wgrad cv2 (G = fp32 concat grad + B*x + C)."""
    N, H, Cin = 4, 13, 64
    kc = _bn_case(N, H, Cout, seed=2)
    xin = bf(torch.randn(N, H, H, Cin, device=DEV))
    g = (kc["dZ"] * kc["A"]).contiguous() if unit else kc["dZ"].to(torch.bfloat16)
    x16 = kc["x"].to(torch.bfloat16)
    aff = fn.bwd_aff(x16, kc["bn"], kc["gsum"], kc["gsumx"], unit_alpha=unit)
    p = k_ // 2
    dw = fn.conv2d_wgrad(xin.to(torch.bfloat16), g, (k_, k_), pads=(p, p), gpro=aff)
    ref = torch.nn.grad.conv2d_weight(xin.permute(0, 3, 1, 2), (Cout, Cin, k_, k_),
                                      bf(kc["dX"]).permute(0, 3, 1, 2), padding=p).permute(2, 3, 1, 0)
    assert relerr(dw, ref) < 2e-2


def test_dgrad_epilogue_accumulates_concat_gradient(fn):
    """Epilogue mode 2: acc += gamma1*rstd1*dZ1 + (pending BatchNorm's B'*x + C') on the same x,
    with dZ1 = dA * relu'(bn1(x)) reduced into bn1's gsum / gsumx."""
    N, H, C, cin = 4, 6, 128, 160
    x = bf(torch.randn(N, H, H, cin, device=DEV) * 1.5 + 0.3)
    kb = _bn_case(N, H, cin, x=x, seed=3, act=1)   # bn1 of this layer (its dZ is computed here)
    kp = _bn_case(N, H, cin, x=x, seed=4)          # the pending BatchNorm over the same channels
    k2 = _bn_case(N, H, C, seed=7)                 # the operand: z2 = dZ of bn2, staged as dt
    t16, z16 = k2["x"].to(torch.bfloat16), k2["dZ"].to(torch.bfloat16)
    bpro = fn.bwd_aff(t16, k2["bn"], k2["gsum"], k2["gsumx"])
    w = bf(torch.randn(1, 1, cin, C, device=DEV) * 0.1)
    acc0 = torch.randn(N, H, H, cin, device=DEV)
    acc = acc0.clone()
    gsum, gsumx = torch.zeros(cin, device=DEV), torch.zeros(cin, device=DEV)
    x16 = x.to(torch.bfloat16)
    bepi = fn.bwd_aff(x16, kp["bn"], kp["gsum"], kp["gsumx"], unit_alpha=True)
    fn.conv2d_dgrad(z16, w, (H, H), mx=x16, mbn=kb["bn"], gsum=gsum, gsumx=gsumx, bpro=bpro, bepi=bepi, acc=acc)
    dy = bf(k2["dX"])
    dA = torch.nn.grad.conv2d_input((N, cin, H, H), w.permute(3, 2, 0, 1), dy.permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
    z = kb["xhat"] * kb["bn"].gamma + kb["bn"].beta
    dZ1 = dA * (z > 0).float()
    pend = kp["dX"] - kp["A"] * kp["dZ"]
    ref = acc0 + kb["A"] * dZ1 + pend
    assert relerr(acc - acc0, ref - acc0) < 2e-2
    assert relerr(gsum, dZ1.sum((0, 1, 2))) < 2e-2
    assert relerr(gsumx, (dZ1 * kb["xhat"]).sum((0, 1, 2))) < 2e-2


def test_pool_bwd_dy_affine_and_f32_output(fn):
    """Stem max-pool backward with dy = fp32 concat grad + pending B*x + C (x at the pool-output
    positions), and the transition avg-pool backward writing gamma*rstd*dZ in fp32."""
    N, H, C = 2, 25, 64
    y = bf(torch.randn(N, H, H, C, device=DEV))
    st = torch.cat([y.sum((0, 1, 2)), (y * y).sum((0, 1, 2))])
    g, b = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.1
    cnt = N * H * H
    bn = fn.BN(stats=st, gamma=g, beta=b, count=cnt, eps=1.001e-5, act=1)
    p, am = fn.pool2d(y.to(torch.bfloat16), 3, 2, pads=(1, 1), is_max=True, pro=bn)
    kp = _bn_case(N, 13, C, x=bf(p.float()), seed=5)
    dy = (kp["dZ"] * kp["A"]).contiguous()
    db, dg = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    aff = fn.bwd_aff(p, kp["bn"], kp["gsum"], kp["gsumx"], unit_alpha=True, fold=(db, dg))
    dz = fn.pool2d_bwd(dy, (N, H, H, C), 3, 2, pads=(1, 1), is_max=True, argmax=am, x=y.to(torch.bfloat16),
                       bn=bn, dyaff=aff)
    dz_ref = fn.pool2d_bwd(kp["dX"].contiguous(), (N, H, H, C), 3, 2, pads=(1, 1), is_max=True, argmax=am,
                           x=y.to(torch.bfloat16), bn=bn)
    assert relerr(dz, dz_ref) < 2e-2
    torch.cuda.synchronize()
    assert torch.equal(db, kp["gsum"]) and torch.equal(dg, kp["gsumx"])
    # transition form: avg-pool backward through bn, fp32 A*dZ output
    gs1, gx1 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    gs2, gx2 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    dq = bf(torch.randn(N, 12, 12, C, device=DEV))
    a32 = fn.pool2d_bwd(dq, (N, H, H, C), 2, 2, is_max=False, x=y.to(torch.bfloat16), bn=bn, gsum=gs1,
                        gsumx=gx1, out_f32=True)
    z16 = fn.pool2d_bwd(dq, (N, H, H, C), 2, 2, is_max=False, x=y.to(torch.bfloat16), bn=bn, gsum=gs2, gsumx=gx2)
    A = g * torch.rsqrt(st[C:] / cnt - (st[:C] / cnt) ** 2 + 1.001e-5)
    assert relerr(a32, z16.float() * A) < 1e-2
    assert relerr(gs1, gs2) < 1e-2 and relerr(gx1, gx2) < 1e-2


def test_bn_bwd_reduce_f32_scaled_output(fn):
    N, H, C = 4, 6, 64
    k = _bn_case(N, H, C, seed=6, act=1)
    dy = torch.randn(N, H, H, C, device=DEV)
    gs, gx = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    a = fn.bn_bwd_reduce(dy, k["x"].to(torch.bfloat16), k["bn"], gs, gx, dz_f32=True)
    z = k["xhat"] * k["bn"].gamma + k["bn"].beta
    dZ = dy * (z > 0).float()
    assert relerr(a, k["A"] * dZ) < 1e-2
    assert relerr(gs, dZ.sum((0, 1, 2))) < 1e-2


def test_bn_statistics_shifted_large_mean(fn):
    """Offset-heavy activations (VERDICT: mean 50, std 0.1): the conv epilogue's fp32 statistics
    cancel catastrophically in E[y^2] - E[y]^2, while statistics shifted by K (the previous step's
    batch mean, common.h "Shifted statistics") give the variance to fp64 accuracy."""
    g = torch.Generator(device="cpu").manual_seed(5)
    N, H, Cin, Cout = 16, 16, 64, 64          # 4096 rows
    x = (1.0 + 0.015 * torch.randn(N, H, H, Cin, generator=g)).to(DEV).to(torch.bfloat16)
    k = torch.full((1, 1, Cin, Cout), 25.0 / 32.0, device=DEV)  # exact in bf16: y = 0.78125 * sum(x)
    k[0, 0, :, 1::2] *= 0.5                                    # second mean level (~25) on odd channels
    M = N * H * H
    s0 = torch.zeros(2 * Cout, device=DEV)
    y = fn.conv2d(x, k, out_f32=True, stats=s0)
    yr = y.reshape(M, Cout).double()
    mref, vref = yr.mean(0), yr.var(0)                         # unbiased, as the kernel reports
    assert float(mref[0]) == pytest.approx(50.0, rel=0.02) and float(vref[0].sqrt()) < 0.2
    m0, v0 = fn.bn_moments(s0, M)                              # K = 0: plain fp32 sums
    K = m0.clone()                                             # the shift the next step would use
    s1 = torch.zeros(2 * Cout, device=DEV)
    fn.conv2d(x, k, out_f32=True, stats=s1, stats_shift=K)
    m1, v1 = fn.bn_moments(s1, M, shift=K)
    err0 = float(((v0.double() - vref) / vref).abs().max())
    err1 = float(((v1.double() - vref) / vref).abs().max())
    assert float(((m1.double() - mref) / mref).abs().max()) < 1e-5
    assert err1 < 2e-3, err1
    assert err0 > 10 * err1, (err0, err1)                      # what the shift buys


@pytest.mark.parametrize("N,H,Cin,xpad,gpad,splits", [
    (8, 13, 128, 0, 0, -1),     # stage 1 (one image per pass), default groups
    (37, 6, 128, 64, 32, 5),    # stage 2: stacked images, channel slices, partial last pass
    (50, 3, 128, 0, 0, 7),      # stage 3: many images per pass
    (16, 3, 192, 32, 0, 1),     # one group, 3 channel blocks
])
def test_wgrad3x3_small_image_path(fn, N, H, Cin, xpad, gpad, splits):
    """conv_wgrad.hip wgrad3x3_img_kernel (3x3 s1 'same', Cout 32, small maps): whole images per
    workgroup, shifted-window operands, BN+ReLU prologue; channel slices of wider buffers."""
    from idc_models_amd.ops import _native as nat
    Cout = 32
    xfull = bf(torch.randn(N, H, H, Cin + xpad, device=DEV) * 2 + 0.5)
    t = xfull[..., :Cin]
    st = torch.cat([t.sum((0, 1, 2)), (t * t).sum((0, 1, 2))])
    g, b = torch.rand(Cin, device=DEV) + 0.5, torch.randn(Cin, device=DEV) * 0.1
    gfull = bf(torch.randn(N, H, H, Cout + gpad, device=DEV))
    dy = gfull[..., :Cout]
    cnt = N * H * H
    bn = fn.BN(stats=st, gamma=g, beta=b, count=cnt, eps=1e-3, act=1)
    out = torch.zeros((3, 3, Cin, Cout), dtype=torch.float32, device=DEV)
    xb, gb = xfull.to(torch.bfloat16).contiguous(), gfull.to(torch.bfloat16).contiguous()
    a = nat.WgradArgs()
    a.x, a.N, a.H, a.W, a.Cin, a.ldx = xb.data_ptr(), N, H, H, Cin, Cin + xpad
    a.g, a.ldg = gb.data_ptr(), Cout + gpad
    a.Ho, a.Wo, a.Cout = H, H, Cout
    a.KH, a.KW, a.SH, a.SW, a.PT, a.PL = 3, 3, 1, 1, 1, 1
    a.pro = bn.args()
    a.dw, a.scale = out.data_ptr(), 1.0
    nat.require().wgrad(nat.raw(a), splits, 0, nat.stream_handle())
    act = bf(bn_ref(t, st, g, b, cnt, 1e-3, 1))
    ref = torch.nn.grad.conv2d_weight(act.permute(0, 3, 1, 2), (Cout, Cin, 3, 3), dy.permute(0, 3, 1, 2),
                                      padding=1).permute(2, 3, 1, 0)
    assert relerr(out, ref) < 1e-2


@pytest.mark.parametrize("big", ["TILE_BIG64", "TILE_BIG128", "TILE_BIG128D", "TILE_BIG256"])
@pytest.mark.parametrize("N,H,Cin,Cout", [(8, 25, 64, 256), (32, 12, 256, 256), (128, 6, 512, 512), (9, 25, 128, 384),
                                          (3, 50, 64, 64)])
def test_conv_big_tile_fwd_and_dgrad(fn, big, N, H, Cin, Cout):
    """conv_big.hip (256 x {128, 256} tiles, global_load_lds staging, source-side swizzle): the
    VGG forward (bias + ReLU epilogue) and data gradient (ReLU mask from the saved input, bias
    gradient of the producer) against fp32 PyTorch; M tails (N*H*W not a multiple of 256), image
    padding rows and Cout tails (384 with 256-wide tiles)."""
    from idc_models_amd.ops import _native as nat
    t = getattr(nat.load(), big)
    x = bf(torch.relu(torch.randn(N, H, H, Cin, device=DEV)))
    w = bf(torch.randn(3, 3, Cin, Cout, device=DEV) * (2.0 / (9 * Cin)) ** 0.5)
    bias = torch.randn(Cout, device=DEV) * 0.1
    y = fn.conv2d(x.to(torch.bfloat16), w, pads=(1, 1), bias=bias, act=1, tile=t)
    ref = ref_conv(x, w, 1, (1, 1, 1, 1), bias, act=1)
    assert relerr(y.float(), ref) < 1e-2
    # data gradient through this conv into its ReLU input x (the previous conv's output)
    dy = bf(torch.randn(N, H, H, Cout, device=DEV))
    gsum = torch.zeros(Cin, device=DEV)
    dz = fn.conv2d_dgrad(dy.to(torch.bfloat16), w, (H, H), pads=(1, 1), mx=x.to(torch.bfloat16),
                         mbn=fn.BN(act=1), gsum=gsum, tile=t)
    dA = torch.nn.grad.conv2d_input((N, Cin, H, H), w.permute(3, 2, 0, 1), dy.permute(0, 3, 1, 2),
                                    padding=1).permute(0, 2, 3, 1)
    dZ = dA * (x > 0).float()
    assert relerr(dz.float(), dZ) < 1e-2
    assert relerr(gsum, dZ.sum((0, 1, 2))) < 1e-2


@pytest.mark.parametrize("big,ks", [("TILE_BIG128", 3), ("TILE_BIG256", 2), ("TILE_BIG128", 8), ("TILE_BIG128D", 4),
                                    ("TILE_BIG128D", 1)])
def test_conv_big_tile_split_k(fn, big, ks):
    """conv_big.hip in-launch split-K (VGG block 5: M = 2304, K = 4608): partial tiles in the
    slab, modulo tickets, the last arriver runs the epilogue; twice in a row (tickets carry over)."""
    from idc_models_amd.ops import _native as nat
    t = getattr(nat.load(), big)
    N, H, Cin, Cout = 256, 3, 512, 512
    x = bf(torch.relu(torch.randn(N, H, H, Cin, device=DEV)))
    w = bf(torch.randn(3, 3, Cin, Cout, device=DEV) * (2.0 / (9 * Cin)) ** 0.5)
    bias = torch.randn(Cout, device=DEV) * 0.1
    ref = ref_conv(x, w, 1, (1, 1, 1, 1), bias, act=1)
    for _ in range(2):
        y = fn.conv2d(x.to(torch.bfloat16), w, pads=(1, 1), bias=bias, act=1, tile=t, ksplit=ks)
        assert relerr(y.float(), ref) < 1e-2
    dy = bf(torch.randn(N, H, H, Cout, device=DEV))
    gsum = torch.zeros(Cin, device=DEV)
    dz = fn.conv2d_dgrad(dy.to(torch.bfloat16), w, (H, H), pads=(1, 1), mx=x.to(torch.bfloat16),
                         mbn=fn.BN(act=1), gsum=gsum, tile=t, ksplit=ks)
    dA = torch.nn.grad.conv2d_input((N, Cin, H, H), w.permute(3, 2, 0, 1), dy.permute(0, 3, 1, 2),
                                    padding=1).permute(0, 2, 3, 1)
    dZ = dA * (x > 0).float()
    assert relerr(dz.float(), dZ) < 1e-2
    assert relerr(gsum, dZ.sum((0, 1, 2))) < 1e-2


@pytest.mark.parametrize("N,H,C", [(4, 50, 64), (3, 25, 128), (2, 13, 256), (5, 6, 512)])
def test_maxpool_bwd_scatter_form(fn, N, H, C):
    """nn_kernels.hip pool_bwd_scatter_kernel (2x2 s2 max pool, no epilogue: the VGG16 pools): each
    pooled element lands on the window position its argmax names, everything else is zero,
    including the row / column floor pooling drops (odd H); the forward matches torch."""
    x = bf(torch.randn(N, H, H, C, device=DEV))
    p, am = fn.pool2d(x.to(torch.bfloat16), 2, 2, is_max=True)
    ref = F.max_pool2d(x.permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1)
    assert torch.equal(p.float(), ref)
    Ho = H // 2
    dy = bf(torch.randn(N, Ho, Ho, C, device=DEV))
    dx = fn.pool2d_bwd(dy.to(torch.bfloat16), (N, H, H, C), 2, 2, is_max=True, argmax=am)
    a = am.view(N, Ho, Ho, C).long()
    exp = torch.zeros(N, H, H, C, device=DEV)
    for dh in range(2):
        for dw in range(2):
            exp[:, dh:2 * Ho:2, dw:2 * Ho:2, :] = torch.where(a == dh * 2 + dw, dy, torch.zeros_like(dy))
    assert torch.equal(dx.float(), exp)


@pytest.mark.parametrize("H", [12, 13])
def test_avgpool_bwd_scatter_bn_epilogue_f32(fn, H):
    """The DenseNet transition pool backward through the scatter form: 2x2 average pool, BN+ReLU
    backward per input pixel (mask, sum dZ, sum dZ*xhat) and the fp32 gamma*rstd*dZ output; odd H
    leaves a dropped row / column that must come out zero."""
    N, C = 4, 256
    x = bf(torch.randn(N, H, H, C, device=DEV) * 2 + 0.3)
    st = torch.cat([x.sum((0, 1, 2)), (x * x).sum((0, 1, 2))])
    g, b = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.1
    cnt = N * H * H
    bn = fn.BN(stats=st, gamma=g, beta=b, count=cnt, eps=1e-3, act=1)
    Ho = H // 2
    dp = bf(torch.randn(N, Ho, Ho, C, device=DEV))
    gsum = torch.zeros(C, device=DEV)
    gsumx = torch.zeros(C, device=DEV)
    out = fn.pool2d_bwd(dp.to(torch.bfloat16), (N, H, H, C), 2, 2, is_max=False, x=x.to(torch.bfloat16),
                        bn=bn, gsum=gsum, gsumx=gsumx, out_f32=True)
    mean = st[:C] / cnt
    var = st[C:] / cnt - mean ** 2
    rstd = torch.rsqrt(var + 1e-3)
    xhat = (x - mean) * rstd
    z = xhat * g + b
    up = torch.zeros(N, H, H, C, device=DEV)
    for dh in range(2):
        for dw in range(2):
            up[:, dh:2 * Ho:2, dw:2 * Ho:2, :] = dp / 4
    dZ = up * (z > 0).float()
    assert relerr(out, g * rstd * dZ) < 1e-2
    if H % 2:
        assert out[:, -1].abs().max().item() == 0 and out[:, :, -1].abs().max().item() == 0
    assert relerr(gsum, dZ.sum((0, 1, 2))) < 1e-2
    assert relerr(gsumx, (dZ * xhat).sum((0, 1, 2))) < 2e-2


@pytest.mark.parametrize("N,H,Cin,Cout,k,s,pads", [
    (2, 25, 64, 128, 3, 1, (1, 1)),     # VGG block 2 conv 1: K = 576 (a partial 256-row k tile)
    (4, 12, 128, 256, 3, 1, (1, 1)),    # block 3
    (8, 3, 512, 512, 3, 1, (1, 1)),     # block 5: 72 pixels, most of each step past the slice
    (2, 13, 64, 128, 3, 2, (1, 1)),     # strided
    (3, 10, 128, 128, 1, 1, (0, 0)),    # 1x1
])
def test_wgrad_big_tiles(fn, N, H, Cin, Cout, k, s, pads):
    """Every large-tile weight-gradient variant (wgrad_big.hip: LDS-DMA operands, transposed LDS
    reads, 32x32x16 MFMA, atomics straight from the accumulators) against fp32 PyTorch, at the
    default and at explicit pixel splits."""
    ext = fn.nat.require()
    x = bf(torch.randn(N, H, H, Cin, device=DEV))
    Ho = (H + 2 * pads[0] - k) // s + 1
    dy = bf(torch.randn(N, Ho, Ho, Cout, device=DEV))
    ref = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2), (Cout, Cin, k, k), dy.permute(0, 3, 1, 2),
                                      stride=s, padding=pads[0]).permute(2, 3, 1, 0)
    xb, dyb = x.to(torch.bfloat16), dy.to(torch.bfloat16)
    ran = 0
    for v in range(1, ext.wgrad_num_variants()):
        if not fn.wgrad_big_applies(xb, dyb, (k, k), (s, s), pads, v):
            assert Cout % 256, (v, Cout)  # only the 256-column variants may decline (Cout 128)
            continue
        for splits in (-1, 1, 3):
            dw = fn.conv2d_wgrad(xb, dyb, (k, k), stride=(s, s), pads=pads, splits=splits, variant=v)
            torch.cuda.synchronize()
            assert relerr(dw, ref) < 1e-2, (v, splits, relerr(dw, ref))
        ran += 1
    assert ran >= 4


def test_wgrad_big_deterministic_partials(fn):
    """Deterministic mode of the large-tile kernel: per-slice partials stored (no atomics), summed
    in slice order — bitwise reproducible, and equal to the fp32 reference."""
    N, H, Cin, Cout = 4, 12, 128, 256
    x = bf(torch.randn(N, H, H, Cin, device=DEV)).to(torch.bfloat16)
    dy = bf(torch.randn(N, H, H, Cout, device=DEV)).to(torch.bfloat16)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (Cout, Cin, 3, 3),
                                      dy.float().permute(0, 3, 1, 2), padding=1).permute(2, 3, 1, 0)
    outs = []
    for _ in range(2):
        part = torch.zeros(3 * 9 * Cin * Cout, device=DEV)
        outs.append(fn.conv2d_wgrad(x, dy, (3, 3), pads=(1, 1), splits=3, variant=2, part=part))
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    assert relerr(outs[0], ref) < 1e-2


def _bn_pro(fn, t, seed):
    g_ = torch.Generator(device=DEV).manual_seed(seed)
    C = t.shape[-1]
    st = torch.cat([t.sum((0, 1, 2)), (t * t).sum((0, 1, 2))])
    gam = torch.rand(C, device=DEV, generator=g_) + 0.5
    bet = torch.randn(C, device=DEV, generator=g_) * 0.1
    cnt = t.shape[0] * t.shape[1] * t.shape[2]
    return fn.BN(stats=st, gamma=gam, beta=bet, count=cnt, eps=1e-3, act=1), (st, gam, bet, cnt)


@pytest.mark.parametrize("kind,N,H", [("1x1", 32, 3), ("1x1", 16, 6), ("3x3", 64, 3), ("3x3", 16, 6),
                                      ("c32", 64, 1)])
def test_wgrad_batch_matches_single_launches(fn, kind, N, H):
    """OP_WGRAD_BATCH (conv_wgrad.h WgBatchEntry): members of mixed Cin in one launch give the
    per-layer launches' dW (fp32 atomic order only) and the fp32 reference (bf16 operands).
    Shapes: DenseNet late-stage 1x1 bottleneck wgrads (Cout 128, BN prologue), the direct 3x3
    growth-conv wgrads on 3x3 / 6x6 maps, and the centre-tap 128 -> 32 wgrads of 1x1 maps."""
    torch.manual_seed(11)
    members, refs, singles = [], [], []
    cins = (256, 288, 544, 992) if kind == "1x1" else (128, 128, 128)
    for j, cin in enumerate(cins):
        cout = 128 if kind == "1x1" else 32
        k = 3 if kind == "3x3" else 1
        x = bf(torch.randn(N, H, H, cin, device=DEV) * (1 + 0.1 * j) + 0.2 * j)
        dy = bf(torch.randn(N, H, H, cout, device=DEV))
        pro, (st, gam, bet, cnt) = _bn_pro(fn, x, 100 + j)
        pads = (1, 1) if k == 3 else (0, 0)
        mb = dict(x=x.to(torch.bfloat16), dy=dy.to(torch.bfloat16), kernel_shape=(k, k), pads=pads, pro=pro)
        members.append(mb)
        singles.append(fn.conv2d_wgrad(mb["x"], mb["dy"], (k, k), pads=pads, pro=pro))
        a = bf(bn_ref(x, st, gam, bet, cnt, 1e-3, 1))
        refs.append(torch.nn.grad.conv2d_weight(a.permute(0, 3, 1, 2), (cout, cin, k, k), dy.permute(0, 3, 1, 2),
                                                padding=pads[0]).permute(2, 3, 1, 0))
    outs = fn.conv2d_wgrad_batch(members)
    for o, s1, r in zip(outs, singles, refs):
        assert relerr(o, s1) < 1e-5
        assert relerr(o, r) < 1.5e-2


@pytest.mark.parametrize("N,H,c0,L,grid,ks", [(4, 3, 64, 3, 256, 1), (6, 1, 96, 4, 7, 1), (3, 5, 32, 2, 1, 1),
                                             (8, 6, 64, 3, 64, 1), (2, 1, 1120, 3, 256, 1), (5, 2, 256, 4, 256, 1),
                                             (256, 3, 256, 24, 256, 1),
                                             # split K of the older channels (helpers + finalizer)
                                             (2, 1, 1120, 3, 256, 8), (4, 3, 64, 3, 256, 3), (6, 1, 96, 4, 7, 4),
                                             (3, 5, 32, 2, 1, 2), (256, 1, 512, 16, 256, 8),
                                             (256, 3, 256, 24, 256, 2),
                                             # row-resident launch (ks = -1 / -2: dense_rows.hip
                                             # with 1 / 2 row blocks per workgroup)
                                             (4, 3, 64, 3, 256, -2), (6, 1, 96, 4, 7, -1),
                                             (3, 5, 32, 2, 1, -2), (5, 2, 256, 4, 256, -2),
                                             (2, 1, 1120, 3, 256, -1), (256, 3, 256, 24, 256, -2),
                                             (256, 3, 256, 24, 256, -1), (256, 1, 512, 16, 256, -2),
                                             (256, 1, 512, 16, 256, -1),
                                             # ks 0: the per-image training launch of large maps
                                             (256, 13, 64, 6, 256, 0), (256, 6, 128, 12, 256, 0),
                                             (5, 13, 64, 6, 256, 0), (301, 6, 128, 4, 256, 0)])
def test_dense_stage_persistent_matches_reference(fn, N, H, c0, L, grid, ks, monkeypatch):
    """The persistent dense-stage launch (work queue + per-phase completion counters, 1x1 partial
    sums over the finished channels accumulated before the newest slice is waited for, slotted
    in-launch statistics) vs a PyTorch fp32 reference of the same dense layers:
    BN1(shifted batch stats)->ReLU->1x1(128) stored bf16 with its shifted statistics,
    BN2->ReLU->3x3(32) (centre tap on 1x1 maps) into the stage buffer slice with its statistics.
    grid 7 / 1: far fewer workgroups than tiles (the queue must still drain: every wait depends only
    on earlier tickets).  c0 1120: DenseNet-201-wide inputs (cin > 1024, several 256-channel
    staging chunks); 2x2 maps: DenseNet-201 @ 32x32's stage 3; (256, 3, 256, 24): DenseNet-121's
    stage 3 at the bench batch exactly (M = 2,304, 24 layers, cin 256 -> 992, lookahead order);
    (256, 1, 512, 16): its stage 4.  ks > 1: each 1x1 tile's older channels split over ks work
    items whose fp32 partials the tile's finalizer adds (grid 1 / 7: helpers queued before their
    finalizer, so the queue drains with any number of workgroups).  ks < 0: the row-resident
    launch with -ks row blocks (16 rows each) of whole images per workgroup.  ks 0: the per-image
    training launch (dense_infer.hip dense_img_fwd, rows 2) at DenseNet-121's stage-1 / stage-2
    bench shapes (13x13 / 6x6, 256 images: 256 workgroups), a small batch, and 301 images (two per
    workgroup, a short last group)."""
    ipg = -(-N // 256)
    if ks < 0:
        monkeypatch.setenv("IDC_DS_ROWS_RB", str(-ks))
        ext = fn.nat.require()
        ok, rb, ipg, g = ext.dense_rows_geometry(N, H, H, c0 + 32 * L, c0 + 32 * (L - 1))
        assert ok and rb == -ks, (ok, rb, ipg, g)
    W = H
    ld = c0 + 32 * L
    g = torch.Generator(device="cpu").manual_seed(N * 100 + H)
    buf = torch.zeros(N, H, W, ld)
    buf[..., :c0] = torch.randn(N, H, W, c0, generator=g) * 1.5 + 0.3
    buf = buf.to(torch.bfloat16).to(DEV)  # the stage buffer is bf16 (kernel operand)
    K = torch.randn(ld, generator=g).to(DEV) * 0.2  # statistics shifts
    x0 = buf[..., :c0].float().reshape(-1, c0)
    sst = torch.zeros(2 * ld, device=DEV)
    sst[:c0] = (x0 - K[:c0]).sum(0)
    sst[ld:ld + c0] = ((x0 - K[:c0]) ** 2).sum(0)
    k2 = 1 if H == 1 else 3
    lays, refs = [], []
    for i in range(L):
        cin = c0 + 32 * i
        w1 = bf(torch.randn(1, 1, cin, 128, generator=g) * (2.0 / cin) ** 0.5).to(DEV)
        w2 = bf(torch.randn(3, 3, 128, 32, generator=g) * (2.0 / 1152) ** 0.5).to(DEV)
        w2l = fn.weight_fwd_layout(w2[1:2, 1:2] if k2 == 1 else w2, 128)
        d = dict(w1=fn.weight_fwd_layout(w1, cin), w2=w2l,
                 g1=(torch.rand(cin, generator=g) + 0.5).to(DEV), b1=(torch.randn(cin, generator=g) * 0.1).to(DEV),
                 g2=(torch.rand(128, generator=g) + 0.5).to(DEV), b2=(torch.randn(128, generator=g) * 0.1).to(DEV),
                 t=torch.zeros(N, H, W, 128, dtype=torch.bfloat16, device=DEV),
                 tstats=torch.zeros(256, device=DEV), tshift=(torch.randn(128, generator=g) * 0.1).to(DEV),
                 eps1=1.001e-5, eps2=1.001e-5, cin=cin)
        lays.append(d)
        refs.append((w1, w2))
    # reference, layer by layer (operands rounded to bf16 where the kernel rounds them)
    rbuf = buf.float().clone()
    rst = sst.clone()
    rts, rtst = [], []
    cnt = N * H * W
    for i, d in enumerate(lays):
        cin = d["cin"]
        w1, w2 = refs[i]
        mean = K[:cin] + rst[:cin] / cnt
        var = (rst[ld:ld + cin] / cnt - (rst[:cin] / cnt) ** 2).clamp_min(0)
        a1 = bf(torch.relu((rbuf[..., :cin] - mean) * torch.rsqrt(var + 1.001e-5) * d["g1"] + d["b1"]))
        t = bf(ref_conv(a1, w1, 1, (0, 0, 0, 0)))
        tk = (t - d["tshift"]).reshape(-1, 128)
        tst = torch.cat([tk.sum(0), (tk * tk).sum(0)])
        m2 = d["tshift"] + tst[:128] / cnt
        v2 = (tst[128:] / cnt - (tst[:128] / cnt) ** 2).clamp_min(0)
        a2 = bf(torch.relu((t - m2) * torch.rsqrt(v2 + 1.001e-5) * d["g2"] + d["b2"]))
        y = bf(ref_conv(a2, w2, 1, (1, 1, 1, 1)))
        rbuf[..., cin:cin + 32] = y
        yk = (y - K[cin:cin + 32]).reshape(-1, 32)
        rst[cin:cin + 32] = yk.sum(0)
        rst[ld + cin:ld + cin + 32] = (yk * yk).sum(0)
        rts.append(t)
        rtst.append(tst)
    sync, err, _ = fn.dense_stage(buf, sst, lays, sshift=K, grid=grid, k2=k2, ksplit=max(ks, 1),
                                  rows=2 if ks == 0 else int(ks < 0))
    M = N * H * W
    nA, nB = -(-M // 32) * 2, -(-M // 32)
    assert int(err[0].item()) == 0 and int(sync[-1].item()) == 0
    cnt = sync[1:1 + 16 * L].reshape(L, 2, 8).sum(-1)  # per layer: A_l, B_l sharded counters
    if ks <= 0:  # barrier arrivals: every workgroup at both barriers of every layer but the last
        G = -(-N // ipg)
        assert cnt[:-1, 0].tolist() == [G] * (L - 1) and cnt[:-1, 1].tolist() == [G] * (L - 1), sync.tolist()
    else:
        assert cnt[:, 0].tolist() == [nA] * L and cnt[:, 1].tolist() == [nB] * L, sync.tolist()
    errs = {}
    for i, d in enumerate(lays):
        errs[f"t{i}"] = relerr(d["t"].float(), rts[i])
        errs[f"tstats{i}"] = relerr(d["tstats"], rtst[i])
    errs["buf"] = relerr(buf.float(), rbuf)
    errs["sst"] = relerr(sst, rst)
    assert all(v < 2e-2 for v in errs.values()), errs


@pytest.mark.parametrize("ks", [1, 4])
def test_dense_stage_timeout_is_counted(fn, ks):
    """A wait that gives up (poll bound forced to 1) fails the launch: every workgroup leaves and
    the persistent error counter records it (dense_stage.hip wait_count)."""
    N, H, c0, L = 64, 3, 64, 4
    ld = c0 + 32 * L
    buf = (torch.randn(N, H, H, ld, device=DEV) * 0.5).to(torch.bfloat16)
    buf[..., c0:] = 0
    x0 = buf[..., :c0].float().reshape(-1, c0)
    sst = torch.zeros(2 * ld, device=DEV)
    sst[:c0], sst[ld:ld + c0] = x0.sum(0), (x0 * x0).sum(0)
    lays = []
    for i in range(L):
        cin = c0 + 32 * i
        lays.append(dict(w1=torch.randn(128 * cin, device=DEV).to(torch.bfloat16) * 0.05,
                         w2=torch.randn(32 * 9 * 128, device=DEV).to(torch.bfloat16) * 0.03,
                         g1=torch.ones(cin, device=DEV), b1=torch.zeros(cin, device=DEV),
                         g2=torch.ones(128, device=DEV), b2=torch.zeros(128, device=DEV),
                         t=torch.zeros(N, H, H, 128, dtype=torch.bfloat16, device=DEV),
                         tstats=torch.zeros(256, device=DEV), tshift=None, eps1=1e-5, eps2=1e-5, cin=cin))
    sync, err, _ = fn.dense_stage(buf, sst, lays, grid=256, k2=3, max_polls=1, ksplit=ks)
    assert int(sync[-1].item()) == 1 and int(err[0].item()) == 1, (sync.tolist(), err.tolist())
    # the same launch with the default bound completes
    sst2 = torch.zeros(2 * ld, device=DEV)
    sst2[:c0], sst2[ld:ld + c0] = x0.sum(0), (x0 * x0).sum(0)
    for d in lays:
        d["tstats"].zero_()
    sync, err, _ = fn.dense_stage(buf, sst2, lays, grid=256, k2=3, ksplit=ks)
    assert int(sync[-1].item()) == 0 and int(err[0].item()) == 0


def _bn_train(x, g, b, eps):
    mean = x.mean((0, 1, 2))
    var = x.var((0, 1, 2), unbiased=False)
    return (x - mean) * torch.rsqrt(var + eps) * g + b


@pytest.mark.parametrize("N,H,c0,L,grid,rows", [(16, 3, 64, 3, 256, 0), (64, 1, 96, 4, 256, 0), (8, 3, 128, 2, 5, 0),
                                               (6, 2, 256, 3, 64, 0), (4, 1, 1120, 2, 256, 0),
                                               (64, 3, 256, 4, 256, 0), (256, 3, 256, 24, 256, 0),
                                               (256, 1, 512, 16, 256, 0), (256, 6, 128, 12, 256, 0),
                                               # row-resident launch (dense_rows_bwd.hip)
                                               (16, 3, 64, 3, 256, 1), (64, 1, 96, 4, 256, 1),
                                               (8, 3, 128, 2, 5, 1), (6, 2, 256, 3, 64, 1),
                                               (20, 3, 256, 4, 256, 1), (256, 3, 256, 24, 256, 1),
                                               (256, 1, 512, 16, 256, 1)])
def test_dense_stage_bwd_matches_autograd(fn, N, H, c0, L, grid, rows):
    """The persistent dense-stage BACKWARD launch (dense_stage_bwd.hip: 3x3 dgrad, dT, newest-slice
    and older-channel 1x1 dgrads, every BatchNorm backward through the summed pending affines,
    d gamma / d beta) vs fp32 autograd of the same dense layers, forward values rounded to bf16
    where the kernels store them (straight-through).  Upstream: a consumer BatchNorm + ReLU over the
    whole stage buffer with a random output gradient (the transition / final BatchNorm of
    lower_densenet).  grid 5: far fewer workgroups than tickets (queue order must still drain);
    c0 1120: DenseNet-201-wide inputs; 1x1 maps: centre-tap 3x3; (256, 3, 256, 24) and
    (256, 1, 512, 16): DenseNet-121's stages 3 and 4 at the bench batch exactly, (256, 6, 128, 12)
    its stage 2.  rows 1: the
    row-resident launch (whole images per workgroup, the concat gradient held in LDS)."""
    if rows:
        ok, ipg, g = fn.nat.require().dense_rows_bwd_geometry(N, H, H, c0 + 32 * L, L)
        assert ok, (N, H, c0, L)
    torch.manual_seed(N * 1000 + c0 + L)
    W = H
    ld = c0 + 32 * L
    k2 = 1 if H == 1 else 3
    eps = 1.001e-5

    def rnd(v):  # round the value to bf16, gradient straight through
        return v + (bf(v) - v).detach()

    x0 = bf(torch.randn(N, H, W, c0, device=DEV) * 1.5 + 0.3).requires_grad_(True)
    params, lays = [], []
    for i in range(L):
        cin = c0 + 32 * i
        p = dict(W1=bf(torch.randn(1, 1, cin, 128, device=DEV) * (2.0 / cin) ** 0.5),
                 W2=bf(torch.randn(3, 3, 128, 32, device=DEV) * (2.0 / 1152) ** 0.5),
                 g1=(torch.rand(cin, device=DEV) + 0.5).requires_grad_(True),
                 b1=(torch.randn(cin, device=DEV) * 0.1).requires_grad_(True),
                 g2=(torch.rand(128, device=DEV) + 0.5).requires_grad_(True),
                 b2=(torch.randn(128, device=DEV) * 0.1).requires_grad_(True))
        params.append(p)
    gc = torch.rand(ld, device=DEV) + 0.5
    bc = torch.randn(ld, device=DEV) * 0.1
    G = torch.randn(N, H, W, ld, device=DEV)
    parts, ts, ys = [x0], [], []
    for i, p in enumerate(params):
        x = torch.cat(parts, -1)
        a1 = rnd(torch.relu(_bn_train(x, p["g1"], p["b1"], eps)))
        t = rnd(ref_conv(a1, p["W1"], 1, (0, 0, 0, 0)))
        t.retain_grad()
        a2 = rnd(torch.relu(_bn_train(t, p["g2"], p["b2"], eps)))
        y = rnd(ref_conv(a2, p["W2"], 1, (1, 1, 1, 1)))
        y.retain_grad()
        ts.append(t)
        ys.append(y)
        parts.append(y)
    xb = torch.cat(parts, -1)
    zc = _bn_train(xb, gc, bc, eps)
    (torch.relu(zc) * G).sum().backward()
    # kernel inputs from the same forward values
    cnt = N * H * W
    buf = xb.detach().to(torch.bfloat16).contiguous()
    xf = buf.float().reshape(-1, ld)
    K = torch.randn(ld, device=DEV) * 0.2
    sst = torch.cat([(xf - K).sum(0), ((xf - K) ** 2).sum(0)])
    mean_c, var_c = xf.mean(0), xf.var(0, unbiased=False)
    rstd_c = torch.rsqrt(var_c + eps)
    zcv = ((xf - mean_c) * rstd_c * gc + bc)
    dZc = G.reshape(-1, ld) * (zcv > 0).float()
    xh_c = (xf - mean_c) * rstd_c
    dbuf = (dZc * gc * rstd_c).reshape(N, H, W, ld).contiguous()
    gsum, gsumx = dZc.sum(0), (dZc * xh_c).sum(0)
    pend = fn.bwd_aff(buf, fn.BN(stats=sst, gamma=gc, beta=bc, count=cnt, eps=eps, shift=K, ld=ld),
                      gsum=gsum, gsumx=gsumx, unit_alpha=True)
    for i, p in enumerate(params):
        cin = c0 + 32 * i
        t = ts[i].detach().to(torch.bfloat16).contiguous()
        tsh = torch.randn(128, device=DEV) * 0.1
        tk = t.float().reshape(-1, 128) - tsh
        w2 = p["W2"][1:2, 1:2] if k2 == 1 else p["W2"]
        lays.append(dict(w1d=fn.weight_dgrad_layout(p["W1"]), w2d=fn.weight_dgrad_layout(w2),
                         g1=p["g1"].detach(), b1=p["b1"].detach(), g2=p["g2"].detach(), b2=p["b2"].detach(),
                         t=t, tstats=torch.cat([tk.sum(0), (tk * tk).sum(0)]), tshift=tsh, eps1=eps, eps2=eps,
                         cin=cin, dO16=torch.zeros(N, H, W, 32, dtype=torch.bfloat16, device=DEV),
                         dt=torch.zeros(N, H, W, 128, dtype=torch.bfloat16, device=DEV),
                         dbeta1=torch.zeros(cin, device=DEV), dgamma1=torch.zeros(cin, device=DEV),
                         dbeta2=torch.zeros(128, device=DEV), dgamma2=torch.zeros(128, device=DEV)))
    dx16, sync, err = fn.dense_stage_bwd(buf, sst, lays, dbuf, pend, sshift=K, grid=grid, k2=k2, rows=rows)
    assert int(err[0].item()) == 0 and int(sync[-1].item()) == 0, sync.tolist()
    errs = {"dx": relerr(dx16, x0.grad)}
    for i, (p, d) in enumerate(zip(params, lays)):
        errs[f"dO{i}"] = relerr(d["dO16"], ys[i].grad)
        errs[f"dt{i}"] = relerr(d["dt"], ts[i].grad)
        errs[f"db2_{i}"] = relerr(d["dbeta2"], p["b2"].grad)
        errs[f"dg2_{i}"] = relerr(d["dgamma2"], p["g2"].grad)
        errs[f"db1_{i}"] = relerr(d["dbeta1"], p["b1"].grad)
        errs[f"dg1_{i}"] = relerr(d["dgamma1"], p["g1"].grad)
    assert all(v < 3e-2 for v in errs.values()), errs


def test_secagg_segment_absmax_matches_torch():
    """Native per-segment max |x| (secure-aggregation ranges): segments from 1 element to more
    than a block's chunk, several vectors merged, exactly the torch reduction."""
    from idc_models_amd.fed.secagg import segment_absmax, segment_ends
    g = torch.Generator().manual_seed(4)
    sizes = [1, 7, 64, 3000, 1, 200000, 17, 4096, 5, 123457]
    vecs = [torch.randn(sum(sizes), generator=g) * (i + 1) for i in range(3)]
    se = segment_ends(sizes)
    got = segment_absmax([v.to(DEV) for v in vecs], se, len(sizes), DEV).cpu()
    ref = segment_absmax(vecs, se, len(sizes), "cpu")
    assert torch.equal(got, ref), (got, ref)


@pytest.mark.parametrize("N,H,c0,L,grid,ks", [(4, 3, 64, 3, 256, 1), (6, 1, 96, 4, 7, 1), (2, 1, 1120, 3, 256, 1),
                                             (6, 1, 96, 4, 7, 3), (2, 1, 1120, 3, 256, 8),
                                             (4, 3, 64, 3, 256, -2), (6, 1, 96, 4, 7, -1),
                                             (2, 1, 1120, 3, 256, -1)])
def test_dense_stage_inference_mode_matches_reference(fn, N, H, c0, L, grid, ks, monkeypatch):
    """Inference-mode dense stage (frozen base / evaluation): BN1 and BN2 from each layer's own
    moving statistics, nothing produced but t and the stage-buffer slices, vs a PyTorch reference."""
    W = H
    ld = c0 + 32 * L
    g = torch.Generator(device="cpu").manual_seed(N * 7 + H)
    buf = torch.zeros(N, H, W, ld)
    buf[..., :c0] = torch.randn(N, H, W, c0, generator=g) * 1.5 + 0.3
    buf = buf.to(torch.bfloat16).to(DEV)
    k2 = 1 if H == 1 else 3
    lays, refs = [], []
    for i in range(L):
        cin = c0 + 32 * i
        w1 = bf(torch.randn(1, 1, cin, 128, generator=g) * (2.0 / cin) ** 0.5).to(DEV)
        w2 = bf(torch.randn(3, 3, 128, 32, generator=g) * (2.0 / 1152) ** 0.5).to(DEV)
        w2l = fn.weight_fwd_layout(w2[1:2, 1:2] if k2 == 1 else w2, 128)
        d = dict(w1=fn.weight_fwd_layout(w1, cin), w2=w2l,
                 g1=(torch.rand(cin, generator=g) + 0.5).to(DEV), b1=(torch.randn(cin, generator=g) * 0.1).to(DEV),
                 g2=(torch.rand(128, generator=g) + 0.5).to(DEV), b2=(torch.randn(128, generator=g) * 0.1).to(DEV),
                 mm1=(torch.randn(cin, generator=g) * 0.3).to(DEV), mv1=(torch.rand(cin, generator=g) * 2 + 0.2).to(DEV),
                 mm2=(torch.randn(128, generator=g) * 0.3).to(DEV), mv2=(torch.rand(128, generator=g) * 2 + 0.2).to(DEV),
                 t=torch.zeros(N, H, W, 128, dtype=torch.bfloat16, device=DEV),
                 tstats=torch.zeros(256, device=DEV), tshift=None, eps1=1e-3, eps2=1.001e-5, cin=cin)
        lays.append(d)
        refs.append((w1, w2))
    rbuf = buf.float().clone()
    rts = []
    for i, d in enumerate(lays):
        cin = d["cin"]
        w1, w2 = refs[i]
        a1 = bf(torch.relu((rbuf[..., :cin] - d["mm1"]) * torch.rsqrt(d["mv1"] + d["eps1"]) * d["g1"] + d["b1"]))
        t = bf(ref_conv(a1, w1, 1, (0, 0, 0, 0)))
        a2 = bf(torch.relu((t - d["mm2"]) * torch.rsqrt(d["mv2"] + d["eps2"]) * d["g2"] + d["b2"]))
        rbuf[..., cin:cin + 32] = bf(ref_conv(a2, w2, 1, (1, 1, 1, 1)))
        rts.append(t)
    if ks < 0:
        monkeypatch.setenv("IDC_DS_ROWS_RB", str(-ks))
    sync, err, _ = fn.dense_stage(buf, None, lays, grid=grid, k2=k2, infer=True, ksplit=max(ks, 1),
                                  rows=int(ks < 0))
    assert int(err[0].item()) == 0 and int(sync[-1].item()) == 0
    errs = {f"t{i}": relerr(d["t"].float(), rts[i]) for i, d in enumerate(lays)}
    errs["buf"] = relerr(buf.float(), rbuf)
    assert all(v < 2e-2 for v in errs.values()), errs
    assert all(float(d["tstats"].abs().sum()) == 0.0 for d in lays)  # no statistics produced


@pytest.mark.parametrize("N,H,c0,L,ipg", [(3, 13, 64, 6, 1), (5, 6, 128, 12, 2), (4, 6, 128, 12, 1),
                                          (2, 13, 64, 3, 1), (3, 5, 96, 4, 3), (5, 3, 256, 24, 1),
                                          (3, 3, 256, 24, 2), (37, 1, 512, 16, 16), (5, 1, 512, 16, 1)])
def test_dense_infer_matches_reference(fn, N, H, c0, L, ipg):
    """A whole dense block in inference mode as ONE launch (dense_infer.hip: whole images per
    workgroup, the concat buffer and the zero-bordered z2 grid in LDS) vs a PyTorch reference of
    the same layers on moving statistics, intermediates rounded to bf16 where the kernel stores
    them.  DenseNet-121 stage 1 (13x13, c0 64, 6 layers), stage 2 (6x6, c0 128, 12 layers), stage 3
    (3x3, c0 256, 24 layers: the 1x1 K in two register chunks) and stage 4 (1x1, c0 512, 16 layers:
    the 3x3's centre slice only; 37 images = a short last group of 16) with one and several images
    per workgroup, and an odd map."""
    W = H
    ld = c0 + 32 * L
    g = torch.Generator(device="cpu").manual_seed(N * 11 + H + L)
    buf = torch.zeros(N, H, W, ld)
    buf[..., :c0] = torch.randn(N, H, W, c0, generator=g) * 1.5 + 0.3
    buf = buf.to(torch.bfloat16).to(DEV)
    lays, refs = [], []
    for i in range(L):
        cin = c0 + 32 * i
        w1 = bf(torch.randn(1, 1, cin, 128, generator=g) * (2.0 / cin) ** 0.5).to(DEV)
        w2 = bf(torch.randn(3, 3, 128, 32, generator=g) * (2.0 / 1152) ** 0.5).to(DEV)
        w2k = w2[1:2, 1:2] if H == 1 else w2  # 1x1 maps: the kernel reads the centre slice
        d = dict(w1=fn.weight_fwd_layout(w1, cin), w2=fn.weight_fwd_layout(w2k, 128),
                 g1=(torch.rand(cin, generator=g) + 0.5).to(DEV), b1=(torch.randn(cin, generator=g) * 0.1).to(DEV),
                 g2=(torch.rand(128, generator=g) + 0.5).to(DEV), b2=(torch.randn(128, generator=g) * 0.1).to(DEV),
                 mm1=(torch.randn(cin, generator=g) * 0.3).to(DEV), mv1=(torch.rand(cin, generator=g) * 2 + 0.2).to(DEV),
                 mm2=(torch.randn(128, generator=g) * 0.3).to(DEV), mv2=(torch.rand(128, generator=g) * 2 + 0.2).to(DEV),
                 eps1=1e-3, eps2=1.001e-5, cin=cin)
        lays.append(d)
        refs.append((w1, w2))
    rbuf = buf.float().clone()
    for i, d in enumerate(lays):
        cin = d["cin"]
        w1, w2 = refs[i]
        a1 = bf(torch.relu((rbuf[..., :cin] - d["mm1"]) * torch.rsqrt(d["mv1"] + d["eps1"]) * d["g1"] + d["b1"]))
        t = ref_conv(a1, w1, 1, (0, 0, 0, 0))
        a2 = bf(torch.relu((t - d["mm2"]) * torch.rsqrt(d["mv2"] + d["eps2"]) * d["g2"] + d["b2"]))
        rbuf[..., cin:cin + 32] = bf(ref_conv(a2, w2, 1, (1, 1, 1, 1)))
    fn.dense_infer(buf, lays, ipg=ipg)
    assert torch.equal(buf[..., :c0].float(), rbuf[..., :c0])  # the block input is left alone
    errs = [relerr(buf[..., c0 + 32 * i:c0 + 32 * (i + 1)].float(), rbuf[..., c0 + 32 * i:c0 + 32 * (i + 1)])
            for i in range(L)]
    assert max(errs) < 2e-2, errs
    assert torch.isfinite(buf.float()).all()


@pytest.mark.parametrize("N,H", [(5, 13), (7, 6), (9, 3), (3, 8), (64, 6)])
def test_conv_img_forward_matches_reference(fn, N, H):
    """Image-resident 3x3 kernel (conv_img.hip, tile TILE_IMG), DenseNet growth conv 128 -> 32:
    pending BN + ReLU staged once per element, shifted output statistics; vs fp32 reference and
    vs the implicit-GEMM tiles."""
    ext = fn.nat.require()
    Cin, Cout = 128, 32
    x = bf(torch.randn(N, H, H, Cin, device=DEV) * 1.5 + 0.4)
    st = torch.cat([x.sum((0, 1, 2)), (x * x).sum((0, 1, 2))])
    gamma = torch.rand(Cin, device=DEV) + 0.5
    beta = torch.randn(Cin, device=DEV) * 0.1
    w = bf(torch.randn(3, 3, Cin, Cout, device=DEV) * 0.05)
    cnt = N * H * H
    shift = torch.randn(Cout, device=DEV) * 0.1
    bn = fn.BN(stats=st, gamma=gamma, beta=beta, count=cnt, eps=1.001e-5, act=1)
    outs = {}
    tk = torch.zeros(17 + 16 * 2 * Cout, dtype=torch.int32, device=DEV)  # slot copies + arrival counter
    for tile, tickets in ((ext.TILE_IMG, None), ("slots", tk), (-1, None)):
        so = torch.zeros(2 * Cout, device=DEV)
        y = fn.conv2d(x.to(torch.bfloat16), w, pads=(1, 1), pro=bn, stats=so, stats_shift=shift,
                      tile=ext.TILE_IMG if tile == "slots" else tile, tickets=tickets)
        outs[tile] = (y.float(), so)
    torch.cuda.synchronize()
    assert int(tk.abs().sum()) == 0  # the last arrival re-zeroed the slots and the counter
    assert torch.equal(outs["slots"][0], outs[ext.TILE_IMG][0])
    assert relerr(outs["slots"][1], outs[ext.TILE_IMG][1]) < 1e-5
    a = bn_ref(x, st, gamma, beta, cnt, 1.001e-5, 1)
    ref = ref_conv(bf(a), w, 1, (1, 1, 1, 1))
    y, so = outs[ext.TILE_IMG]
    assert relerr(y, ref) < 1e-2
    assert relerr(y, outs[-1][0]) < 5e-3
    d = y - shift
    assert relerr(so[:Cout], d.sum((0, 1, 2))) < 1e-3
    assert relerr(so[Cout:], (d * d).sum((0, 1, 2))) < 1e-3


@pytest.mark.parametrize("N,H", [(5, 13), (7, 6), (9, 3), (48, 6)])
def test_conv_img_dgrad_matches_reference(fn, N, H):
    """Image-resident 3x3 data gradient 32 -> 128 as DenseNet's dgrad cv2 issues it: fp32 concat-
    gradient operand holding A*dZ with the pending B*x + C added while staging (plus the fold and
    the bf16 staged copy), epilogue dZ2 = dA * relu'(bn2(t)) reduced into gsum / gsumx."""
    ext = fn.nat.require()
    C, cin = 32, 128
    k = _bn_case(N, H, C, seed=3)
    v = (k["dZ"] * k["A"]).contiguous()
    w = bf(torch.randn(3, 3, cin, C, device=DEV) * 0.1)
    x16 = k["x"].to(torch.bfloat16)
    t = bf(torch.randn(N, H, H, cin, device=DEV) * 1.2 + 0.2)
    st2 = torch.cat([t.sum((0, 1, 2)), (t * t).sum((0, 1, 2))])
    g2 = torch.rand(cin, device=DEV) + 0.5
    b2 = torch.randn(cin, device=DEV) * 0.1
    cnt = N * H * H
    res = {}
    tk = torch.zeros(17 + 16 * 2 * cin, dtype=torch.int32, device=DEV)
    for tile in (ext.TILE_IMG, "slots", -1):
        db, dg = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        aff = fn.bwd_aff(x16, k["bn"], k["gsum"], k["gsumx"], unit_alpha=True, fold=(db, dg))
        staged = torch.zeros(N, H, H, C, dtype=torch.bfloat16, device=DEV)
        gsum, gsumx = torch.zeros(cin, device=DEV), torch.zeros(cin, device=DEV)
        dz = fn.conv2d_dgrad(v, w, (H, H), pads=(1, 1), bpro=aff, aout=staged, mx=t.to(torch.bfloat16),
                             mbn=fn.BN(stats=st2, gamma=g2, beta=b2, count=cnt, eps=1e-3, act=1),
                             gsum=gsum, gsumx=gsumx, tile=ext.TILE_IMG if tile == "slots" else tile,
                             tickets=tk if tile == "slots" else None)
        torch.cuda.synchronize()
        res[tile] = (dz.float(), staged.float(), gsum, gsumx, db, dg)
    assert int(tk.abs().sum()) == 0
    assert torch.equal(res["slots"][0], res[ext.TILE_IMG][0])
    assert relerr(res["slots"][2], res[ext.TILE_IMG][2]) < 1e-5 and relerr(res["slots"][3], res[ext.TILE_IMG][3]) < 1e-5
    dA = torch.nn.grad.conv2d_input((N, cin, H, H), w.permute(3, 2, 0, 1), bf(k["dX"]).permute(0, 3, 1, 2),
                                    padding=1).permute(0, 2, 3, 1)
    mean = st2[:cin] / cnt
    var = st2[cin:] / cnt - mean ** 2
    xhat = (t - mean) * torch.rsqrt(var + 1e-3)
    dZ2 = dA * ((xhat * g2 + b2) > 0).float()
    dz, staged, gsum, gsumx, db, dg = res[ext.TILE_IMG]
    assert relerr(dz, dZ2) < 2e-2
    assert relerr(dz, res[-1][0]) < 5e-3
    assert relerr(staged, k["dX"]) < 1e-2 and torch.equal(staged, res[-1][1])
    assert relerr(gsum, dZ2.sum((0, 1, 2))) < 2e-2
    assert relerr(gsumx, (dZ2 * xhat).sum((0, 1, 2))) < 2e-2
    assert torch.equal(db, k["gsum"]) and torch.equal(dg, k["gsumx"])


@pytest.mark.parametrize("N,H,Cin,Cexp,Cout,S,residual,xin,ipg,cs", [
    (8, 25, 32, None, 16, 1, False, "bnrelu6", 1, None),   # block 0: no expand, stem BN + ReLU6 pending
    (4, 25, 16, 96, 24, 2, False, "id", 1, None),          # block 1: stride 2 from the 25x25 map
    (6, 13, 24, 144, 24, 1, True, "bnres", 1, None),       # block 2: pending project BN + shortcut input
    (6, 13, 24, 144, 24, 1, True, "bnres", 1, 64),         # same, 3 slices (last one 16 channels)
    (9, 7, 32, 192, 32, 1, True, "id", 2, None),           # 7x7 identity block, last group one image
    (20, 4, 96, 576, 160, 2, False, "id", 16, None),       # block 13: stride 2 to 2x2, 16 images a group
    (33, 2, 160, 960, 320, 1, False, "id", 16, None),      # block 16: 20 output tiles per group, 15 slices
    (17, 2, 160, 960, 160, 1, True, "bnres", 16, 128),     # block 14, 8 slices (last one 64 channels)
    (17, 2, 160, 960, 160, 1, True, "bnres", 16, 96)])     # block 14, 10 slices
def test_mb_infer_matches_reference(fn, N, H, Cin, Cexp, Cout, S, residual, xin, ipg, cs):
    """One MobileNetV2 block in inference mode as ONE launch (mb_infer.hip) vs an fp32 PyTorch
    reference of the same block: x_eff = xbn(x) (+ res), expand 1x1 + BN + ReLU6, depthwise 3x3
    (Keras correct_pad on stride 2) + BN + ReLU6, project 1x1 + BN (+ x_eff).  Intermediates are
    rounded to bf16 where the kernel stores them (x_eff, the expanded and depthwise slices).  ``cs``:
    expanded channels per workgroup (several slices: partials summed by the group's last arriver;
    None: the launch default); the second launch of the same op must agree bit for bit (tickets
    count modulo the slices, the partials sum in slice order)."""
    from idc_models_amd.models.layers import correct_pad
    torch.manual_seed(N * 100 + Cin + H)
    W = H
    if S == 1:
        pt, pb, pl, pr = 1, 1, 1, 1
    else:
        (pt, pb), (pl, pr) = correct_pad(H, W, 3)
    Ho, Wo = (H + pt + pb - 3) // S + 1, (W + pl + pr - 3) // S + 1
    ce = Cexp or Cin

    def bnp(C, act):
        return fn.BN(gamma=torch.rand(C, device=DEV) + 0.5, beta=torch.randn(C, device=DEV) * 0.1,
                     mean=torch.randn(C, device=DEV) * 0.2, var=torch.rand(C, device=DEV) + 0.5, eps=1e-3,
                     mode=2, act=act)

    def bn_apply(v, bn):
        z = (v - bn.mean) * torch.rsqrt(bn.var + bn.eps) * bn.gamma + bn.beta
        return z.clamp(0, 6) if bn.act == 2 else z

    x = bf(torch.randn(N, H, W, Cin, device=DEV))
    res = bf(torch.randn(N, H, W, Cin, device=DEV)) if xin == "bnres" else None
    xbn = bnp(Cin, 2 if xin == "bnrelu6" else 0) if xin != "id" else None
    we = torch.randn(1, 1, Cin, ce, device=DEV) * (2.0 / Cin) ** 0.5 if Cexp else None
    ebn = bnp(ce, 2) if Cexp else None
    wd = torch.randn(3, 3, ce, 1, device=DEV) * (2.0 / 9) ** 0.5
    dbn = bnp(ce, 2)
    wp = torch.randn(1, 1, ce, Cout, device=DEV) * (1.0 / ce) ** 0.5
    pbn = bnp(Cout, 0)
    y = fn.mb_infer(x.to(torch.bfloat16), we, ebn, wd, dbn, wp, pbn, stride=S, pads=(pt, pl), out_hw=(Ho, Wo),
                    xbn=xbn, res=res.to(torch.bfloat16) if res is not None else None, residual=residual, ipg=ipg,
                    cs=cs)
    # fp32 reference
    xe = bn_apply(x, xbn) if xbn is not None else x
    if res is not None:
        xe = xe + res
    xe = bf(xe)
    e = bf(bn_apply(ref_conv(xe, bf(we), 1, (0, 0, 0, 0)), ebn)) if Cexp else xe
    ec = F.pad(e.permute(0, 3, 1, 2), (pl, pr, pt, pb))
    d = F.conv2d(ec, wd.permute(2, 3, 0, 1), stride=S, groups=ce).permute(0, 2, 3, 1)
    d = bf(bn_apply(d, dbn))
    ref = bn_apply(ref_conv(d, bf(wp), 1, (0, 0, 0, 0)), pbn)
    if residual:
        ref = ref + xe
    assert y.shape == ref.shape
    assert torch.isfinite(y.float()).all()
    assert relerr(y, ref) < 1.5e-2, relerr(y, ref)
    y2 = fn.mb_infer(x.to(torch.bfloat16), we, ebn, wd, dbn, wp, pbn, stride=S, pads=(pt, pl), out_hw=(Ho, Wo),
                     xbn=xbn, res=res.to(torch.bfloat16) if res is not None else None, residual=residual,
                     ipg=ipg, cs=cs)
    assert torch.equal(y, y2)
