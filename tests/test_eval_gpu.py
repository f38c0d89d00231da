"""The inference path: the fused ``eval_step`` program -- inference-mode
BatchNorm on the MOVING statistics, no backward -- against the eager fp32 model on identical
weights, for every backbone at the benchmark batch.  The moving statistics, gamma and beta are
randomised first (a fresh model's mean 0 / variance 1 would hide a wrong statistic), and the
comparison is judged at the bf16 floor (eager under bf16 autocast vs fp32).  Reference: the
reference evaluates before and after every fit (``dist_model_tf_vgg.py:134``,
``secure_fed_model.py:81-82,153``)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _randomise_bn(net, seed):
    g = torch.Generator().manual_seed(seed)
    n = 0
    with torch.no_grad():
        for l in net.base.layers:
            if getattr(l, "keras_class", "") != "BatchNormalization":
                continue
            C = l.moving_mean.numel()
            l.moving_mean.copy_((torch.randn(C, generator=g) * 0.3).to(l.moving_mean.device))
            l.moving_variance.copy_((0.5 + torch.rand(C, generator=g)).to(l.moving_variance.device))
            l.gamma.copy_((0.8 + 0.4 * torch.rand(C, generator=g)).to(l.gamma.device))
            l.beta.copy_((torch.randn(C, generator=g) * 0.1).to(l.beta.device))
            n += 1
    return n


@pytest.mark.parametrize("arch,B,shape,fuse_all", [("densenet121", 256, None, False), ("vgg16", 256, None, False),
                                                   ("mobilenetv2", 256, None, False), ("mobilenetv2", 256, None, True),
                                                   ("densenet201", 256, (32, 32, 3), False)])
def test_fused_eval_matches_eager_inference(monkeypatch, arch, B, shape, fuse_all):
    """``fuse_all``: every MobileNetV2 block as one mb_infer launch (IDC_MB_INFER_MAX_CEXP lifted;
    the default fuses blocks 0-13 only)."""
    if fuse_all:
        monkeypatch.setenv("IDC_MB_INFER_MAX_CEXP", "4096")
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model
    net = build_model(arch, shape, num_outputs=1, seed=21)
    nbn = _randomise_bn(net, 5) if arch != "vgg16" else 0
    ref = copy.deepcopy(net).to(DEV).eval()
    ref16 = copy.deepcopy(ref)
    m = Model(net, device=DEV)
    m.compile(RMSprop(1e-4), "binary_crossentropy", ["accuracy"], backend="fused")
    assert type(m.impl).__name__ == "FusedStep"
    H, W, C = net.input_shape
    g = torch.Generator().manual_seed(7)
    x = torch.randint(0, 256, (B, H, W, C), generator=g, dtype=torch.uint8)
    y = torch.randint(0, 2, (B,), generator=g)
    loss, logits = m.impl.eval_step(x, y)
    torch.cuda.synchronize()
    with torch.no_grad():
        lr = ref(x.to(DEV).float() / 255.0).float().reshape(-1)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            l16 = ref16(x.to(DEV).float() / 255.0).float().reshape(-1)
    lf = logits.reshape(-1).float()
    dev_fused = float((lf - lr).abs().max())
    dev_auto = float((l16 - lr).abs().max())
    spread = float(lr.std())
    assert dev_fused <= 2 * dev_auto + 0.02 * spread + 1e-3, (arch, nbn, dev_fused, dev_auto, spread)
    # the inference program must not have touched the moving statistics
    for a, b in zip(m.net.non_trainable_weights, ref.non_trainable_weights):
        assert torch.equal(a.to(DEV), b.to(DEV))
    bce = torch.nn.functional.binary_cross_entropy_with_logits(lr, y.to(DEV).float())
    assert abs(float(loss) - float(bce)) <= 2 * abs(float(torch.nn.functional.binary_cross_entropy_with_logits(
        l16, y.to(DEV).float())) - float(bce)) + 0.01


def test_mobilenetv2_fused_fit_auc_matches_eager_fit_auc():
    """tools/check_eval.py as a test, small scale: MobileNetV2 trained by the fused program, then
    evaluated (exact AUC, inference BatchNorm) by both backends on the same weights: the two AUCs
    agree within 0.02."""
    from idc_models_amd.data import synthetic_dataset
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model
    net = build_model("mobilenetv2", None, num_outputs=1, seed=0)
    # Keras' MobileNetV2 BatchNorm momentum 0.999 needs ~4600 updates before the moving statistics
    # leave their init; after this test's 48 the inference output would be a constant (AUC = noise
    # of near-tied logits in both backends).  0.9 converges within the fit, so the comparison
    # judges a model that actually ranks the held-out set.
    for l in net.base.layers:
        if getattr(l, "keras_class", "") == "BatchNormalization":
            l.momentum = 0.9
    m = Model(net, device=DEV)
    m.compile(RMSprop(1e-3), "binary_crossentropy", ["accuracy", "auc"], backend="fused")
    tr = synthetic_dataset(64 * 12, net.input_shape, 2, seed=11, signal=8.0, label_noise=0.1)
    te = synthetic_dataset(512, net.input_shape, 2, seed=12, signal=8.0, label_noise=0.1)
    m.fit(tr.batch(64, True, 1000, True, seed=1), epochs=4, verbose=0)
    fused = m.evaluate(te.batch(64, False), return_dict=True)
    ref = Model(copy.deepcopy(m.net), device=DEV)
    ref.compile(RMSprop(1e-3), "binary_crossentropy", ["accuracy", "auc"], backend="eager")
    eager = ref.evaluate(te.batch(64, False), return_dict=True)
    assert abs(fused["auc"] - eager["auc"]) <= 0.02, (fused, eager)
    assert abs(fused["loss"] - eager["loss"]) <= 0.05 * max(1.0, eager["loss"]), (fused, eager)
