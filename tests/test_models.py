"""Model zoo parity with Keras Applications — CPU."""
import math

import numpy as np
import pytest
import torch

from idc_models_amd.models import build_backbone, build_model, clone_model
from idc_models_amd.models.layers import BatchNormalization, correct_pad


@pytest.mark.parametrize("arch,shape,total,nontrain,nlayers,out_hw,out_c", [
    ("vgg16", (50, 50, 3), 14714688, 0, 19, (1, 1), 512),
    ("mobilenetv2", (50, 50, 3), 2257984, 34112, 155, (2, 2), 1280),
    ("densenet121", (50, 50, 3), 7037504, 83648, 427, (1, 1), 1024),
    ("densenet201", (32, 32, 3), 18321984, 229056, 707, (1, 1), 1920),
])
def test_backbone_param_counts_match_keras(arch, shape, total, nontrain, nlayers, out_hw, out_c):
    b = build_backbone(arch, shape)
    assert sum(t.numel() for t in b.weight_tensors()) == total
    assert sum(t.numel() for t in b.non_trainable_weights) == nontrain
    assert len(b.layers) == nlayers
    assert b.output_hw == out_hw and b.output_channels == out_c


@pytest.mark.parametrize("arch,idx,name", [
    ("vgg16", 15, "block5_conv1"),
    ("mobilenetv2", 100, "block_11_expand_BN"),
    ("densenet121", 150, "conv4_block2_1_conv"),
    ("densenet201", 150, "conv4_block2_1_conv"),
])
def test_fine_tune_at_layer_names(arch, idx, name):
    assert build_backbone(arch).layers[idx].name == name


def test_phase2_trainable_counts():
    """SURVEY §2.4.2/§2.4.3 phase-2 trainable parameter counts."""
    m = build_model("mobilenetv2")
    m.base.trainable = True
    for l in m.base.layers[:100]:
        l.trainable = False
    assert sum(p.numel() for p in m.trainable_weights) == 1863873
    d = build_model("densenet121")
    for l in d.base.layers[:150]:
        l.trainable = False
    assert sum(p.numel() for p in d.trainable_weights) == 5454273
    d201 = build_model("densenet201", (32, 32, 3), num_outputs=10)
    for l in d201.base.layers[:150]:
        l.trainable = False
    assert sum(p.numel() for p in d201.trainable_weights) == 16611530
    v = build_model("vgg16")
    for l in v.base.layers[:15]:
        l.trainable = False
    assert sum(p.numel() for p in v.trainable_weights) == 7079937


def test_full_train_counts_for_benchmarks():
    assert sum(p.numel() for p in build_model("densenet121").trainable_weights) == 6954881
    assert sum(p.numel() for p in build_model("vgg16").trainable_weights) == 14715201
    assert sum(p.numel() for p in build_model("mobilenetv2").trainable_weights) == 2225153


def test_tiny_cnn_shapes_match_reference():
    t = build_model("tinycnn")
    assert t.count_params() == 1937
    assert [tuple(w.shape) for w in t.weights] == [(3, 3, 3, 32), (32,), (128, 8), (8,), (8, 1), (1,)]
    assert t(torch.rand(4, 10, 10, 3)).shape == (4, 1)


@pytest.mark.parametrize("arch", ["vgg16", "mobilenetv2", "densenet121"])
def test_forward_shapes(arch):
    m = build_model(arch)
    m.eval()
    with torch.no_grad():
        assert m(torch.rand(2, 50, 50, 3)).shape == (2, 1)


def test_correct_pad_asymmetric():
    assert correct_pad(50, 50, 3) == ((0, 1), (0, 1))
    assert correct_pad(25, 25, 3) == ((1, 1), (1, 1))


def test_mobilenet_spatial_chain():
    b = build_backbone("mobilenetv2")
    x = torch.rand(1, 50, 50, 3)
    b.eval()
    shapes = []
    saved = []
    h = x
    with torch.no_grad():
        for kind, layer in b.graph:
            if kind == "seq":
                h = layer(h)
                if layer.keras_class == "DepthwiseConv2D":
                    shapes.append(h.shape[1])
            elif kind == "save":
                saved.append(h)
            elif kind == "add":
                h = layer(saved.pop(), h)
            else:
                saved.pop()
    assert sorted(set(shapes), reverse=True) == [25, 13, 7, 4, 2]


def test_glorot_init_and_bn_defaults():
    b = build_backbone("vgg16")
    k = b.get_layer("block3_conv1").kernel
    limit = math.sqrt(6.0 / (9 * 128 + 9 * 256))
    assert k.abs().max().item() <= limit + 1e-6
    assert abs(k.std().item() - limit / math.sqrt(3)) < 0.1 * limit
    assert b.get_layer("block3_conv1").bias.abs().max().item() == 0.0
    d = build_backbone("densenet121")
    bn = d.get_layer("conv1/bn")
    assert bn.epsilon == pytest.approx(1.001e-5) and bn.momentum == pytest.approx(0.99)
    assert torch.all(bn.gamma == 1) and torch.all(bn.moving_variance == 1)
    mb = build_backbone("mobilenetv2").get_layer("bn_Conv1")
    assert mb.epsilon == pytest.approx(1e-3) and mb.momentum == pytest.approx(0.999)


def test_frozen_bn_uses_moving_stats_and_is_not_updated():
    bn = BatchNormalization(4, 1e-3, 0.9, "bn")
    bn.train()
    x = torch.randn(8, 3, 3, 4) * 3 + 2
    bn(x)
    assert not torch.allclose(bn.moving_mean, torch.zeros(4))
    bn.trainable = False
    mm = bn.moving_mean.clone()
    y = bn(x)
    assert torch.equal(bn.moving_mean, mm)
    ref = (x - bn.moving_mean) / torch.sqrt(bn.moving_variance + 1e-3)
    assert torch.allclose(y, ref, atol=1e-5)


def test_bn_moving_variance_is_bessel_corrected():
    bn = BatchNormalization(2, 1e-3, 0.0, "bn")  # momentum 0: moving = batch
    bn.train()
    x = torch.randn(5, 1, 1, 2)
    bn(x)
    assert torch.allclose(bn.moving_variance, x.reshape(-1, 2).var(0, unbiased=True), atol=1e-6)


def test_weights_order_trainable_then_nontrainable_and_keras_names():
    m = build_model("mobilenetv2")
    names = m.base.keras_weight_names()
    n_tr = len(m.base.trainable_weights)
    assert all(not n.endswith(("moving_mean:0", "moving_variance:0")) for n in names[:n_tr])
    assert all(n.endswith(("moving_mean:0", "moving_variance:0")) for n in names[n_tr:])
    assert names[0] == "Conv1/kernel:0"
    # freezing moves the frozen layers' weights to the non-trainable group (Keras semantics)
    m.base.trainable = False
    assert m.base.trainable_weights == []
    assert len(m.base.non_trainable_weights) == len(names)


def test_clone_model_fresh_weights_same_flags():
    m = build_model("tinycnn", seed=1)
    m.layers[0].trainable = False
    c = clone_model(m)
    assert c.layers[0].trainable is False
    assert not torch.equal(c.layers[0].kernel, m.layers[0].kernel)
