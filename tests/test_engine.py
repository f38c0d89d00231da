"""Keras-style engine on the CPU reference path."""
import numpy as np
import pytest
import torch

from idc_models_amd.data import prepare_for_training, split, synthetic_dataset
from idc_models_amd.engine import Model, ModelCheckpoint, RMSprop
from idc_models_amd.engine.arena import ParamArena
from idc_models_amd.engine.losses import BinaryCrossentropy, CategoricalCrossentropy
from idc_models_amd.engine.metrics import AUC, Accuracy, exact_auc
from idc_models_amd.models import build_model
from idc_models_amd.parallel import OneDeviceStrategy

CPU = OneDeviceStrategy("cpu")


def test_rmsprop_keras_semantics():
    p = torch.nn.Parameter(torch.tensor([1.0, -2.0, 3.0, 0.5]))
    ar = ParamArena([p], "cpu")
    opt = RMSprop(0.01)
    opt.bind(ar)
    g1 = torch.tensor([0.1, -0.2, 0.3, 0.0])
    ar.grad[:4] = g1
    opt.step(ar)
    ms = 0.1 * g1 * g1
    ref = torch.tensor([1.0, -2.0, 3.0, 0.5]) - 0.01 * g1 / (ms.sqrt() + 1e-7)
    assert torch.allclose(p.detach(), ref, atol=1e-6)
    assert opt.iterations == 1


def test_rmsprop_grad_scale_folds_world_average():
    a = torch.nn.Parameter(torch.ones(4))
    b = torch.nn.Parameter(torch.ones(4))
    ar1, ar2 = ParamArena([a], "cpu"), ParamArena([b], "cpu")
    o1, o2 = RMSprop(0.1), RMSprop(0.1)
    o1.bind(ar1)
    o2.bind(ar2)
    ar1.grad[:4] = 2.0
    ar2.grad[:4] = 1.0
    o1.step(ar1, grad_scale=0.5)
    o2.step(ar2)
    assert torch.allclose(a, b)


def test_losses():
    logits = torch.tensor([[2.0], [-1.0], [0.5]])
    y = torch.tensor([1, 0, 1])
    bce = BinaryCrossentropy()(logits, y)
    x, z = logits.reshape(-1), y.float()
    ref = (torch.clamp(x, min=0) - x * z + torch.log1p(torch.exp(-x.abs()))).mean()
    assert torch.allclose(bce, ref)
    l10 = torch.randn(4, 10)
    yi = torch.tensor([1, 3, 5, 7])
    cce = CategoricalCrossentropy()(l10, yi)  # sparse labels are one-hot encoded (quirk Q5)
    assert torch.allclose(cce, torch.nn.functional.cross_entropy(l10, yi))


def test_accuracy_thresholds_logit0_vs_keras_compat():
    logits = torch.tensor([0.2, -0.1, 0.7, 0.4])
    y = torch.tensor([1, 0, 1, 1])
    a = Accuracy()
    a.update(logits, y)
    assert a.result() == 1.0
    k = Accuracy(keras_compat=True)  # Keras thresholds logits at 0.5 (quirk Q11)
    k.update(logits, y)
    assert k.result() == 0.5


def test_exact_auc_matches_sklearn():
    from sklearn.metrics import roc_auc_score
    rng = np.random.default_rng(0)
    s = rng.normal(size=500)
    l = (rng.random(500) < 0.4).astype(int)
    s[:50] = 0.25  # ties
    assert abs(exact_auc(torch.tensor(s), torch.tensor(l)) - roc_auc_score(l, s)) < 1e-10
    m = AUC(mode="per_batch")
    m.update(torch.tensor(s[:100]), torch.tensor(l[:100]))
    m.update(torch.tensor(s[100:200]), torch.tensor(l[100:200]))
    ref = (roc_auc_score(l[:100], s[:100]) + roc_auc_score(l[100:200], s[100:200])) / 2
    assert abs(m.result() - ref) < 1e-10


def test_two_phase_recipe_epochs_and_initial_epoch_quirk():
    ds = synthetic_dataset(96, seed=2)
    tr, va, _ = split(ds)
    m = Model(build_model("mobilenetv2", seed=0), CPU)
    m.net.base.trainable = False
    m.compile(RMSprop(1e-3), "binary_crossentropy", ["accuracy"])
    h = m.fit(prepare_for_training(tr, 32), epochs=2, validation_data=prepare_for_training(va, 32),
              validation_steps=1, verbose=0)
    assert h.epoch == [0, 1]
    assert set(h.history) == {"loss", "accuracy", "val_loss", "val_accuracy"}
    m.net.base.trainable = True
    for l in m.net.base.layers[:100]:
        l.trainable = False
    m.compile(RMSprop(1e-4), "binary_crossentropy", ["accuracy"])
    h2 = m.fit(prepare_for_training(tr, 32), epochs=4, initial_epoch=h.epoch[-1], steps_per_epoch=1,
               verbose=0)
    assert h2.epoch == [1, 2, 3]  # Q6: fine-tuning re-runs the last pre-training epoch


def test_phase1_frozen_base_bn_stats_untouched_and_base_weights_fixed():
    ds = synthetic_dataset(64, seed=3)
    m = Model(build_model("mobilenetv2", seed=0), CPU)
    m.net.base.trainable = False
    bn = m.net.base.get_layer("block_3_expand_BN")
    mm = bn.moving_mean.clone()
    k = m.net.base.get_layer("Conv1").kernel.detach().clone()
    m.compile(RMSprop(1e-3), "binary_crossentropy", ["accuracy"])
    assert len(m.arena.params) == 2
    m.fit(prepare_for_training(ds, 32), epochs=1, verbose=0)
    assert torch.equal(bn.moving_mean, mm)
    assert torch.equal(m.net.base.get_layer("Conv1").kernel.detach(), k)


def test_tiny_cnn_overfits():
    torch.manual_seed(0)
    ds = synthetic_dataset(64, (10, 10, 3), seed=4, signal=60.0)
    m = Model(build_model("tinycnn", seed=0), CPU)
    m.compile(RMSprop(1e-2), "binary_crossentropy", ["accuracy", "auc"])
    h = m.fit(prepare_for_training(ds, 16), epochs=25, verbose=0)
    assert h.history["accuracy"][-1] > 0.9
    assert h.history["loss"][-1] < h.history["loss"][0]


def test_get_set_weights_roundtrip_and_evaluate_list():
    ds = synthetic_dataset(32, (10, 10, 3), seed=5)
    m = Model(build_model("tinycnn", seed=0), CPU)
    m.compile(RMSprop(1e-3), "binary_crossentropy", ["accuracy"])
    w = m.get_weights()
    assert [a.shape for a in w] == [(3, 3, 3, 32), (32,), (128, 8), (8,), (8, 1), (1,)]
    m2 = Model(build_model("tinycnn", seed=9), CPU)
    m2.compile(RMSprop(1e-3), "binary_crossentropy", ["accuracy"])
    m2.set_weights(w)
    r1 = m.evaluate(prepare_for_training(ds, 32))
    r2 = m2.evaluate(prepare_for_training(ds, 32))
    assert r1 == pytest.approx(r2)


def test_model_checkpoint_callback_writes_each_epoch(tmp_path):
    ds = synthetic_dataset(32, (10, 10, 3), seed=6)
    m = Model(build_model("tinycnn", seed=0), CPU)
    m.compile(RMSprop(1e-3), "binary_crossentropy", ["accuracy"])
    path = str(tmp_path / "pretrained" / "cp.h5")
    m.fit(prepare_for_training(ds, 16), epochs=2, callbacks=[ModelCheckpoint(path)], verbose=0)
    m2 = Model(build_model("tinycnn", seed=3), CPU)
    m2.compile(RMSprop(1e-3), "binary_crossentropy", ["accuracy"])
    m2.load_weights(path)
    for a, b in zip(m.get_weights(), m2.get_weights()):
        assert np.array_equal(a, b)


def test_reset_optimizer_in_place():
    m = Model(build_model("tinycnn", seed=0), CPU)
    m.compile(RMSprop(1e-3), "binary_crossentropy", [])
    ms = m.optimizer.ms
    ms.fill_(3.0)
    m.reset_optimizer()
    assert m.optimizer.ms is ms and float(ms.abs().max()) == 0.0


def test_skip_nonfinite_gradients():
    ds = synthetic_dataset(16, (10, 10, 3), seed=7)
    m = Model(build_model("tinycnn", seed=0), CPU)
    m.compile(RMSprop(1e-3), "binary_crossentropy", [], skip_nonfinite=True)
    w0 = [w.copy() for w in m.get_weights()]
    x, y = next(iter(prepare_for_training(ds, 16)))
    xf = x.float() / 255.0
    xf[0, 0, 0, 0] = float("nan")
    m.impl.train_step(xf, y)
    assert m.skipped_steps() == 1
    for a, b in zip(w0, m.get_weights()):
        assert np.array_equal(a, b)
    m.impl.train_step(x, y)
    assert m.skipped_steps() == 1
    assert not all(np.array_equal(a, b) for a, b in zip(w0, m.get_weights()))
