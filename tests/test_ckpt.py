"""Checkpoint compatibility: Keras-layout HDF5 and full-state resume."""
import numpy as np
import pytest
import torch

from idc_models_amd.ckpt import load_checkpoint, load_weights, read_weights, save_checkpoint, save_weights
from idc_models_amd.engine import Model, RMSprop
from idc_models_amd.models import build_backbone, build_model
from idc_models_amd.parallel import OneDeviceStrategy

CPU = OneDeviceStrategy("cpu")


def test_keras_layout(tmp_path):
    m = build_model("vgg16", seed=0)
    p = str(tmp_path / "w.h5")
    save_weights(m, p)
    from idc_models_amd import _idc_h5
    attrs, dsets = _idc_h5.read(p)
    assert attrs[("/", "layer_names")] == [b"vgg16", b"global_average_pooling2d", b"dense"]
    assert attrs[("/", "backend")] == [b"tensorflow"]
    wn = attrs[("/vgg16", "weight_names")]
    assert wn[0] == b"block1_conv1/kernel:0" and wn[1] == b"block1_conv1/bias:0"
    assert dsets["/vgg16/block1_conv1/kernel:0"].shape == (3, 3, 3, 64)  # HWIO
    assert attrs[("/dense", "weight_names")] == [b"dense/kernel:0", b"dense/bias:0"]
    assert dsets["/dense/dense/kernel:0"].shape == (512, 1)


def test_roundtrip_by_name_across_freeze_states(tmp_path):
    a = build_model("mobilenetv2", seed=1)
    p = str(tmp_path / "m.h5")
    save_weights(a, p)
    b = build_model("mobilenetv2", seed=2)
    # different freeze state => different Keras weight ORDER; load must match by name
    b.base.trainable = True
    for l in b.base.layers[:100]:
        l.trainable = False
    load_weights(b, p)
    for (n, x), y in zip(a.named_parameters(), b.parameters()):
        assert torch.equal(x, y), n
    assert torch.equal(a.base.get_layer("Conv_1_bn").moving_variance,
                       b.base.get_layer("Conv_1_bn").moving_variance)


def test_bare_backbone_file_loads_into_classifier(tmp_path):
    """Keras *_notop.h5 layout: flat layer groups of the backbone only."""
    base = build_backbone("densenet121")
    p = str(tmp_path / "notop.h5")
    save_weights(base, p)
    data = read_weights(p)
    assert "conv1/conv/conv1/conv/kernel:0" in data
    m = build_model("densenet121", seed=5)
    missing = load_weights(m, p)
    assert torch.equal(m.base.get_layer("conv5_block16_2_conv").kernel,
                       base.get_layer("conv5_block16_2_conv").kernel)
    assert any("dense" in n for n in missing)  # head not in a notop file


def test_shape_mismatch_raises(tmp_path):
    p = str(tmp_path / "t.h5")
    save_weights(build_model("densenet121"), p)
    with pytest.raises(ValueError):
        load_weights(build_model("densenet121", num_outputs=10), p)


def test_full_state_checkpoint_resume(tmp_path):
    from idc_models_amd.data import prepare_for_training, synthetic_dataset
    ds = synthetic_dataset(32, (10, 10, 3), seed=0)
    m = Model(build_model("tinycnn", seed=0), CPU)
    m.compile(RMSprop(1e-3), "binary_crossentropy", ["accuracy"])
    m.fit(prepare_for_training(ds, 16), epochs=1, verbose=0)
    p = str(tmp_path / "state.pt")
    m.save_checkpoint(p, {"epoch": 3, "round": 7})
    m2 = Model(build_model("tinycnn", seed=4), CPU)
    m2.compile(RMSprop(1e-3), "binary_crossentropy", ["accuracy"])
    info = m2.load_checkpoint(p)
    assert info["epoch"] == 3 and info["round"] == 7
    assert torch.equal(m.optimizer.ms, m2.optimizer.ms)
    for a, b in zip(m.get_weights(), m2.get_weights()):
        assert np.array_equal(a, b)
