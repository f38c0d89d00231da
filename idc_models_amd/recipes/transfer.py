"""Two-phase transfer learning recipe (``dist_model_tf_{vgg,mobile,dense}.py main()``).

Flow: data -> strategy -> base (frozen) + GAP + Dense -> compile(RMSprop(lr)) ->
evaluate(val, steps=20) -> Timer("Pre-training with N devices"): fit(initial_epochs) ->
unfreeze, refreeze ``layers[:fine_tune_at]`` -> recompile(RMSprop(lr/10)) ->
Timer("Fine-tuning with N devices"): fit(total_epochs, initial_epoch=history.epoch[-1]) ->
plot ``{path}/logs/plot_dev{N}.png``.

Per-script defaults: vgg lr 1e-3 / fine_tune_at 15 / IDC balanced; mobile lr 1e-4 /
100 / IDC patient layout; dense lr 1e-4 / 150 / CIFAR-10 with DenseNet-201 @32, 10 classes, CCE,
per-replica batch 256.  ``initial_epoch=history.epoch[-1]`` reproduces quirk Q6 (epoch 9 rerun).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Optional, Tuple

import torch

from ..data import (ArrayDataset, cifar10_dataset, idc_dataset, prepare_for_training, split,
                    synthetic_dataset)
from ..engine import Model, RMSprop
from ..models import build_model
from ..utils.plot import log as plot_log
from ..utils.timer import Timer


@dataclass
class TransferConfig:
    arch: str = "vgg16"
    path: str = "."
    dataset: str = "idc"               # idc | idc_patient | cifar10 | synthetic
    input_shape: Tuple[int, int, int] = (50, 50, 3)
    num_classes: int = 1
    batch_size: int = 32               # GLOBAL batch (vgg/mobile convention)
    per_replica_batch: Optional[int] = None  # dense convention: global = per_replica * N
    base_learning_rate: float = 1e-3
    initial_epochs: int = 10
    fine_tune_epochs: int = 10
    fine_tune_at: int = 15
    validation_steps: int = 20
    strategy: str = "mirrored"         # mirrored | central | one
    synthetic_size: int = 4096
    seed: int = 0
    backend: str = "auto"
    keras_compat_accuracy: bool = False
    plot: bool = True
    ylim: Optional[tuple] = None
    steps_per_epoch: Optional[int] = None
    verbose: int = 0


PRESETS = {
    "vgg": dict(arch="vgg16", dataset="idc", base_learning_rate=1e-3, fine_tune_at=15),
    "mobile": dict(arch="mobilenetv2", dataset="idc_patient", base_learning_rate=1e-4, fine_tune_at=100,
                   ylim=((0.8, 1.0), (0.0, 1.0))),
    "dense": dict(arch="densenet201", dataset="cifar10", input_shape=(32, 32, 3), num_classes=10,
                  per_replica_batch=256, base_learning_rate=1e-4, fine_tune_at=150,
                  ylim=((0.8, 1.0), (0.0, 1.0))),
}


def fine_tune_at_for(arch: str) -> int:
    """The reference's phase-2 cut for a backbone: VGG16 15 (``dist_model_tf_vgg.py:146``, block5
    trains), MobileNetV2 100 (``dist_model_tf_mobile.py:146``), DenseNets 150
    (``dist_model_tf_dense.py:158``)."""
    for pre in PRESETS.values():
        if pre["arch"] == arch:
            return int(pre["fine_tune_at"])
    if arch.startswith("densenet"):
        return int(PRESETS["dense"]["fine_tune_at"])
    raise KeyError(f"no reference fine-tuning cut for {arch!r}")


def make_strategy(kind: str):
    from ..parallel import CentralStorageStrategy, MirroredStrategy, OneDeviceStrategy
    if kind == "central":
        return CentralStorageStrategy()
    if kind == "one":
        return OneDeviceStrategy()
    return MirroredStrategy()


def load_data(cfg: TransferConfig):
    if cfg.dataset == "cifar10":
        root = os.path.join(cfg.path, "data", "cifar-10-batches-bin")
        if os.path.isdir(root):
            tr, te = cifar10_dataset(root, True), cifar10_dataset(root, False)
        else:
            tr = synthetic_dataset(cfg.synthetic_size, cfg.input_shape, 10, cfg.seed)
            te = synthetic_dataset(max(cfg.synthetic_size // 5, 64), cfg.input_shape, 10, cfg.seed + 1)
        return tr, te, te
    if cfg.dataset == "synthetic":
        ds = synthetic_dataset(cfg.synthetic_size, cfg.input_shape, max(cfg.num_classes, 2), cfg.seed)
    else:
        layout = "patient" if cfg.dataset == "idc_patient" else "balanced"
        ds = idc_dataset(cfg.path, layout, cfg.input_shape[0], cfg.seed)
    return tuple(split(ds, (0.8, 0.1, 0.1)))


def run_transfer_learning(cfg: TransferConfig, printer=print):
    strategy = make_strategy(cfg.strategy)
    n = strategy.num_replicas_in_sync
    gbatch = cfg.per_replica_batch * n if cfg.per_replica_batch else cfg.batch_size
    train_ds, val_ds, test_ds = load_data(cfg)
    repeat = 2 if cfg.dataset == "cifar10" else 1  # dist_model_tf_dense.py:122-123 .repeat(2)
    train = train_ds.batch(gbatch, True, 1000, False, cfg.seed, repeat)
    val = val_ds.batch(gbatch, True, 1000, False, cfg.seed + 1, repeat)
    loss = "categorical_crossentropy" if cfg.num_classes > 1 else "binary_crossentropy"
    with strategy.scope():
        net = build_model(cfg.arch, cfg.input_shape, cfg.num_classes, seed=cfg.seed)
        net.base.trainable = False
        model = Model(net, strategy)
        model.compile(RMSprop(cfg.base_learning_rate), loss, ["accuracy"],
                      keras_compat_accuracy=cfg.keras_compat_accuracy, backend=cfg.backend)
    loss0, acc0 = model.evaluate(val, steps=cfg.validation_steps)
    if strategy.is_chief:
        printer(f"initial loss: {loss0:.4f}, initial accuracy: {acc0:.4f}")
    with Timer(f"Pre-training with {n} devices", printer if strategy.is_chief else None):
        history = model.fit(train, epochs=cfg.initial_epochs, validation_data=val,
                            validation_steps=cfg.validation_steps, steps_per_epoch=cfg.steps_per_epoch,
                            verbose=cfg.verbose)
    net.base.trainable = True
    if strategy.is_chief:
        printer("Number of layers in the base model: ", len(net.base.layers))
    with strategy.scope():
        for layer in net.base.layers[:cfg.fine_tune_at]:
            layer.trainable = False
        model.compile(RMSprop(cfg.base_learning_rate / 10), loss, ["accuracy"],
                      keras_compat_accuracy=cfg.keras_compat_accuracy, backend=cfg.backend)
    total = cfg.initial_epochs + cfg.fine_tune_epochs
    with Timer(f"Fine-tuning with {n} devices", printer if strategy.is_chief else None):
        history_fine = model.fit(train, epochs=total, initial_epoch=history.epoch[-1],
                                 validation_data=val, validation_steps=cfg.validation_steps,
                                 steps_per_epoch=cfg.steps_per_epoch, verbose=cfg.verbose)
    if cfg.plot and strategy.is_chief:
        plot_log(cfg.path, history, history_fine, n, cfg.initial_epochs, cfg.ylim, printer=printer)
    return model, history, history_fine
