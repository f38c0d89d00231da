"""Federated recipes: ``fed_model.py main()`` (FedAvg) and ``secure_fed_model.py main()``.

FedAvg: 10 clients of 3,000 examples (8 train / 2 test), IID or non-IID ordering,
VGG16 pre-trained centrally for 10 epochs with a per-epoch ModelCheckpoint (or loaded from it),
unfreeze + refreeze ``layers[:15]``, FedAvg with client RMSprop(1e-4), federated evaluation before
and after every round; prints ``round, train acc, train loss, test acc, test loss``.
North-star variant: MobileNetV2, 8 clients one per GPU.

Secure FL: 2 clients (strided shards of the first 24,000 examples, 80/20 per
client), tiny CNN on 10x10 patches, 5 local epochs, protect ``percent`` of the tensors, client 0
evaluates on the next 6,000 examples and prints ``loss acc auc``.
North-star variant: DenseNet-121 @50x50, 8 clients, additive-mask aggregation.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional, Tuple

import torch

from ..data import (contiguous_clients, idc_dataset, prepare_for_training, shard_clients,
                    synthetic_dataset, train_test_clients)
from ..engine import Model, ModelCheckpoint, RMSprop
from ..fed import (broadcast_server_state, build_federated_averaging_process, build_federated_evaluation,
                   load_server_extra, load_server_state, save_server_state, state_with_new_model_weights)
from ..fed.secure import SecureFederatedProcess
from ..models import build_model
from ..parallel import OneDeviceStrategy, comm
from ..utils.timer import Timer


def _local_device():
    if torch.cuda.is_available():
        _, _, local = comm.env_world()
        return torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    return torch.device("cpu")


@dataclass
class FedConfig:
    path: str = "."
    rounds: int = 5
    iid: bool = True
    arch: str = "vgg16"
    input_shape: Tuple[int, int, int] = (50, 50, 3)
    num_clients: int = 10
    num_test_clients: int = 2
    dataset_size: int = 30000
    batch_size: int = 32
    base_learning_rate: float = 1e-3
    fine_tune_at: int = 15
    pretrain_epochs: int = 10
    synthetic: bool = False
    average_bn_stats: bool = False
    seed: int = 0
    backend: str = "auto"
    secure_aggregation: Optional[str] = None  # "mask": config #5 secure FedAvg
    resume: bool = True                       # continue from {path}/fed_state/state.pt if present
                                              # (refused when it was written by another config)
    concurrent_clients: int = 1               # clients a rank trains at once (own model + stream)


def _fed_data(cfg: FedConfig):
    if cfg.synthetic or not os.path.isdir(os.path.join(cfg.path, "data")):
        ds = synthetic_dataset(cfg.dataset_size, cfg.input_shape, 2, cfg.seed)
        if not cfg.iid:  # label-sorted ordering like get_data(non-iid)
            ds = ds.filter_label(1).concatenate(ds.filter_label(0))
        return ds
    return idc_dataset(cfg.path, "balanced", cfg.input_shape[0], cfg.seed, iid=cfg.iid)


def _fed_fingerprint(cfg: FedConfig, state) -> dict:
    """What a resumed run must share with the run that wrote the state."""
    shapes = ";".join("x".join(str(d) for d in t.shape) for t in state.model.trainable)
    return {"arch": cfg.arch, "num_clients": int(cfg.num_clients),
            "secure_aggregation": str(cfg.secure_aggregation), "average_bn_stats": bool(cfg.average_bn_stats),
            "trainable_shapes": shapes}


def run_fedavg(cfg: FedConfig, printer=print):
    comm.init_process_group()
    dev = _local_device()
    strategy = OneDeviceStrategy(dev)
    labeled = _fed_data(cfg)
    train_size = int(0.8 * cfg.dataset_size)
    client_size = cfg.dataset_size // cfg.num_clients
    # ---- central pre-training (fed_model.py:99-147), gated on an existing checkpoint (fix Q7)
    ckpt = os.path.join(cfg.path, "pretrained", "cp.h5")
    net = build_model(cfg.arch, cfg.input_shape, 1, seed=cfg.seed)
    net.base.trainable = False
    pre = Model(net, strategy)
    pre.compile(RMSprop(cfg.base_learning_rate), "binary_crossentropy", ["binary_accuracy"],
                backend=cfg.backend)
    if os.path.exists(ckpt):
        printer("Loading pretrained model")
        pre.load_weights(ckpt, strict=True)  # a stale checkpoint of another arch must not load silently
    elif comm.rank() == 0:
        # one central pre-training (rank 0), not one per rank: the fused kernels are not bitwise
        # reproducible, so per-rank runs would start the federation from different servers
        tr = prepare_for_training(labeled.take(train_size), cfg.batch_size, seed=cfg.seed)
        va = prepare_for_training(labeled.skip(train_size).take(cfg.dataset_size - train_size),
                                  cfg.batch_size, seed=cfg.seed + 1)
        pre.evaluate(va, steps=20)
        with Timer("Pre-training", printer):
            pre.fit(tr, epochs=cfg.pretrain_epochs, validation_data=va, validation_steps=20,
                    callbacks=[ModelCheckpoint(ckpt, save_weights_only=True, rank=0)], verbose=0)
    if comm.world_size() > 1:
        pre.impl.sync_to_module()
        for t in pre.net.weight_tensors():  # rank 0's pre-trained (or loaded) model everywhere
            comm.broadcast_(t.data, 0)
        pre.impl.sync_from_module()
    net.base.trainable = True
    for layer in net.base.layers[:cfg.fine_tune_at]:
        layer.trainable = False
    pre.compile(RMSprop(cfg.base_learning_rate), "binary_crossentropy", ["binary_accuracy"], backend=cfg.backend)
    # ---- clients (fed_model.py:178-189): client i = skip(i*CLIENT_SIZE).take(CLIENT_SIZE)
    clients = contiguous_clients(labeled, cfg.num_clients, client_size)
    train_clients, test_clients = train_test_clients(clients, cfg.num_test_clients)
    fed_train = [prepare_for_training(c, cfg.batch_size, seed=cfg.seed + i) for i, c in enumerate(train_clients)]
    fed_test = [prepare_for_training(c, cfg.batch_size, seed=cfg.seed + 100 + i) for i, c in enumerate(test_clients)]

    def model_fn():
        import copy
        m_net = copy.deepcopy(net)  # clone_model: same architecture + trainable flags
        m_net.reset_parameters()
        return Model(m_net, strategy)

    fed_avg = build_federated_averaging_process(
        model_fn, client_optimizer_fn=lambda: RMSprop(cfg.base_learning_rate / 10),
        average_bn_stats=cfg.average_bn_stats, metrics=("binary_accuracy",),
        secure_aggregation=cfg.secure_aggregation, concurrent_clients=cfg.concurrent_clients)
    evaluation = build_federated_evaluation(model_fn, metrics=("binary_accuracy",))
    results = []
    printer("Starting federated training")
    state_path = os.path.join(cfg.path, "fed_state", "state.pt")
    with Timer("Federated training", printer if comm.rank() == 0 else None):
        state = fed_avg.initialize()
        fp = _fed_fingerprint(cfg, state)
        if cfg.resume and os.path.exists(state_path):
            saved = load_server_extra(state_path) or {}
            # a state written before fingerprints were saved carries none: unknown, not different
            # (load_server_state still checks every tensor shape against the model)
            diff = {k: (saved[k], v) for k, v in fp.items() if k in saved and saved[k] != v}
            if not saved:
                printer(f"{state_path} carries no configuration fingerprint; resuming without the check")
            if diff:
                raise ValueError(f"{state_path} was written by a different federated configuration "
                                 f"(saved, current): {diff}; use another path or resume=False")
            state = load_server_state(state_path, state.model.trainable[0].device)
            if comm.rank() == 0:
                printer(f"Resuming federated training at round {state.round_num}")
                if state.round_num >= cfg.rounds:
                    printer(f"All {cfg.rounds} rounds are already done in {state_path}; nothing to train")
            # every client's shuffle continues where the finished rounds left it (one local
            # epoch per round), instead of replaying round 0's order
            for d in fed_train:
                if hasattr(d, "_epoch"):
                    d._epoch = state.round_num
        else:
            state = state_with_new_model_weights(
                state, [t.detach() for t in pre.net.trainable_weights],
                [t.detach() for t in pre.net.non_trainable_weights])
        state = broadcast_server_state(state)
        init_metrics = evaluation(state.model, fed_test)
        if comm.rank() == 0:
            printer("Initial model: {0:f} \n".format(init_metrics["binary_accuracy"]))
        for r in range(state.round_num, cfg.rounds):
            state, train_metrics = fed_avg.next(state, fed_train)
            test_metrics = evaluation(state.model, fed_test)
            results.append((r, train_metrics, test_metrics))
            if comm.rank() == 0:
                save_server_state(state, state_path, extra=fp)
                printer("{0:2d}, {1:f}, {2:f}, {3:f}, {4:f} \n".format(
                    r, train_metrics["binary_accuracy"], train_metrics["loss"],
                    test_metrics["binary_accuracy"], test_metrics["loss"]))
    return state, results


@dataclass
class SecureConfig:
    path: str = "."
    rounds: int = 5
    percent: float = 0.5
    arch: str = "tinycnn"
    input_shape: Tuple[int, int, int] = (10, 10, 3)
    num_clients: int = 2
    dataset_size: int = 30000
    batch_size: int = 32
    base_learning_rate: float = 1e-3
    epochs: int = 5
    mode: str = "mask"
    synthetic: bool = False
    seed: int = 0
    backend: str = "auto"


def run_secure(cfg: SecureConfig, printer=print):
    comm.init_process_group()
    dev = _local_device()
    strategy = OneDeviceStrategy(dev)
    if cfg.synthetic or not os.path.isdir(os.path.join(cfg.path, "data")):
        ds = synthetic_dataset(cfg.dataset_size, cfg.input_shape, 2, cfg.seed)
    else:
        ds = idc_dataset(cfg.path, "balanced", cfg.input_shape[0], cfg.seed)
    train_size = int(0.8 * cfg.dataset_size)
    test_size = int(0.2 * cfg.dataset_size)
    client_data = ds.take(train_size)
    test = prepare_for_training(ds.skip(train_size).take(test_size), cfg.batch_size, seed=cfg.seed + 3)
    client_size = train_size // cfg.num_clients
    ctrain, cval = int(0.8 * client_size), int(0.2 * client_size)
    shards = shard_clients(client_data, cfg.num_clients)
    cdata = [(prepare_for_training(s.take(ctrain), cfg.batch_size, seed=cfg.seed + i),
              prepare_for_training(s.skip(ctrain).take(cval), cfg.batch_size, seed=cfg.seed + 50 + i))
             for i, s in enumerate(shards)]

    def model_fn():
        net = build_model(cfg.arch, cfg.input_shape, 1, seed=cfg.seed)
        m = Model(net, strategy)
        m.compile(RMSprop(cfg.base_learning_rate), "binary_crossentropy", ["binary_accuracy", "auc"],
                  backend=cfg.backend)
        return m

    proc = SecureFederatedProcess(model_fn, cdata, cfg.percent, cfg.mode, cfg.epochs, cfg.seed)
    out = []
    with Timer("Secure fed model", printer if comm.rank() == 0 else None):
        for r in range(cfg.rounds):
            logs = proc.run_round(test)
            if logs is not None:
                printer(logs["loss"], logs.get("accuracy"), logs.get("auc"))
                out.append(logs)
    return proc, out
