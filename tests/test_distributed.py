"""Multi-process data parallelism on the CPU (gloo, world_size 2) — SURVEY §4.2 T4.

The same code paths run over RCCL on MI355X (backend "nccl"); here they are exercised with gloo so
the invariants are checked without a GPU: DP(N, B/N) == single process (B), CentralStorage ==
Mirrored, metrics reduced over the whole global batch, BN moving statistics identical on every
rank, FedAvg / secure aggregation results independent of how clients are spread over ranks.
"""
import numpy as np
import pytest
import torch

from idc_models_amd.parallel.launch import spawn

B = 16


def _data():
    from idc_models_amd.data import synthetic_dataset
    return synthetic_dataset(64, (10, 10, 3), seed=11, signal=30.0)


def _nodrop(net):
    """Dropout masks come from per-process RNG streams; the equivalences are checked without it."""
    for l in net.layers:
        if l.keras_class == "Dropout":
            l.rate = 0.0
    return net


def _fit(strategy, arch="tinycnn", shape=(10, 10, 3), epochs=2, ds=None):
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model
    ds = ds if ds is not None else _data()
    torch.manual_seed(0)
    m = Model(_nodrop(build_model(arch, shape, seed=3)), strategy)
    m.compile(RMSprop(1e-2), "binary_crossentropy", ["accuracy", "auc"], backend="eager")
    batches = ds.batch(B, drop_remainder=True)
    h = m.fit(batches, epochs=epochs, verbose=0)
    ev = m.evaluate(batches, return_dict=True)
    return [w for w in m.get_weights()], {k: v[-1] for k, v in h.history.items()}, ev


def _dp_worker(rank, world, kind):
    from idc_models_amd.parallel import CentralStorageStrategy, MirroredStrategy
    st = MirroredStrategy(backend="gloo") if kind == "mirrored" else CentralStorageStrategy(backend="gloo")
    st.bucket_bytes = 4096  # several buckets even for the tiny model
    return _fit(st)


def _single():
    from idc_models_amd.parallel import OneDeviceStrategy
    return _fit(OneDeviceStrategy("cpu"))


@pytest.fixture(scope="module")
def single():
    return _single()


@pytest.mark.parametrize("kind", ["mirrored", "central"])
def test_data_parallel_equals_single_process(kind, single):
    res = spawn(_dp_worker, 2, (kind,))
    w0, logs0, ev0 = res[0]
    w1, _, ev1 = res[1]
    ws, logss, evs = single
    for a, b, c in zip(w0, w1, ws):
        np.testing.assert_array_equal(a, b)  # replicas stay bit-identical
        np.testing.assert_allclose(a, c, rtol=2e-4, atol=2e-5)
    # metrics are over the GLOBAL batch on every rank
    assert ev0 == ev1
    for k in evs:
        assert ev0[k] == pytest.approx(evs[k], rel=1e-3, abs=1e-4), k
    assert logs0["loss"] == pytest.approx(logss["loss"], rel=1e-3)


def _bn_worker(rank, world):
    from idc_models_amd.data import synthetic_dataset
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model
    from idc_models_amd.parallel import MirroredStrategy
    st = MirroredStrategy(backend="gloo")
    m = Model(build_model("mobilenetv2", (32, 32, 3), seed=1), st)
    m.compile(RMSprop(1e-3), "binary_crossentropy", ["accuracy"], backend="eager")
    ds = synthetic_dataset(32, (32, 32, 3), seed=2)
    m.fit(ds.batch(16, drop_remainder=True), epochs=1, verbose=0)
    bn = m.net.base.get_layer("Conv_1_bn")
    return bn.moving_mean.numpy().copy(), bn.moving_variance.numpy().copy()


def test_bn_moving_stats_synchronised():
    (m0, v0), (m1, v1) = spawn(_bn_worker, 2)
    np.testing.assert_array_equal(m0, m1)
    np.testing.assert_array_equal(v0, v1)
    assert not np.allclose(m0, 0.0)


def _fed_worker(rank, world):
    return _fedavg_run()


def _fedavg_run():
    from idc_models_amd.data import contiguous_clients, prepare_for_training, synthetic_dataset
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.fed import build_federated_averaging_process, build_federated_evaluation
    from idc_models_amd.models import build_model
    from idc_models_amd.parallel import OneDeviceStrategy
    ds = synthetic_dataset(120, (10, 10, 3), seed=4, signal=30.0)
    clients = contiguous_clients(ds, 6, 20)
    fed_train = [c.batch(10) for c in clients[:4]]
    fed_test = [c.batch(10) for c in clients[4:]]

    def model_fn():
        return Model(_nodrop(build_model("tinycnn", seed=5)), OneDeviceStrategy("cpu"))

    proc = build_federated_averaging_process(model_fn, lambda: RMSprop(1e-2))
    ev = build_federated_evaluation(model_fn)
    state = proc.initialize()
    out = []
    for _ in range(2):
        state, tm = proc.next(state, fed_train)
        out.append((dict(tm), dict(ev(state.model, fed_test))))
    return [t.numpy().copy() for t in state.model.trainable], out


def test_fedavg_independent_of_rank_layout():
    single = _fedavg_run()
    res = spawn(_fed_worker, 2)
    for a, b in zip(res[0][0], single[0]):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)
    for (tm, em), (tm1, em1) in zip(res[0][1], single[1]):
        for k in tm:
            assert tm[k] == pytest.approx(tm1[k], rel=1e-5)
        for k in em:
            assert em[k] == pytest.approx(em1[k], rel=1e-5)


def _secure_worker(rank, world, mode):
    return _secure_run(mode)


def _secure_run(mode):
    from idc_models_amd.data import shard_clients, synthetic_dataset
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.fed import SecureFederatedProcess
    from idc_models_amd.models import build_model
    from idc_models_amd.parallel import OneDeviceStrategy
    ds = synthetic_dataset(80, (10, 10, 3), seed=7, signal=30.0)
    shards = shard_clients(ds, 4)
    cdata = [(s.take(16).batch(8), s.skip(16).batch(8)) for s in shards]

    def model_fn():
        m = Model(_nodrop(build_model("tinycnn", seed=1)), OneDeviceStrategy("cpu"))
        m.compile(RMSprop(1e-3), "binary_crossentropy", ["accuracy", "auc"], backend="eager")
        return m

    proc = SecureFederatedProcess(model_fn, cdata, percent=0.5, mode=mode, epochs=1, seed=3)
    for k in proc.mine:
        proc.client_fit(k)
    local = {k: [w.clone() for w in proc.states[k].weights] for k in proc.mine}
    avg = proc.aggregate()
    return [a.numpy().copy() for a in avg], {k: [w.numpy() for w in v] for k, v in local.items()}


def test_secure_masked_aggregation_two_ranks():
    res = spawn(_secure_worker, 2, ("mask",))
    avg0, loc0 = res[0]
    avg1, loc1 = res[1]
    allw = {**loc0, **loc1}
    assert sorted(allw) == [0, 1, 2, 3]
    for i, a in enumerate(avg0):
        plain = np.mean([allw[k][i] for k in range(4)], axis=0)
        np.testing.assert_array_equal(a, avg1[i])
        np.testing.assert_allclose(a, plain, atol=1e-6)


def _secure_fedavg_run():
    from idc_models_amd.data import contiguous_clients, synthetic_dataset
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.fed import build_federated_averaging_process
    from idc_models_amd.models import build_model
    from idc_models_amd.parallel import OneDeviceStrategy
    ds = synthetic_dataset(120, (10, 10, 3), seed=4, signal=30.0)
    clients = [c.batch(10) for c in contiguous_clients(ds, 4, 30)]

    def model_fn():
        return Model(_nodrop(build_model("tinycnn", seed=5)), OneDeviceStrategy("cpu"))

    proc = build_federated_averaging_process(model_fn, lambda: RMSprop(1e-2), secure_aggregation="mask")
    state = proc.initialize()
    state, tm = proc.next(state, clients)
    return [t.numpy().copy() for t in state.model.trainable], dict(tm)


def _secure_fedavg_worker(rank, world):
    return _secure_fedavg_run()


def test_secure_fedavg_two_ranks_equals_single_process():
    """Masked weighted-delta FedAvg over 2 gloo ranks (clients 0,2 | 1,3; the int32 masked sums and
    the public keys cross ranks) equals the single-process masked run and matches it bit for bit
    across the two ranks."""
    single = _secure_fedavg_run()
    res = spawn(_secure_fedavg_worker, 2)
    for a, b, c in zip(res[0][0], res[1][0], single[0]):
        np.testing.assert_array_equal(a, b)
        np.testing.assert_allclose(a, c, rtol=1e-5, atol=1e-6)
    for k in single[1]:
        assert res[0][1][k] == pytest.approx(single[1][k], rel=1e-5)
