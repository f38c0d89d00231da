"""Federated learning and secure aggregation on the CPU."""
import numpy as np
import pytest
import torch

from idc_models_amd.fed import secagg
from idc_models_amd.fed.paillier import (decrypt_vector, encrypt_vector, generate_paillier_keypair,
                                         sum_ciphertexts)


@pytest.mark.parametrize("K", [2, 3, 8])
def test_pairwise_masks_cancel_exactly(K):
    rng = np.random.default_rng(K)
    xs = [torch.tensor(rng.normal(size=1000).astype(np.float32)) for _ in range(K)]
    scale = secagg.choose_scale(max(float(x.abs().max()) for x in xs), K)
    total = np.zeros(1000, np.uint64)
    masked = []
    for k, x in enumerate(xs):
        m = secagg.mask_quantize(x, scale, K, k, seed=123, round_=5)
        masked.append(m)
        total = (total + m.numpy().view(np.uint32).astype(np.uint64)) & np.uint64(0xFFFFFFFF)
    t32 = torch.from_numpy(total.astype(np.uint32).view(np.int32).copy())
    mean = secagg.unmask_mean(t32, scale, K, float(K))
    isum = sum(torch.round(x * scale).to(torch.int64) for x in xs)
    assert torch.equal(t32.to(torch.int64), isum)  # masks cancel: the exact fixed-point sum
    plain = isum.to(torch.int32).float() / (scale * K)
    assert torch.equal(mean, plain)  # bit-exact vs the unmasked fixed-point mean
    assert torch.allclose(mean, torch.stack(xs).mean(0), atol=1.0 / scale)
    # a single masked vector carries no usable signal about its input
    q0 = torch.round(xs[0] * scale).to(torch.int64)
    corr = np.corrcoef(masked[0].numpy().astype(np.float64), q0.numpy().astype(np.float64))[0, 1]
    assert abs(corr) < 0.1


def test_masks_change_every_round_and_pair():
    x = torch.zeros(64)
    a = secagg.mask_quantize(x, 1.0, 3, 0, 1, 0)
    b = secagg.mask_quantize(x, 1.0, 3, 0, 1, 1)
    c = secagg.mask_quantize(x, 1.0, 3, 1, 1, 0)
    assert not torch.equal(a, b) and not torch.equal(a, c)


def test_philox_known_answer():
    """Philox4x32-10 word 0 for counter=0, key=0 (Random123 KAT: 6627e8d5)."""
    out = secagg._philox_np(np.zeros(1, np.uint64), np.zeros(1, np.uint64), 0, 0, 0, 0)
    assert int(out[0]) == 0x6627E8D5


def test_paillier_homomorphic_mean():
    pub, priv = generate_paillier_keypair(256)
    vals = [[0.5, -1.25, 3.0], [1.5, 0.25, -3.0], [-0.5, 1.0, 0.0]]
    cts = [encrypt_vector(pub, v, 2 ** 20) for v in vals]
    mean = decrypt_vector(priv, sum_ciphertexts(pub, cts), 2 ** 20, 3.0)
    np.testing.assert_allclose(mean, np.mean(vals, axis=0), atol=1e-5)


def _tiny_fed(n_clients=3, bad=None):
    from idc_models_amd.data import contiguous_clients, synthetic_dataset
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.fed import build_federated_averaging_process
    from idc_models_amd.models import build_model
    from idc_models_amd.parallel import OneDeviceStrategy
    ds = synthetic_dataset(60, (10, 10, 3), seed=1)
    clients = [c.batch(10, shuffle=False) for c in contiguous_clients(ds, n_clients, 60 // n_clients)]

    def model_fn():
        net = build_model("tinycnn", seed=2)
        for l in net.layers:
            if l.keras_class == "Dropout":
                l.rate = 0.0
        return Model(net, OneDeviceStrategy("cpu"))

    return build_federated_averaging_process(model_fn, lambda: RMSprop(1e-2)), clients, model_fn


def test_fedavg_is_example_weighted_mean_of_client_models():
    from idc_models_amd.engine import RMSprop
    proc, clients, model_fn = _tiny_fed()
    state = proc.initialize()
    new, metrics = proc.next(state, clients)
    # independent clients trained from the same start with a fresh optimizer
    finals = []
    for c in clients:
        m = model_fn()
        m.compile(RMSprop(1e-2), "binary_crossentropy", ["binary_accuracy"])
        for t, w in zip(m.net.trainable_weights, state.model.trainable):
            t.data.copy_(w)
        m.fit(c, epochs=1, verbose=0)
        finals.append([t.detach().clone() for t in m.net.trainable_weights])
    for i, w in enumerate(new.model.trainable):
        ref = sum(f[i] for f in finals) / len(finals)  # equal client sizes
        assert torch.allclose(w, ref, atol=1e-6)
    assert set(metrics) == {"binary_accuracy", "loss"} and new.round_num == 1


def test_fedavg_skips_non_finite_client():
    proc, clients, _ = _tiny_fed()
    state = proc.initialize()
    m = proc.worker()
    orig_fit = m.fit
    calls = {"n": 0}

    def fit(ds, **kw):
        calls["n"] += 1
        h = orig_fit(ds, **kw)
        if calls["n"] == 2:
            with torch.no_grad():
                m.net.trainable_weights[0].fill_(float("nan"))
        return h

    m.fit = fit
    new, _ = proc.next(state, clients)
    assert all(torch.isfinite(w).all() for w in new.model.trainable)


def test_state_with_new_model_weights_shape_check():
    from idc_models_amd.fed import state_with_new_model_weights
    proc, _, _ = _tiny_fed()
    st = proc.initialize()
    st2 = state_with_new_model_weights(st, [w + 1 for w in st.model.trainable], st.model.non_trainable)
    assert torch.equal(st2.model.trainable[0], st.model.trainable[0] + 1)
    with pytest.raises(ValueError):
        state_with_new_model_weights(st, [w[:1] for w in st.model.trainable], [])


def test_secure_process_paillier_equals_plain_mean():
    from idc_models_amd.data import shard_clients, synthetic_dataset
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.fed import SecureFederatedProcess
    from idc_models_amd.models import build_model
    from idc_models_amd.parallel import OneDeviceStrategy
    ds = synthetic_dataset(40, (10, 10, 3), seed=3)
    cdata = [(s.take(16).batch(8), s.skip(16).batch(8)) for s in shard_clients(ds, 2)]

    def model_fn():
        m = Model(build_model("tinycnn", seed=0), OneDeviceStrategy("cpu"))
        m.compile(RMSprop(1e-3), "binary_crossentropy", ["binary_accuracy", "auc"])
        return m

    proc = SecureFederatedProcess(model_fn, cdata, percent=0.5, mode="paillier", epochs=1,
                                  paillier_bits=256)
    for k in proc.mine:
        proc.client_fit(k)
    plain = [(a + b) / 2 for a, b in zip(proc.states[0].weights, proc.states[1].weights)]
    avg = proc.aggregate()
    for a, p in zip(avg, plain):
        assert torch.allclose(a, p, atol=1e-6)
    logs = proc.run_round(cdata[0][1])
    assert {"loss", "accuracy", "auc"} <= set(logs)
    # Q15: client optimizer state persists across rounds
    assert float(proc.states[0].opt_slots["ms"].abs().sum()) > 0


def test_fedavg_participating_subset_reweights():
    from idc_models_amd.engine import RMSprop
    proc, clients, model_fn = _tiny_fed(n_clients=3)
    state = proc.initialize()
    new, _ = proc.next(state, clients, participating=[0, 2])
    finals = []
    for k in (0, 2):
        m = model_fn()
        m.compile(RMSprop(1e-2), "binary_crossentropy", ["binary_accuracy"])
        for t, w in zip(m.net.trainable_weights, state.model.trainable):
            t.data.copy_(w)
        m.fit(clients[k], epochs=1, verbose=0)
        finals.append([t.detach().clone() for t in m.net.trainable_weights])
    for i, w in enumerate(new.model.trainable):
        assert torch.allclose(w, (finals[0][i] + finals[1][i]) / 2, atol=1e-6)


@pytest.mark.parametrize("mode", ["mask", "paillier"])
def test_secure_aggregation_survives_client_dropout(mode):
    """A client drops out before masking: the round is re-keyed among the survivors, whose masks
    still cancel, and the result is the survivors' plain mean."""
    from idc_models_amd.data import shard_clients, synthetic_dataset
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.fed import SecureFederatedProcess
    from idc_models_amd.models import build_model
    from idc_models_amd.parallel import OneDeviceStrategy
    ds = synthetic_dataset(80, (10, 10, 3), seed=5)
    cdata = [(s.take(12).batch(6), s.skip(12).batch(6)) for s in shard_clients(ds, 4)]

    def model_fn():
        m = Model(build_model("tinycnn", seed=0), OneDeviceStrategy("cpu"))
        m.compile(RMSprop(1e-3), "binary_crossentropy", ["binary_accuracy"])
        return m

    proc = SecureFederatedProcess(model_fn, cdata, percent=1.0, mode=mode, epochs=1, paillier_bits=256)
    for k in (0, 1, 3):
        proc.client_fit(k)
    avg = proc.aggregate(dropped={2})
    for i, a in enumerate(avg):
        plain = sum(proc.states[k].weights[i] for k in (0, 1, 3)) / 3
        assert torch.allclose(a, plain, atol=1e-5)
    # without re-keying the dropped client's masks would not cancel: check that it matters
    from idc_models_amd.fed import secagg
    x = torch.ones(16)
    full = [secagg.mask_quantize(x, 1.0, 4, k, 1, 0) for k in (0, 1, 3)]
    s = sum(t.to(torch.int64) for t in full) % (1 << 32)
    assert not torch.equal(s, torch.full((16,), 3, dtype=torch.int64))
