"""Federated learning and secure aggregation on the CPU."""
import numpy as np
import pytest
import torch

from idc_models_amd.fed import secagg
from idc_models_amd.fed.paillier import (decrypt_vector, encrypt_vector, generate_paillier_keypair,
                                         sum_ciphertexts)


def _keys(K, round_=5, participants=None):
    from idc_models_amd.fed.keyagree import ClientKeys
    ks = {k: ClientKeys(k) for k in range(K)}
    pubs = {k: ks[k].public for k in range(K)}
    parts = list(range(K)) if participants is None else list(participants)
    return ks, pubs, {k: ks[k].round_keys(pubs, round_, parts) for k in parts}


@pytest.mark.parametrize("K", [2, 3, 8])
def test_pairwise_masks_cancel_exactly(K):
    rng = np.random.default_rng(K)
    sizes = [700, 300]  # two protected tensors with their own fixed-point scales
    xs = [torch.tensor(np.concatenate([rng.normal(size=700), 50 * rng.normal(size=300)]).astype(np.float32))
          for _ in range(K)]
    seg = secagg.segment_ends(sizes)
    mx = [max(float(x[:700].abs().max()) for x in xs), max(float(x[700:].abs().max()) for x in xs)]
    scales = secagg.choose_scales(mx, K)
    assert scales[0] > scales[1]  # the small-range tensor gets the finer scale
    _, _, rk = _keys(K)
    total = np.zeros(1000, np.uint64)
    masked = []
    for k, x in enumerate(xs):
        m = secagg.mask_quantize(x, scales, seg, K, k, rk[k], round_=5)
        masked.append(m)
        total = (total + m.numpy().view(np.uint32).astype(np.uint64)) & np.uint64(0xFFFFFFFF)
    t32 = torch.from_numpy(total.astype(np.uint32).view(np.int32).copy())
    mean = secagg.unmask(t32, scales, seg, float(K))
    sc = torch.from_numpy(np.repeat(scales, sizes))
    isum = sum(torch.round(x * sc).to(torch.int64) for x in xs)
    assert torch.equal(t32.to(torch.int64), isum)  # masks cancel: the exact fixed-point sum
    plain = isum.to(torch.int32).float() / (sc * K)
    assert torch.equal(mean, plain)  # bit-exact vs the unmasked fixed-point mean
    assert torch.allclose(mean, torch.stack(xs).mean(0), atol=float(1.0 / scales.min()))
    # a single masked vector carries no usable signal about its input
    q0 = torch.round(xs[0] * sc).to(torch.int64)
    corr = np.corrcoef(masked[0].numpy().astype(np.float64), q0.numpy().astype(np.float64))[0, 1]
    assert abs(corr) < 0.1


def test_masks_change_every_round_and_pair():
    x = torch.zeros(64)
    seg = secagg.segment_ends([64])
    ks, pubs, rk = _keys(3, round_=0)
    a = secagg.mask_quantize(x, [1.0], seg, 3, 0, rk[0], 0)
    b = secagg.mask_quantize(x, [1.0], seg, 3, 0, ks[0].round_keys(pubs, 1, range(3)), 1)
    c = secagg.mask_quantize(x, [1.0], seg, 3, 1, rk[1], 0)
    assert not torch.equal(a, b) and not torch.equal(a, c)


def test_aggregator_view_does_not_determine_masks():
    """Pair keys come from Diffie-Hellman secrets: both endpoints derive the same key, the masks
    still cancel, but nothing the aggregator holds (public keys, masked vectors, indices, round,
    configuration seeds) reproduces a client's mask — and the same public configuration with fresh
    private keys yields unrelated masks."""
    from idc_models_amd.fed import keyagree
    K, n, rnd = 3, 256, 4
    seg = secagg.segment_ends([n])
    zero = torch.zeros(n)
    ks, pubs, rk = _keys(K, rnd)
    assert rk[0][1] == rk[1][0] and rk[1][2] == rk[2][1]  # S_ij = S_ji
    masks = [secagg.mask_quantize(zero, [1.0], seg, K, k, rk[k], rnd) for k in range(K)]  # x=0: pure masks
    assert int(sum(m.to(torch.int64) for m in masks).remainder(1 << 32).abs().sum()) == 0
    # candidate keys an aggregator could derive from its view
    cands = []
    for seed in (0, 7919, 1234):  # the old public-seed derivation
        for lo, hi in ((0, 1), (0, 2)):
            cands.append(((seed & 0xFFFFFFFF) ^ ((lo * 0x9E3779B1) & 0xFFFFFFFF),
                          ((seed >> 32) & 0xFFFFFFFF) ^ ((hi * 0x85EBCA77) & 0xFFFFFFFF)))
    cands.append(keyagree.pair_mask_key(pubs[0] * pubs[1] % keyagree.P, rnd, 0, 1))
    cands.append(keyagree.pair_mask_key(pubs[0] ^ pubs[1], rnd, 0, 1))
    for c1 in cands:
        for c2 in cands:
            guess = secagg.mask_quantize(zero, [1.0], seg, K, 0, {1: c1, 2: c2}, rnd)
            assert not torch.equal(guess, masks[0])
    # same public configuration, fresh private keys: unrelated masks (not a function of it)
    _, _, rk2 = _keys(K, rnd)
    again = secagg.mask_quantize(zero, [1.0], seg, K, 0, rk2[0], rnd)
    assert not torch.equal(again, masks[0])
    assert (again == masks[0]).float().mean() < 0.01
    # degenerate / out-of-subgroup public values are refused
    for bad in (0, 1, keyagree.P - 1, keyagree.P):
        with pytest.raises(ValueError):
            keyagree.check_public(bad)
    nonres = next(g for g in range(3, 50) if pow(g, keyagree.Q, keyagree.P) != 1)
    with pytest.raises(ValueError):
        keyagree.check_public(nonres)


def test_per_tensor_scales_keep_small_tensor_resolution():
    """One global scale chosen from the largest protected value (a BN moving variance of ~1e4)
    leaves a small conv kernel a few quantisation steps; per-tensor scales keep its resolution."""
    K = 4
    rng = np.random.default_rng(0)
    small = [rng.normal(scale=1e-3, size=512).astype(np.float32) for _ in range(K)]
    big = [np.abs(rng.normal(scale=1e4, size=64)).astype(np.float32) for _ in range(K)]
    xs = [torch.tensor(np.concatenate([a, b])) for a, b in zip(small, big)]
    sizes = [512, 64]
    seg = secagg.segment_ends(sizes)
    _, _, rk = _keys(K)
    ref = torch.stack(xs).mean(0)

    def run(scales):
        tot = sum(secagg.mask_quantize(x, scales, seg, K, k, rk[k], 5).to(torch.int64) for k, x in enumerate(xs))
        t = tot.remainder(1 << 32)
        t32 = torch.where(t >= (1 << 31), t - (1 << 32), t).to(torch.int32)
        return secagg.unmask(t32, scales, seg, float(K))

    per = run(secagg.choose_scales([max(np.abs(a).max() for a in small), max(b.max() for b in big)], K))
    glob = secagg.choose_scales([max(b.max() for b in big)], K)[0]
    one = run([glob, glob])
    e_per = float((per[:512] - ref[:512]).abs().max())
    e_one = float((one[:512] - ref[:512]).abs().max())
    assert e_per < 1e-7 < e_one and e_per * 1000 < e_one


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
            # a diverged client also reports a non-finite loss / metric: it must not
            # reach the round's metrics (NaN * weight 0 is still NaN)
            for k in h.history:
                h.history[k][-1] = float("nan")
        return h

    m.fit = fit
    new, mets = proc.next(state, clients)
    assert all(torch.isfinite(w).all() for w in new.model.trainable)
    assert mets and all(np.isfinite(v) for v in mets.values()), mets


def test_fedavg_secure_mask_equals_plain_weighted_mean():
    """Secure FedAvg (config #5): masked example-weighted deltas sum to the plain FedAvg update
    within the per-tensor fixed-point resolution; a non-finite client still takes part in the
    masking (zero vector, weight 0) so the others' masks cancel."""
    from idc_models_amd.engine import RMSprop
    from idc_models_amd.fed import build_federated_averaging_process
    plain, clients, model_fn = _tiny_fed()
    sec = build_federated_averaging_process(model_fn, lambda: RMSprop(1e-2), secure_aggregation="mask")
    s0 = plain.initialize()
    s1 = sec.initialize()
    for a, b in zip(s0.model.trainable, s1.model.trainable):
        b.copy_(a)
    n0, m0 = plain.next(s0, clients)
    n1, m1 = sec.next(s1, clients)
    for a, b in zip(n0.model.trainable, n1.model.trainable):
        assert torch.allclose(a, b, atol=1e-6), float((a - b).abs().max())
    assert m0 == pytest.approx(m1)
    # a poisoned client: weight 0 in both, masks still cancel
    w = sec.worker()
    orig = w.fit
    calls = {"n": 0}

    def fit(ds, **kw):
        calls["n"] += 1
        h = orig(ds, **kw)
        if calls["n"] == 1:
            with torch.no_grad():
                w.net.trainable_weights[0].fill_(float("inf"))
        return h

    w.fit = fit
    n2, _ = sec.next(n1, clients)
    assert all(torch.isfinite(t).all() for t in n2.model.trainable)


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
    ks, pubs, _ = _keys(4, 0)
    seg = secagg.segment_ends([16])
    full = [secagg.mask_quantize(x, [1.0], seg, 4, k, ks[k].round_keys(pubs, 0, range(4)), 0) for k in (0, 1, 3)]
    s = sum(t.to(torch.int64) for t in full) % (1 << 32)
    assert not torch.equal(s, torch.full((16,), 3, dtype=torch.int64))


def test_choose_scales_stays_finite_for_tiny_segments():
    """A tiny-but-nonzero protected tensor must not overflow its float32 fixed-point scale."""
    sc = secagg.choose_scales([1e-35, 1.0, 0.0], 8)
    assert np.all(np.isfinite(sc)) and sc[0] == np.float32(2.0 ** 100)
    x = torch.tensor([1e-35, -3e-36, 0.5, -0.25, 0.0])
    q = secagg.mask_quantize(x, sc[:2], np.array([2, 5]), 1, 0, {}, 0)
    back = secagg.unmask(q, sc[:2], np.array([2, 5]))
    assert torch.isfinite(back).all()
    assert torch.allclose(back[2:4], x[2:4], atol=1e-8)


def test_fedavg_skips_client_with_non_finite_bn_statistics():
    """average_bn_stats: a client whose BatchNorm statistics are non-finite gets weight 0 too."""
    from idc_models_amd.data import synthetic_dataset, contiguous_clients
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.fed import build_federated_averaging_process
    from idc_models_amd.models import build_model
    from idc_models_amd.parallel import OneDeviceStrategy
    ds = synthetic_dataset(16, (32, 32, 3), 2, seed=1)
    clients = [c.batch(8, True, 100, True, seed=i) for i, c in enumerate(contiguous_clients(ds, 2, 8))]
    base = build_model("mobilenetv2", (32, 32, 3), 1, seed=0)

    def model_fn():
        import copy
        return Model(copy.deepcopy(base), OneDeviceStrategy("cpu"))

    proc = build_federated_averaging_process(model_fn, lambda: RMSprop(1e-3), average_bn_stats=True,
                                             backend="eager")
    state = proc.initialize()
    m = proc.worker()
    orig_fit = m.fit
    calls = {"n": 0}

    def fit(d, **kw):
        calls["n"] += 1
        h = orig_fit(d, **kw)
        if calls["n"] == 2:
            with torch.no_grad():
                m.net.non_trainable_weights[0].fill_(float("inf"))
        return h

    m.fit = fit
    new, _ = proc.next(state, clients)
    assert all(torch.isfinite(w).all() for w in new.model.non_trainable)
    assert all(torch.isfinite(w).all() for w in new.model.trainable)


def test_fed_resume_refuses_a_foreign_state(tmp_path):
    from idc_models_amd.fed import ModelWeights, ServerState, save_server_state
    from idc_models_amd.recipes.federated import FedConfig, _fed_fingerprint
    cfg = FedConfig(path=str(tmp_path), arch="tinycnn")
    st = ServerState(ModelWeights([torch.zeros(3, 3)], []), 2)
    fp = _fed_fingerprint(cfg, st)
    p = tmp_path / "fed_state" / "state.pt"
    save_server_state(st, str(p), extra=fp)
    from idc_models_amd.fed import load_server_extra
    assert load_server_extra(str(p)) == fp
    other = _fed_fingerprint(FedConfig(path=str(tmp_path), arch="vgg16", num_clients=4), st)
    assert other != fp
