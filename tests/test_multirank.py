"""Multi-GPU readiness without an 8-GPU node, on the CPU:

* the world > 1 unique-id bootstrap of the native RCCL communicator (``parallel/native_comm.py``)
  against a real TCPStore, with a fake native module standing in for RCCL;
* 4-rank gloo runs: data parallelism over an unevenly split global batch equals the single process
  on that batch; FedAvg with 8 clients over 4 ranks equals 1 rank; the masked secure sum of 8
  clients over 4 ranks is bitwise the plain fixed-point sum, through the mod-2^32 ring sum whose
  operands cross 2^31;
* (the communicator watchdog: ``tests/test_watchdog.py``).

Reference configurations these rehearse: 4 GPUs (``/root/reference/dist_model_tf_dense.py:16-22``),
8 train clients (``/root/reference/fed_model.py:47-49,207-229``), the secure aggregation round
(``/root/reference/secure_fed_model.py:156-168``).
"""
import numpy as np
import pytest
import torch

from idc_models_amd.parallel.launch import spawn

# ---------------------------------------------------------------------------------------------
# native bootstrap with a fake RCCL module


class _FakeComm:
    made = []

    def __init__(self, rank, world, uid, device, init_timeout_s=0.0):
        self.rank, self.world, self.uid, self.device, self.init_timeout_s = rank, world, uid, device, init_timeout_s
        self.stream = 0
        _FakeComm.made.append(self)

    @staticmethod
    def make_unique_id():
        return bytes(np.random.default_rng().integers(0, 256, 128, dtype=np.uint8))

    def close(self):
        pass


class _FakeExt:
    Communicator = _FakeComm


def _bootstrap_worker(rank, world):
    from idc_models_amd.parallel.native_comm import NativeCommunicator
    # the default group's TCPStore (gloo here, RCCL's bootstrap on a GPU node) carries the id
    nc = NativeCommunicator(rank, world, torch.device("cuda", rank), ext=_FakeExt(), watchdog=False)
    c = nc.c
    return c.uid, c.rank, c.world, c.device, c.init_timeout_s


def test_native_bootstrap_world4_shares_one_unique_id():
    res = spawn(_bootstrap_worker, 4)
    uids = {r[0] for r in res}
    assert len(uids) == 1 and len(next(iter(uids))) == 128
    for r, (_, rank, world, device, tmo) in enumerate(res):
        assert (rank, world, device) == (r, 4, r)
        assert tmo > 0  # a world > 1 is created non-blocking, with an init timeout


# ---------------------------------------------------------------------------------------------
# 4-rank gloo runs

GB = 14  # global batch: 4 ranks -> 4, 4, 3, 3 rows (uneven)


def _batches():
    from idc_models_amd.data import synthetic_dataset
    ds = synthetic_dataset(3 * GB, (10, 10, 3), seed=21, signal=30.0)
    x, y = torch.as_tensor(ds.x), torch.as_tensor(ds.y)
    return [(x[i:i + GB], y[i:i + GB]) for i in range(0, 3 * GB, GB)]


def _dp_fit(strategy):
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model
    net = build_model("tinycnn", seed=3)
    for l in net.layers:
        if l.keras_class == "Dropout":
            l.rate = 0.0
    m = Model(net, strategy)
    m.compile(RMSprop(1e-2), "binary_crossentropy", ["accuracy"], backend="eager")
    m.fit(_batches(), epochs=2, verbose=0)
    return [w.copy() for w in m.get_weights()]


def _dp4_worker(rank, world):
    from idc_models_amd.parallel import MirroredStrategy
    st = MirroredStrategy(backend="gloo")
    st.bucket_bytes = 2048
    return _dp_fit(st)


def test_dp_world4_uneven_split_equals_single_process():
    from idc_models_amd.parallel import OneDeviceStrategy
    single = _dp_fit(OneDeviceStrategy("cpu"))
    res = spawn(_dp4_worker, 4)
    for r in range(1, 4):
        for a, b in zip(res[0], res[r]):
            np.testing.assert_array_equal(a, b)  # replicas stay bit-identical
    for a, c in zip(res[0], single):
        np.testing.assert_allclose(a, c, rtol=2e-4, atol=2e-5)


def _fedavg8():
    from idc_models_amd.data import contiguous_clients, synthetic_dataset
    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.fed import build_federated_averaging_process
    from idc_models_amd.models import build_model
    from idc_models_amd.parallel import OneDeviceStrategy
    ds = synthetic_dataset(160, (10, 10, 3), seed=4, signal=30.0)
    clients = [c.batch(10) for c in contiguous_clients(ds, 8, 20)]

    def model_fn():
        net = build_model("tinycnn", seed=5)
        for l in net.layers:
            if l.keras_class == "Dropout":
                l.rate = 0.0
        return Model(net, OneDeviceStrategy("cpu"))

    proc = build_federated_averaging_process(model_fn, lambda: RMSprop(1e-2))
    state = proc.initialize()
    mets = []
    for _ in range(2):
        state, tm = proc.next(state, clients)
        mets.append(dict(tm))
    return [t.numpy().copy() for t in state.model.trainable], mets


def _fedavg8_worker(rank, world):
    return _fedavg8()


def test_fedavg_8_clients_over_4_ranks_equals_one_rank():
    single = _fedavg8()
    res = spawn(_fedavg8_worker, 4)
    for r in range(1, 4):
        for a, b in zip(res[0][0], res[r][0]):
            np.testing.assert_array_equal(a, b)
    for a, c in zip(res[0][0], single[0]):
        np.testing.assert_allclose(a, c, rtol=1e-5, atol=1e-6)
    for tm, tm1 in zip(res[0][1], single[1]):
        for k in tm1:
            assert tm[k] == pytest.approx(tm1[k], rel=1e-5)


def _ring_worker(rank, world):
    from idc_models_amd.parallel import comm
    # every rank contributes values just below 2^31 (as uint32 patterns: some above 2^31), so the
    # running sum wraps several times
    base = np.array([0x7FFFFFF0, 0xFFFFFFF0, 0x80000001, 12345], dtype=np.uint64) + rank
    t = torch.from_numpy(base.astype(np.uint32).view(np.int32).copy())
    comm.ring_sum_u32_(t)
    return t.numpy().view(np.uint32).copy()


def test_ring_sum_u32_world4_wraps_mod_2_32():
    res = spawn(_ring_worker, 4)
    base = np.array([0x7FFFFFF0, 0xFFFFFFF0, 0x80000001, 12345], dtype=np.uint64)
    want = ((4 * base + 0 + 1 + 2 + 3) % (1 << 32)).astype(np.uint32)
    for r in res:
        np.testing.assert_array_equal(r, want)


K8 = 8
SIZES = [37, 5, 130]


def _client_vec(k):
    g = torch.Generator().manual_seed(100 + k)
    v = torch.randn(sum(SIZES), generator=g) * (1.0 + k)
    v[0] = 50.0 * (1 if k % 2 else -1)  # big entries: fixed-point values near the int32 limit
    return v


def _secure8_worker(rank, world):
    from idc_models_amd.fed.secagg import MaskedAggregator
    from idc_models_amd.parallel import comm
    mine = [k for k in range(K8) if k % world == rank]
    agg = MaskedAggregator(K8, mine, "cpu")
    out = agg.masked_sum({k: _client_vec(k) for k in mine}, SIZES, round_=3)
    assert comm.world_size() == world
    return out.numpy().copy(), np.asarray(agg.last_scales).copy()


def test_secure_masked_sum_8_clients_over_4_ranks_is_bitwise_plain_sum():
    from idc_models_amd.fed.secagg import segment_ends, unmask
    res = spawn(_secure8_worker, 4)
    scales = res[0][1]
    seg_end = segment_ends(SIZES)
    sidx = np.searchsorted(seg_end, np.arange(sum(SIZES)), side="right")
    # the plain fixed-point sum of the 8 unmasked clients (int64: no wrap), as unmask decodes it
    from idc_models_amd.fed.secagg import default_clip
    clip = default_clip(K8)
    sc = torch.from_numpy(scales[sidx])
    q = [torch.round(torch.clamp(_client_vec(k) * sc, -clip, clip)).to(torch.int64).numpy() for k in range(K8)]
    plain = np.sum(q, axis=0)
    assert np.abs(plain).max() > 2 ** 27  # a large share of the int32 range (masked operands: all of it)
    want = unmask(torch.from_numpy(plain.astype(np.int32)), scales, seg_end).numpy()
    for out, sc in res:
        np.testing.assert_array_equal(sc, scales)
        np.testing.assert_array_equal(out, want)  # bit for bit, on every rank
