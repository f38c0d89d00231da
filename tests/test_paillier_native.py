"""Native GMP Paillier (csrc/fed/paillier_gmp.cpp) vs the pure-Python reference implementation."""
import numpy as np
import pytest

from idc_models_amd.fed import paillier as P

pytestmark = pytest.mark.skipif(P._native() is None, reason="_idc_paillier not built")


@pytest.fixture(scope="module")
def keys():
    return P.generate_paillier_keypair(512)


def test_native_encrypt_decrypts_with_python_and_vice_versa(keys):
    pub, priv = keys
    vals = [0.0, 1.5, -2.25, 1e-3, -7.0, 123.456]
    cts = P.encrypt_vector(pub, vals, 2 ** 16)          # native encryption
    py_dec = [priv.decrypt(c) / 2 ** 16 for c in cts]   # pure-Python decryption
    np.testing.assert_allclose(py_dec, vals, atol=2 ** -16)
    cts_py = [pub.encrypt(int(round(v * 2 ** 16))) for v in vals]
    np.testing.assert_allclose(P.decrypt_vector(priv, cts_py, 2 ** 16), vals, atol=2 ** -16)


def test_native_homomorphic_mean_is_exact(keys):
    pub, priv = keys
    rng = np.random.default_rng(0)
    clients = [rng.normal(size=64) for _ in range(3)]
    scale = 2.0 ** 24
    enc = [P.encrypt_vector(pub, c, scale) for c in clients]
    summed = P.sum_ciphertexts(pub, enc)
    mean = P.decrypt_vector(priv, summed, scale, 3.0)
    exact = sum(np.round(c * scale) for c in clients) / scale / 3.0
    np.testing.assert_array_equal(np.asarray(mean), exact)


def test_native_add_block(keys):
    pub, priv = keys
    nat = P._native()
    a = nat.encrypt(P._be(pub.n), np.array([5, -9, 100], np.int64), 2)
    b = nat.encrypt(P._be(pub.n), np.array([-5, 4, 1], np.int64), 2)
    s = nat.add(P._be(pub.n), a, b)
    out = nat.decrypt(P._be(priv.p), P._be(priv.q), s, 2)
    assert out.tolist() == [0, -5, 101]


def test_ciphertexts_are_randomised(keys):
    pub, _ = keys
    c = P.encrypt_vector(pub, [1.0, 1.0], 1.0)
    assert c[0] != c[1]
