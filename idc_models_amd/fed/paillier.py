"""Minimal Paillier cryptosystem (capability parity with ``phe`` used by ``secure_fed_model.py:32,79``).

Only what the reference needs: a keypair, encryption/decryption of (fixed-point) integers, and
homomorphic addition of ciphertexts.  ``phe`` is not installed here, so this is a small pure-Python
implementation on Python's arbitrary-precision ``pow``; when the native GMP module
(``csrc/fed/paillier_gmp.cpp`` -> ``_idc_paillier``) is built, the vector entry points
(``encrypt_vector`` / ``decrypt_vector``) run their modular exponentiations there, on C++ threads,
with CRT decryption.  It is the PARITY mode of secure aggregation (CPU bound); the default mode is
the additive pairwise-mask scheme in ``secagg.py``, which runs on the GPU at HBM bandwidth.
"""
from __future__ import annotations

import importlib
import os
import secrets
from dataclasses import dataclass
from math import gcd
from typing import List, Optional

import numpy as np

_NATIVE = None


def _native():
    global _NATIVE
    if _NATIVE is None:
        _NATIVE = False
        if os.environ.get("IDC_NATIVE_PAILLIER", "1") != "0":
            try:
                from ..utils.hostext import import_host_ext
                _NATIVE = import_host_ext("_idc_paillier")
            except ImportError:
                _NATIVE = False
    return _NATIVE or None


def _threads() -> int:
    return max(1, min(16, os.cpu_count() or 1))


def _be(x: int) -> bytes:
    return x.to_bytes((x.bit_length() + 7) // 8, "big")

_SMALL_PRIMES = [p for p in range(3, 2000, 2) if all(p % q for q in range(3, int(p ** 0.5) + 1, 2))]


def _is_probable_prime(n: int, rounds: int = 40) -> bool:
    if n < 2:
        return False
    for p in _SMALL_PRIMES:
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for _ in range(rounds):
        a = secrets.randbelow(n - 3) + 2
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = pow(x, 2, n)
            if x == n - 1:
                break
        else:
            return False
    return True


def _random_prime(bits: int) -> int:
    while True:
        c = secrets.randbits(bits) | (1 << (bits - 1)) | 1
        if _is_probable_prime(c):
            return c


@dataclass
class PublicKey:
    n: int

    @property
    def n2(self) -> int:
        return self.n * self.n

    def encrypt(self, m: int) -> int:
        n, n2 = self.n, self.n2
        m %= n
        while True:
            r = secrets.randbelow(n - 1) + 1
            if gcd(r, n) == 1:
                break
        # g = n + 1  =>  g^m = 1 + m*n (mod n^2)
        return ((1 + m * n) % n2) * pow(r, n, n2) % n2

    def add(self, c1: int, c2: int) -> int:
        return c1 * c2 % self.n2


@dataclass
class PrivateKey:
    pub: PublicKey
    lam: int
    mu: int
    p: Optional[int] = None  # the factors enable CRT decryption (native path)
    q: Optional[int] = None

    def decrypt(self, c: int) -> int:
        n, n2 = self.pub.n, self.pub.n2
        u = pow(c, self.lam, n2)
        m = ((u - 1) // n) * self.mu % n
        return m - n if m > n // 2 else m  # signed


def generate_paillier_keypair(n_length: int = 3072):
    """Default key length 3072 bits as ``phe`` (the reference's setting)."""
    while True:
        p = _random_prime(n_length // 2)
        q = _random_prime(n_length // 2)
        if p != q:
            break
    n = p * q
    lam = (p - 1) * (q - 1) // gcd(p - 1, q - 1)
    pub = PublicKey(n)
    mu = pow(lam, -1, n)
    return pub, PrivateKey(pub, lam, mu, p, q)


def encrypt_vector(pub: PublicKey, values, scale: float) -> List[int]:
    ms = [int(round(float(v) * scale)) for v in values]
    nat = _native()
    if nat is not None and ms and all(-(1 << 62) < m < (1 << 62) for m in ms):
        blk = nat.encrypt(_be(pub.n), np.asarray(ms, dtype=np.int64), _threads())
        return [int.from_bytes(row.tobytes(), "big") for row in blk]
    return [pub.encrypt(m) for m in ms]


def decrypt_vector(priv: PrivateKey, cts: List[int], scale: float, divisor: float = 1.0) -> List[float]:
    nat = _native()
    if nat is not None and priv.p and priv.q and cts:
        n2 = priv.pub.n2
        w = (n2.bit_length() + 7) // 8
        blk = np.frombuffer(b"".join(c.to_bytes(w, "big") for c in cts), dtype=np.uint8).reshape(len(cts), w)
        try:
            ms = nat.decrypt(_be(priv.p), _be(priv.q), blk, _threads())
            return [float(m) / scale / divisor for m in ms.tolist()]
        except OverflowError:
            pass  # plaintext beyond int64: exact Python path below
    return [priv.decrypt(c) / scale / divisor for c in cts]


def native_powm(base: int, exp: int, mod: int) -> int:
    """base^exp mod mod on GMP (the Diffie-Hellman key agreement of fed/keyagree.py)."""
    nat = _native()
    if nat is None or not hasattr(nat, "powm"):
        raise ImportError("native GMP module not built")
    return int.from_bytes(nat.powm(_be(base % mod) or b"\0", _be(exp) or b"\0", _be(mod)), "big")


def sum_ciphertexts(pub: PublicKey, vectors: List[List[int]]) -> List[int]:
    out = list(vectors[0])
    for v in vectors[1:]:
        out = [pub.add(a, b) for a, b in zip(out, v)]
    return out
