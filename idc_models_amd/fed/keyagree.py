"""Pairwise secrets for additive-mask secure aggregation: finite-field Diffie-Hellman.

The reference keeps key material away from the aggregator: every client holds the Paillier
private key and the server only ever sees ciphertexts (``secure_fed_model.py:79,109-129``).  The
mask-based replacement needs the same property: the masks that client i adds for the pair (i, j)
must be reproducible by i and j only.  Each client therefore owns a private exponent ``a_i`` and
publishes ``A_i = g^a_i mod p`` over the RFC 3526 2048-bit MODP group (group 14, g = 2; p is a safe
prime and g generates its subgroup of prime order q = (p-1)/2).  The pair secret is
``S_ij = A_j^a_i = A_i^a_j mod p``; the Philox mask key of the pair for a round is
``SHA-256(S_ij || round || i || j)``.  The aggregator's view — the public values and the masked
vectors — determines no mask (computational Diffie-Hellman), while the masks of every pair still
cancel exactly in the sum.

Modular exponentiation runs on GMP (the Paillier extension, ``csrc/fed/paillier_gmp.cpp``) when it
is built, else on Python integers.
"""
from __future__ import annotations

import hashlib
import secrets
from dataclasses import dataclass
from typing import Dict, Tuple

P = int(
    "FFFFFFFFFFFFFFFFC90FDAA22168C234C4C6628B80DC1CD129024E088A67CC74020BBEA63B139B22514A08798E3404DD"
    "EF9519B3CD3A431B302B0A6DF25F14374FE1356D6D51C245E485B576625E7EC6F44C42E9A637ED6B0BFF5CB6F406B7ED"
    "EE386BFB5A899FA5AE9F24117C4B1FE649286651ECE45B3DC2007CB8A163BF0598DA48361C55D39A69163FA8FD24CF5F"
    "83655D23DCA3AD961C62F356208552BB9ED529077096966D670C354E4ABC9804F1746C08CA18217C32905E462E36CE3B"
    "E39E772C180E86039B2783A2EC07A28FB5C55DF06F4C52C9DE2BCBF6955817183995497CEA956AE515D2261898FA0510"
    "15728E5A8AACAA68FFFFFFFFFFFFFFFF", 16)
G = 2
Q = (P - 1) // 2
NBYTES = (P.bit_length() + 7) // 8
PRIV_BITS = 256  # >= 2x the 112-bit security level of a 2048-bit group


def _powm(base: int, exp: int, mod: int) -> int:
    try:
        from .paillier import native_powm
        return native_powm(base, exp, mod)
    except (ImportError, AttributeError):
        return pow(base, exp, mod)


@dataclass
class DHKeyPair:
    private: int
    public: int

    @classmethod
    def generate(cls) -> "DHKeyPair":
        a = secrets.randbelow(1 << PRIV_BITS) | (1 << (PRIV_BITS - 1))  # full-length exponent
        return cls(a, _powm(G, a, P))


def check_public(pub: int) -> int:
    """Reject public values outside the prime-order subgroup (small-subgroup / degenerate keys)."""
    if not (2 <= pub <= P - 2) or _powm(pub, Q, P) != 1:
        raise ValueError("invalid Diffie-Hellman public value")
    return pub


def shared_secret(mine: DHKeyPair, peer_public: int) -> int:
    return _powm(check_public(peer_public), mine.private, P)


def pair_mask_key(secret: int, round_: int, i: int, j: int) -> Tuple[int, int]:
    """(k0, k1) Philox key of the unordered pair {i, j} for ``round_``."""
    lo, hi = min(i, j), max(i, j)
    h = hashlib.sha256(secret.to_bytes(NBYTES, "big") + round_.to_bytes(8, "big") + lo.to_bytes(4, "big")
                       + hi.to_bytes(4, "big")).digest()
    return int.from_bytes(h[:4], "little"), int.from_bytes(h[4:8], "little")


class ClientKeys:
    """One client's key pair and its cached pair secrets with the other clients."""

    def __init__(self, client: int):
        self.client = client
        self.pair = DHKeyPair.generate()
        self._secrets: Dict[int, Tuple[int, int]] = {}

    @property
    def public(self) -> int:
        return self.pair.public

    def round_keys(self, publics: Dict[int, int], round_: int, participants) -> Dict[int, Tuple[int, int]]:
        """Philox keys for every other participant (client index -> (k0, k1))."""
        out = {}
        for j in participants:
            j = int(j)
            if j == self.client:
                continue
            pub = publics[j]
            cached = self._secrets.get(j)
            if cached is None or cached[0] != pub:
                cached = (pub, shared_secret(self.pair, pub))
                self._secrets[j] = cached
            out[j] = pair_mask_key(cached[1], round_, self.client, j)
        return out
