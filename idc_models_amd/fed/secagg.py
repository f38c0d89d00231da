"""Additive-mask secure aggregation (north-star replacement of the reference's Paillier scheme).

Reference: ``secure_fed_model.py:79,109-168`` — one global Paillier keypair, each client encrypts
the first ``int(n_tensors*percent)`` weight tensors element-wise, the server averages ciphertexts
homomorphically, every client decrypts (quirk Q13: every client can decrypt everything).

Here: each client quantises its weights to fixed point (int32 two's complement),
adds pairwise Philox masks ``+m_ij`` / ``-m_ij`` for every other client, and the masked vectors
are summed with ONE integer all-reduce (RCCL over xGMI; uint32/int32 sums wrap mod 2^32).  The
masks cancel exactly, so the result equals the plain fixed-point sum BIT-EXACTLY, while any single
masked vector is uniformly random.  ``percent`` keeps its meaning: the fraction of weight tensors
that are protected (the rest are averaged in the clear, as the reference does).

GPU: native kernel (``csrc/kernels/secagg.hip``).  CPU: the identical Philox in numpy, so both
paths produce the same bits.
"""
from __future__ import annotations

import numpy as np
import torch

M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
MASK32 = 0xFFFFFFFF


def _philox_np(c0, c1, c2, c3, k0, k1):
    c0 = c0.astype(np.uint64)
    c1 = c1.astype(np.uint64)
    c2 = np.full_like(c0, np.uint64(c2 & MASK32))
    c3 = np.full_like(c0, np.uint64(c3 & MASK32))
    k0, k1 = np.uint64(k0 & MASK32), np.uint64(k1 & MASK32)
    m0, m1 = np.uint64(M0), np.uint64(M1)
    for _ in range(10):
        p0 = m0 * c0
        p1 = m1 * c2
        h0, l0 = p0 >> np.uint64(32), p0 & np.uint64(MASK32)
        h1, l1 = p1 >> np.uint64(32), p1 & np.uint64(MASK32)
        c0, c1, c2, c3 = (h1 ^ c1 ^ k0) & np.uint64(MASK32), l1, (h0 ^ c3 ^ k1) & np.uint64(MASK32), l0
        k0 = (k0 + np.uint64(W0)) & np.uint64(MASK32)
        k1 = (k1 + np.uint64(W1)) & np.uint64(MASK32)
    return c0.astype(np.uint32)


def _pair_keys(seed: int, lo: int, hi: int):
    k0 = (seed & MASK32) ^ ((lo * 0x9E3779B1) & MASK32)
    k1 = ((seed >> 32) & MASK32) ^ ((hi * 0x85EBCA77) & MASK32)
    return k0, k1


def _quantize(x: torch.Tensor, scale: float, clip: float) -> torch.Tensor:
    v = torch.clamp(x.float() * scale, -clip, clip)
    return torch.round(v).to(torch.int32)


def default_clip(nclients: int) -> float:
    """Per-client clip so the K-client sum cannot overflow int32."""
    return float((2 ** 31 - 1) // max(nclients, 1))


def _alive_mask(nclients: int, participants) -> int:
    if participants is None:
        return (1 << nclients) - 1
    m = 0
    for j in participants:
        m |= 1 << int(j)
    return m


def mask_quantize(x: torch.Tensor, scale: float, nclients: int, rank: int, seed: int, round_: int,
                  clip: float = None, participants=None) -> torch.Tensor:
    """Fixed-point quantise ``x`` and add this client's pairwise masks -> int32 tensor.

    ``participants``: the clients taking part in this round (default: all).  Masks are only
    exchanged between participants, so when a client drops out before masking the round is
    re-keyed among the survivors and their masks still cancel exactly."""
    if nclients > 64:
        raise ValueError("secure aggregation supports at most 64 clients per round")
    clip = default_clip(nclients) if clip is None else clip
    alive = _alive_mask(nclients, participants)
    x = x.reshape(-1).contiguous().float()
    n = x.numel()
    if x.is_cuda:
        from ..ops import _native as nat
        out = torch.empty(n, dtype=torch.int32, device=x.device)
        nat.require().secagg_mask(x.data_ptr(), out.data_ptr(), n, float(scale), float(clip), int(nclients),
                                  int(rank), int(seed) & ((1 << 64) - 1), int(round_), alive,
                                  nat.stream_handle())
        return out
    q = _quantize(x, scale, clip).numpy().view(np.uint32).astype(np.uint64)
    idx = np.arange(n, dtype=np.uint64)
    c0 = idx & np.uint64(MASK32)
    c1 = idx >> np.uint64(32)
    acc = q
    for j in range(nclients):
        if j == rank or not (alive >> j) & 1:
            continue
        lo, hi = min(j, rank), max(j, rank)
        k0, k1 = _pair_keys(int(seed), lo, hi)
        m = _philox_np(c0, c1, round_ & MASK32, (round_ >> 32) & MASK32, k0, k1).astype(np.uint64)
        acc = (acc + m) if rank == lo else (acc + (np.uint64(1 << 32) - m))
        acc &= np.uint64(MASK32)
    return torch.from_numpy(acc.astype(np.uint32).view(np.int32).copy())


def unmask_mean(total: torch.Tensor, scale: float, nclients: int, divisor: float) -> torch.Tensor:
    """Masked int32 SUM over all clients -> float mean (sum / divisor)."""
    total = total.reshape(-1).contiguous()
    if total.dtype != torch.int32:
        total = total.view(torch.int32) if total.element_size() == 4 else total.to(torch.int32)
    if total.is_cuda:
        from ..ops import _native as nat
        out = torch.empty(total.numel(), dtype=torch.float32, device=total.device)
        nat.require().secagg_unmask(total.data_ptr(), out.data_ptr(), total.numel(), float(scale), int(nclients),
                                    float(divisor), nat.stream_handle())
        return out
    return total.float() / (scale * divisor)


def choose_scale(max_abs: float, nclients: int, headroom: float = 2.0) -> float:
    """Largest power-of-two scale with K * max|x| * scale < 2^31 (with headroom)."""
    if max_abs <= 0:
        return float(2 ** 16)
    s = (2 ** 31 - 1) / (nclients * max_abs * headroom)
    return float(2 ** int(np.floor(np.log2(max(s, 1.0)))))
