"""Additive-mask secure aggregation (north-star replacement of the reference's Paillier scheme).

Reference: ``secure_fed_model.py:79,109-168`` — one global Paillier keypair, each client encrypts
the first ``int(n_tensors*percent)`` weight tensors element-wise, the server averages ciphertexts
homomorphically, every client decrypts (quirk Q13: every client can decrypt everything).

Here: each client quantises its weights to fixed point (int32 two's complement,
one power-of-two scale per protected tensor), adds pairwise Philox masks ``+m_ij`` / ``-m_ij`` for
every other participant, and the masked vectors are summed with ONE integer all-reduce (RCCL over
xGMI over ``ncclUint32``: unsigned sums wrap mod 2^32 by definition).  The masks cancel exactly, so the result equals the plain
fixed-point sum BIT-EXACTLY, while any single masked vector is uniformly random.  The pair keys come
from a Diffie-Hellman agreement between the two clients (``keyagree.py``): the aggregator, which
sees only public keys and masked vectors, cannot regenerate any mask.  ``percent`` keeps its
meaning: the fraction of weight tensors that are protected (the rest are averaged in the clear,
as the reference does).

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


def segment_ends(sizes) -> np.ndarray:
    """Exclusive end offsets of consecutive segments (one per protected tensor)."""
    return np.cumsum(np.asarray(list(sizes), dtype=np.int64)).astype(np.int64)


def _seg_index(n: int, seg_end: np.ndarray) -> np.ndarray:
    return np.searchsorted(seg_end, np.arange(n, dtype=np.int64), side="right")


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


def _key_table(nclients: int, keys) -> np.ndarray:
    t = np.zeros(2 * max(nclients, 1), dtype=np.uint32)
    for j, (k0, k1) in (keys or {}).items():
        t[2 * int(j)], t[2 * int(j) + 1] = k0 & MASK32, k1 & MASK32
    return t


def mask_quantize(x: torch.Tensor, scales, seg_end, nclients: int, rank: int, keys, round_: int,
                  clip: float = None, participants=None, out: torch.Tensor = None) -> torch.Tensor:
    """Fixed-point quantise ``x`` (segment s scaled by ``scales[s]``) and add this client's
    pairwise masks -> int32 tensor.  ``out`` (GPU, int32): ADD into it instead (mod 2^32) and
    return it -- a rank's running masked sum over its clients.  ``keys``: {peer client -> (k0, k1)} pair keys of this round
    (``keyagree.ClientKeys.round_keys``).  ``participants``: the clients taking part (default all);
    masks are only exchanged between participants, so a round re-keyed after a dropout still
    cancels exactly."""
    if nclients > 64:
        raise ValueError("secure aggregation supports at most 64 clients per round")
    clip = default_clip(nclients) if clip is None else clip
    alive = _alive_mask(nclients, participants)
    for j in range(nclients):
        if j != rank and (alive >> j) & 1 and j not in (keys or {}):
            raise ValueError(f"no pair key with participant {j}")
    x = x.reshape(-1).contiguous().float()
    n = x.numel()
    scales = np.asarray(scales, dtype=np.float32)
    seg_end = np.asarray(seg_end, dtype=np.int64)
    if n and int(seg_end[-1]) != n:
        raise ValueError("segments do not cover the vector")
    table = _key_table(nclients, keys)
    if x.is_cuda:
        from ..ops import _native as nat
        dev = x.device
        accumulate = out is not None
        if out is None:
            out = torch.empty(n, dtype=torch.int32, device=dev)
        elif out.dtype != torch.int32 or out.numel() != n or out.device != dev:
            raise ValueError("mask_quantize: out must be an int32 tensor of the vector's size on its device")
        sc = torch.from_numpy(scales).to(dev)
        se = torch.from_numpy(seg_end).to(dev)
        kt = torch.from_numpy(table.view(np.int32)).to(dev)
        nat.require().secagg_mask(x.data_ptr(), out.data_ptr(), n, sc.data_ptr(), se.data_ptr(), len(seg_end),
                                  float(clip), int(nclients), int(rank), kt.data_ptr(), int(round_), alive,
                                  nat.stream_handle(), 1 if accumulate else 0)
        # no host sync: the small tables above were allocated on this stream, so the caching
        # allocator hands their memory out again only to work ordered after this kernel
        return out
    sidx = _seg_index(n, seg_end)
    v = torch.clamp(x * torch.from_numpy(scales[sidx]), -clip, clip)
    q = torch.round(v).to(torch.int32).numpy().view(np.uint32).astype(np.uint64)
    idx = np.arange(n, dtype=np.uint64)
    c0 = idx & np.uint64(MASK32)
    c1 = idx >> np.uint64(32)
    acc = q
    for j in range(nclients):
        if j == rank or not (alive >> j) & 1:
            continue
        m = _philox_np(c0, c1, round_ & MASK32, (round_ >> 32) & MASK32, int(table[2 * j]),
                       int(table[2 * j + 1])).astype(np.uint64)
        acc = (acc + m) if rank < j else (acc + (np.uint64(1 << 32) - m))
        acc &= np.uint64(MASK32)
    return torch.from_numpy(acc.astype(np.uint32).view(np.int32).copy())


def unmask(total: torch.Tensor, scales, seg_end, divisor: float = 1.0) -> torch.Tensor:
    """Masked int32 SUM over all participants -> float (sum / divisor), per-segment scale."""
    total = total.reshape(-1).contiguous()
    if total.dtype != torch.int32:
        total = total.view(torch.int32) if total.element_size() == 4 else total.to(torch.int32)
    scales = np.asarray(scales, dtype=np.float32)
    seg_end = np.asarray(seg_end, dtype=np.int64)
    n = total.numel()
    if total.is_cuda:
        from ..ops import _native as nat
        dev = total.device
        out = torch.empty(n, dtype=torch.float32, device=dev)
        sc = torch.from_numpy(scales).to(dev)
        se = torch.from_numpy(seg_end).to(dev)
        nat.require().secagg_unmask(total.data_ptr(), out.data_ptr(), n, sc.data_ptr(), se.data_ptr(),
                                    len(seg_end), float(divisor), nat.stream_handle())
        return out
    sidx = _seg_index(n, seg_end)
    return total.float() / (torch.from_numpy(scales[sidx]) * divisor)


def segment_absmax(vecs, seg_end, nseg: int, dev) -> torch.Tensor:
    """max |x| per segment over all vectors in ``vecs`` (float32 [nseg]); GPU: the native
    ``secagg_absmax`` kernel, one launch per vector."""
    seg_end = np.asarray(seg_end, dtype=np.int64)
    dev = torch.device(dev)
    if not vecs:
        return torch.zeros(nseg, dtype=torch.float32, device=dev)
    if dev.type == "cuda":
        from ..ops import _native as nat
        bits = torch.zeros(nseg, dtype=torch.int32, device=dev)
        se = torch.from_numpy(seg_end).to(dev)
        ext = nat.require()
        for v in vecs:
            v = v.reshape(-1).contiguous()
            if v.numel() != int(seg_end[-1]):
                raise ValueError("segments do not cover the vector")
            ext.secagg_absmax(v.data_ptr(), v.numel(), se.data_ptr(), nseg, bits.data_ptr(), nat.stream_handle())
        return bits.view(torch.float32)
    # CPU: one scatter-amax per vector over the element -> segment index (empty segments stay 0)
    n = int(seg_end[-1]) if len(seg_end) else 0
    seg_of = torch.from_numpy(_seg_index(n, seg_end))
    mx = torch.zeros(nseg, dtype=torch.float32)
    for v in vecs:
        a = v.reshape(-1).float().abs().cpu()
        if a.numel() != n:
            raise ValueError("segments do not cover the vector")
        mx.scatter_reduce_(0, seg_of, a, reduce="amax", include_self=True)
    return mx.to(dev)


def choose_scales(max_abs, nclients: int, headroom: float = 2.0) -> np.ndarray:
    """Per segment: the largest power-of-two scale with K * max|x| * scale < 2^31 (with headroom),
    so each protected tensor keeps the resolution its own range allows."""
    m = np.asarray(max_abs, dtype=np.float64).reshape(-1)
    if not np.isfinite(m).all():
        raise ValueError("non-finite value in a protected tensor")
    pos = m > 0
    with np.errstate(divide="ignore"):
        s = np.where(pos, (2 ** 31 - 1) / (nclients * np.where(pos, m, 1.0) * headroom), 1.0)
    # capped at 2^100: a tiny-but-nonzero segment (|x| < ~1e-29) would otherwise overflow the
    # float32 scale to inf (0*inf = NaN in the kernel, and the decode divides by inf); all-zero
    # segments get 2^16
    e = np.minimum(np.floor(np.log2(np.maximum(s, 1.0))), 100.0)
    return np.where(pos, np.exp2(e), 2.0 ** 16).astype(np.float32)


class MaskedAggregator:
    """Secure SUM over K clients spread over the ranks (one process per GPU).

    Each client owned by this rank holds a Diffie-Hellman key pair (``keyagree.ClientKeys``); the
    public values are exchanged once (the only thing any party learns about another's keys).
    ``masked_sum`` quantises every local client's vector with per-segment scales agreed through a
    MAX all-reduce of the segment ranges, masks it with its pair keys of the round, adds the local
    clients' masked vectors, and combines the ranks with ONE int32 SUM all-reduce — the only
    protected data that crosses a process boundary is masked."""

    def __init__(self, num_clients: int, my_clients, device):
        from ..parallel import comm
        from .keyagree import NBYTES, ClientKeys
        self.K = int(num_clients)
        self.device = torch.device(device)
        self.keys = {int(k): ClientKeys(int(k)) for k in my_clients}
        pub = torch.zeros(self.K, NBYTES, dtype=torch.int64)
        for k, ck in self.keys.items():
            pub[k] = torch.tensor(list(ck.public.to_bytes(NBYTES, "big")), dtype=torch.int64)
        if comm.world_size() > 1:
            pub = pub.to(self.device)
            comm.all_reduce_(pub)  # every client's row is filled by exactly one rank
            pub = pub.cpu()
        self.publics = {k: int.from_bytes(bytes(pub[k].to(torch.uint8).tolist()), "big") for k in range(self.K)}
        self.last_timings = {}

    def masked_sum(self, vecs, sizes, round_: int, participants=None, printer=None) -> torch.Tensor:
        """vecs: {client -> flat float tensor (segments ``sizes``)} for this rank's participating
        clients.  Returns the float SUM over all participating clients (every rank gets it)."""
        import time
        from ..parallel import comm
        from ..utils.timer import Timer
        parts = sorted(int(k) for k in (participants if participants is not None else range(self.K)))
        dev = self.device
        n = int(sum(sizes))
        seg_end = segment_ends(sizes)
        # per-segment |max| over every local client: one native launch per client (not one torch
        # reduction per client and segment: ~600 segments x 8 clients per DenseNet-121 round)
        mx = segment_absmax([v.reshape(-1).to(dev).float() for v in vecs.values()], seg_end, len(sizes), dev)
        if comm.world_size() > 1:
            import torch.distributed as dist
            comm.all_reduce_(mx, op=dist.ReduceOp.MAX)
        scales = choose_scales(mx.cpu().numpy(), self.K)
        gpu = dev.type == "cuda"
        total = torch.zeros(n, dtype=torch.int32 if gpu else torch.int64, device=dev)
        for k, v in sorted(vecs.items()):
            with Timer(f"Encryption for client {k}", printer):
                keys = self.keys[k].round_keys(self.publics, round_, parts)
                if gpu:  # the mask kernel adds into the rank's int32 ring sum (wraps mod 2^32)
                    mask_quantize(v.reshape(-1).to(dev), scales, seg_end, self.K, k, keys, round_,
                                  participants=parts, out=total)
                else:
                    masked = mask_quantize(v.reshape(-1).to(dev), scales, seg_end, self.K, k, keys, round_,
                                           participants=parts)
                    total = (total + masked.to(torch.int64)) % (1 << 32)
        t32 = total if gpu else torch.where(total >= (1 << 31), total - (1 << 32), total).to(torch.int32)
        comm.ring_sum_u32_(t32)  # SUM mod 2^32 (RCCL: one ncclUint32 all-reduce, defined wrap)
        t0 = time.perf_counter()
        out = unmask(t32, scales, seg_end, 1.0).to(dev)
        dt = time.perf_counter() - t0
        if printer is not None:
            for k in sorted(vecs):  # every client runs the same unmasking of the same sum
                printer(f"Decryption for client {k} took {dt} seconds")
        self.last_scales = scales
        return out
