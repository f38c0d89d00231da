"""Secure federated learning: the reference's Client/Server loop with protected aggregation.

Reference ``secure_fed_model.py:101-236``:
* every client keeps ITS OWN model and optimizer across rounds (quirk Q15: RMSprop slot state
  persists), trains ``epochs`` local epochs on its 80% split with validation on its 20% split;
* the first ``int(n_tensors * percent)`` weight tensors of ``get_weights()`` (trainable then
  non-trainable, Keras order) are protected, the rest are averaged in the clear;
* the server computes the UNWEIGHTED mean of every tensor over clients; every client sets it;
* client 0 evaluates on the global test set -> (loss, accuracy, AUC).

Protection modes:
* ``"mask"`` (default, north star): fixed-point quantisation (one scale per protected tensor) +
  pairwise Philox masks on the GPU keyed by Diffie-Hellman pair secrets (``keyagree.py``: the
  aggregator sees only public keys and masked vectors), summed with one int32 all-reduce over RCCL
  (wraps mod 2^32, masks cancel exactly);
* ``"paillier"``: the reference's homomorphic scheme (3072-bit keys as ``phe``; GMP, CPU; parity);
* ``"none"``: plain averaging (``percent == 0`` in the reference).

MI355X mapping: clients are spread round-robin over the ranks; a rank holds its clients' states
(flat weights + optimizer slots) and swaps them into ONE compiled model (device memcpy); the
masked/plain sums are single all-reduces.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import torch

from ..parallel import comm
from . import secagg
from .fedavg import assign_clients


@dataclass
class ClientState:
    weights: List[torch.Tensor]       # get_weights() order
    opt_slots: dict


class SecureFederatedProcess:
    def __init__(self, model_fn: Callable, client_data: Sequence[Tuple], percent: float = 0.0,
                 mode: str = "mask", epochs: int = 5, seed: int = 0, paillier_bits: int = 3072,
                 verbose: int = 0, timer_printer=print):
        self.model_fn = model_fn
        self.client_data = list(client_data)
        self.K = len(self.client_data)
        self.percent = float(percent)
        self.mode = mode if self.percent > 0 else "none"
        self.epochs = epochs
        self.seed = seed
        self.round = 0
        self.verbose = verbose
        self.printer = timer_printer
        self.rank, self.world = comm.rank(), comm.world_size()
        self.mine = assign_clients(self.K, self.rank, self.world)
        self.m = model_fn()
        self.states = {}
        init_w = [t.detach().clone() for t in self.m.net.weights]
        # each client starts from its OWN fresh init in the reference (create_model per client)
        for k in self.mine:
            torch.manual_seed(seed * 1000 + k)
            self.m.net.reset_parameters()
            self.states[k] = ClientState([t.detach().clone() for t in self.m.net.weights],
                                         {n: torch.zeros_like(v) for n, v in
                                          self.m.optimizer.state_tensors().items() if v is not None})
        self._set(init_w)
        if self.mode == "paillier":
            from .paillier import generate_paillier_keypair
            self.pub, self.priv = generate_paillier_keypair(paillier_bits)
        elif self.mode == "mask":
            self.agg = secagg.MaskedAggregator(self.K, self.mine, self.m.device)

    # ------------------------------------------------------------------ state swapping
    def _set(self, weights: List[torch.Tensor]):
        with torch.no_grad():
            for t, w in zip(self.m.net.weights, weights):
                t.copy_(w)
        if self.m.impl is not None:
            self.m.impl.sync_from_module()

    def _swap_in(self, k: int):
        st = self.states[k]
        self._set(st.weights)
        for n, v in self.m.optimizer.state_tensors().items():
            if v is not None and n in st.opt_slots:
                v.copy_(st.opt_slots[n])

    def _swap_out(self, k: int):
        if self.m.impl is not None:
            self.m.impl.sync_to_module()
        st = self.states[k]
        st.weights = [t.detach().clone() for t in self.m.net.weights]
        st.opt_slots = {n: v.detach().clone() for n, v in self.m.optimizer.state_tensors().items()
                        if v is not None}

    # ------------------------------------------------------------------ one round
    def client_fit(self, k: int):
        from ..utils.timer import Timer
        train, val = self.client_data[k]
        self._swap_in(k)
        with Timer(f"Training for client {k}", self.printer if self.verbose else None):
            h = self.m.fit(train, epochs=self.epochs, validation_data=val, verbose=0)
        self._swap_out(k)
        return h

    def aggregate(self, dropped=()) -> List[torch.Tensor]:
        """Unweighted mean of every weight tensor over the participating clients
        (secure_fed_model.py:160-168).  ``dropped``: clients that dropped out of this round before
        sending — the mean is over the survivors and the pairwise masks are re-keyed among them
        (the reference has no dropout handling at all)."""
        from ..utils.timer import Timer
        dropped = set(int(k) for k in dropped)
        self.alive = [k for k in range(self.K) if k not in dropped]
        if not self.alive:
            raise RuntimeError("every client dropped out of the round")
        mine = [k for k in self.mine if k not in dropped]
        n_alive = len(self.alive)
        shapes = [w.shape for w in self.states[self.mine[0]].weights] if self.mine else \
            [t.shape for t in self.m.net.weights]
        n_prot = int(len(shapes) * self.percent)
        dev = self.m.device
        prot_sizes = [int(torch.Size(s).numel()) for s in shapes[:n_prot]]
        plain_sizes = [int(torch.Size(s).numel()) for s in shapes[n_prot:]]
        plain_sum = torch.zeros(sum(plain_sizes), device=dev)
        for k in mine:
            ws = self.states[k].weights
            if plain_sizes:
                plain_sum += torch.cat([w.reshape(-1).to(dev) for w in ws[n_prot:]])
        comm.all_reduce_(plain_sum)
        plain_mean = plain_sum / n_alive
        prot_mean = torch.zeros(sum(prot_sizes), device=dev)
        if n_prot:
            with Timer("Secure aggregation", self.printer if self.verbose else None):
                if self.mode == "mask":
                    prot_mean = self._masked_mean(prot_sizes, dev, mine)
                elif self.mode == "paillier":
                    prot_mean = self._paillier_mean(n_prot, dev, mine)
                else:
                    s = torch.zeros(sum(prot_sizes), device=dev)
                    for k in mine:
                        s += torch.cat([w.reshape(-1).to(dev) for w in self.states[k].weights[:n_prot]])
                    comm.all_reduce_(s)
                    prot_mean = s / n_alive
        flat = torch.cat([prot_mean, plain_mean])
        out, off = [], 0
        for s in shapes:
            n = int(torch.Size(s).numel())
            out.append(flat[off:off + n].view(s).clone())
            off += n
        return out

    def _masked_mean(self, prot_sizes, dev, mine) -> torch.Tensor:
        n_prot = len(prot_sizes)
        vecs = {k: torch.cat([w.reshape(-1).to(dev) for w in self.states[k].weights[:n_prot]]) for k in mine}
        s = self.agg.masked_sum(vecs, prot_sizes, self.round, self.alive,
                                printer=self.printer if self.verbose else None)
        return s / float(len(self.alive))

    def _paillier_mean(self, n_prot: int, dev, mine) -> torch.Tensor:
        from ..utils.timer import Timer
        from .paillier import decrypt_vector, encrypt_vector, sum_ciphertexts
        if self.world > 1:
            raise NotImplementedError("Paillier parity mode runs single-process (as the reference)")
        scale = float(2 ** 24)
        pr = self.printer if self.verbose else None
        cts = []
        for k in mine:  # secure_fed_model.py:137: Timer("Encryption for client i")
            with Timer(f"Encryption for client {k}", pr):
                v = torch.cat([w.reshape(-1).float().cpu() for w in self.states[k].weights[:n_prot]])
                cts.append(encrypt_vector(self.pub, v.tolist(), scale))
        summed = sum_ciphertexts(self.pub, cts)
        mean = None
        for k in mine:  # secure_fed_model.py:145: every client decrypts the aggregate
            with Timer(f"Decryption for client {k}", pr):
                mean = decrypt_vector(self.priv, summed, scale, float(len(self.alive)))
        return torch.tensor(mean, dtype=torch.float32, device=dev)

    def run_round(self, test_data=None, dropped=()):
        dropped = set(int(k) for k in dropped)
        for k in self.mine:
            if k not in dropped:
                self.client_fit(k)
        avg = self.aggregate(dropped)
        for k in self.mine:  # every client (a dropped one rejoins next round) takes the new mean
            self.states[k].weights = [w.clone() for w in avg]
        self.round += 1
        if test_data is not None and 0 in self.states:
            self._swap_in(0)
            logs = self.m.evaluate(test_data, return_dict=True)
            return logs
        return None
