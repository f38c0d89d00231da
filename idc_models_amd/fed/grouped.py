"""Client-batched local training: a rank's K federated clients advance in lockstep through ONE
grouped program (``runtime/grouped.py``): every kernel launch of a step covers all K clients, each
with its own weights, BatchNorm statistics, RMSprop slots, inputs and labels.

Semantics are exactly those of training the clients one after another on one worker model
(``FedAvgProcess._train_client``, TFF ``fed_model.py:207-229``): every client starts from the
server weights with a fresh client optimizer and fresh statistics shifts, and draws its own
shuffled batches (its dataset's own seed and epoch counter).  Under ``IDC_DETERMINISTIC=1`` the
per-client results are bitwise those of the sequential path (``tests/test_fed_gpu.py``).

Eligibility (else the sequential path runs): fused backend on a GPU, one logit, and client datasets
that are ``BatchedDataset`` s with ``drop_remainder`` and the same batch size and step count.
"""
from __future__ import annotations

import os
from typing import Dict, List, Sequence, Tuple

import torch

from ..runtime.grouped import GroupRegion


def eligible(datasets: Sequence, model) -> bool:
    from ..data.dataset import BatchedDataset
    if model.device.type != "cuda" or getattr(model.impl, "name", "") != "fused":
        return False
    if getattr(model.net, "num_outputs", 1) != 1 or not datasets:
        return False
    if not all(isinstance(d, BatchedDataset) and d.drop_remainder and d.repeat == 1 for d in datasets):
        return False
    # the grouped program takes uint8 pixels (its xin is [K, B, H, W, C] uint8): float or other
    # integer client data would be silently truncated by the index_select copy into it
    if not all(str(getattr(d.ds.x, "dtype", "")) in ("uint8", "torch.uint8") for d in datasets):
        return False
    bs = {d.batch_size for d in datasets}
    steps = {len(d) for d in datasets}
    return len(bs) == 1 and len(steps) == 1 and next(iter(steps)) > 0


class GroupedClientTrainer:
    def __init__(self, model_fn, optimizer_fn, loss, metric_names, k: int, batch: int, device):
        self.k, self.B = int(k), int(batch)
        self.region = GroupRegion(self.k, device)
        with self.region.allocating():
            m = model_fn()
            m.compile(optimizer_fn(), loss, list(metric_names), backend="fused")
            if getattr(m.impl, "name", "") != "fused":
                raise RuntimeError("client batching needs the fused backend")
            m.impl.group = self.region
            H, W, C = m.net.input_shape
            self.prog = m.impl._prog(self.B, True, torch.uint8)
        self.m = m
        self.device = m.device
        p = self.prog
        R = self.region
        self.xin_v = R.view(p.xin)           # [K, B, H, W, C] uint8
        self.lab_v = R.view(p.io.labels)     # [K, B] float32
        self.loss_v = R.view(p.io.loss)      # [K, 1]
        self.logit_v = R.view(p.io.logits)   # [K, B, 1]
        self.threshold = 0.5 if getattr(m, "keras_compat_accuracy", False) else 0.0
        self._data: Dict[int, Tuple[torch.Tensor, torch.Tensor]] = {}
        self._epoch = None  # (rows, X0, Y0): a local epoch's inputs and labels inside the region
        self.ext = R.ext

    def _epoch_buffers(self, rows: int):
        """Copy-0 tensors [rows, H, W, C] uint8 / [rows] fp32 INSIDE the region, so copy g holds
        client g's shuffled epoch and the input op reads step t's batch in place (its pointers
        are shifted per copy like every other; no per-step staging copies).  None if the region
        has no room left (the caller stages through copies)."""
        if self._epoch is not None and self._epoch[0] >= rows:
            return self._epoch
        H, W, C = self.m.net.input_shape
        need = rows * (H * W * C + 4) + (1 << 20)
        if os.environ.get("IDC_GROUP_EPOCH_INPUT", "1") != "1" or self.prog.input_op != self.prog.seg["fwd"][0] \
                or self.region.used + need > self.region.stride:
            return None
        with self.region.allocating():
            X0 = torch.empty((rows, H, W, C), dtype=torch.uint8, device=self.device)
            Y0 = torch.empty((rows,), dtype=torch.float32, device=self.device)
        self._epoch = (rows, X0, Y0)
        return self._epoch

    def _device_data(self, ds):
        """The client's whole example set on the GPU (uploaded once; 288 GB of HBM)."""
        key = id(ds.ds.x)  # client subsets share one backing array: upload it once
        hit = self._data.get(key)
        if hit is None:
            x = torch.as_tensor(ds.ds.x).to(self.device)
            y = torch.as_tensor(ds.ds.y).to(self.device).float().reshape(x.shape[0])
            hit = self._data[key] = (x, y)
        return hit

    def state_views(self):
        """[K, n] views of every copy's flat trainable / non-trainable weights (built once: the
        worker's weights never move, and ~600 views cost ~2.7 ms of host time per round)."""
        if getattr(self, "_views", None) is None:
            R = self.region
            tr = [R.view(t.detach()).reshape(self.k, -1) for t in self.m.net.trainable_weights]
            ntr = [R.view(t.detach()).reshape(self.k, -1) for t in self.m.net.non_trainable_weights]
            self._views = (tr, ntr)
        return self._views

    @torch.no_grad()
    def train(self, load_weights, datasets: Sequence) -> List[tuple]:
        """One local epoch of ``len(datasets) <= K`` clients from the weights ``load_weights(m)``
        writes into the worker model.  Returns, per client, (flat trainable, flat non-trainable,
        example count, last-epoch logs) like ``FedAvgProcess._train_client``."""
        n = len(datasets)
        if n > self.k:
            raise ValueError(f"{n} clients for a group of {self.k}")
        m, p, R = self.m, self.prog, self.region
        B, K = self.B, self.k
        T = len(datasets[0])
        load_weights(m)                      # copy 0: server weights, recast
        m.reset_optimizer()                  # fresh client optimizer (TFF)
        m.impl.reset_stats_shift()
        R.replicate(p.stream)                # every copy starts from copy 0
        cur = torch.cuda.current_stream(self.device)
        H, W, C = m.net.input_shape
        ep = self._epoch_buffers(T * B)
        # replicate() also copies copy 0's epoch buffers (from the second round on they lie in
        # its used part): the per-copy fills below must come after it
        cur.wait_stream(p.stream)
        if ep is not None:
            X, Y = R.view(ep[1]), R.view(ep[2])    # [K, rows, ...] views of the copies
        else:
            X = torch.empty((K, T * B, H, W, C), dtype=torch.uint8, device=self.device)
            Y = torch.empty((K, T * B), dtype=torch.float32, device=self.device)
        orders = [d.epoch_order()[:T * B] for d in datasets]  # each client's own shuffle
        for g in range(K):
            j = g if g < n else 0  # idle copies (fewer clients than copies) recompute client 0
            xd, yd = self._device_data(datasets[j])
            idx = torch.as_tensor(orders[j], device=self.device)
            torch.index_select(xd, 0, idx, out=X[g, :T * B])
            torch.index_select(yd, 0, idx, out=Y[g, :T * B])
        # acc[2g], acc[2g+1]: client g's loss sum and correct count (one group_metrics launch a step)
        acc = torch.zeros(2 * K, dtype=torch.float64, device=self.device)
        io = p.io
        p.stream.wait_stream(cur)
        lo, hi = p.seg["bwd"]
        xrow, op = H * W * C, p.input_op
        with torch.cuda.stream(p.stream):
            sh = p.stream.cuda_stream
            for t in range(T):
                if ep is not None:
                    # the input op reads this step's rows of every copy's epoch in place;
                    # run_segment issues it directly and then restores the program's own xin
                    p.plan.set_ptr(op, 0, ep[1].data_ptr() + t * B * xrow)
                    p.plan.set_ptr(op, 2, ep[2].data_ptr() + t * B * 4)
                    p.plan.set_int(op, 6, 1)
                else:
                    self.xin_v.copy_(X[:, t * B:(t + 1) * B])
                    self.lab_v.copy_(Y[:, t * B:(t + 1) * B])
                p.run_segment("fwd")
                p.run_range(lo, hi)
                p.run_segment("opt")
                self.ext.group_metrics(io.loss.data_ptr(), io.logits.data_ptr(), io.labels.data_ptr(),
                                       R.stride, K, B, float(self.threshold), acc.data_ptr(), sh)
        cur.wait_stream(p.stream)
        err = getattr(p.b, "dense_err", None)
        if err is not None:
            # every copy's persistent-launch error counter (a give-up skipped that client's step)
            tot = int(R.view(err)[:, 0].sum().item())
            if tot > getattr(self, "_err_seen", 0):
                self._err_seen = tot
                from ..runtime.builder import PersistentLaunchError
                raise PersistentLaunchError(f"{tot} persistent dense-stage launch(es) of the grouped client "
                                            "program gave up on a wait")
        tr, ntr = self.state_views()
        flat_tr = torch.cat(tr, 1) if tr else torch.zeros(K, 0, device=self.device)
        flat_ntr = torch.cat(ntr, 1) if ntr else None
        lv, cv = (acc[0::2] / T).tolist(), (acc[1::2] / (T * B)).tolist()
        out = []
        for g in range(n):
            logs = {"loss": lv[g], "accuracy": cv[g]}
            out.append((flat_tr[g].clone(), flat_ntr[g].clone() if flat_ntr is not None else None,
                        float(len(datasets[g].ds)), logs))
        return out
