"""Federated averaging with TFF semantics, simulated over the GPUs of one node.

Reference: ``fed_model.py:196-229`` — ``tff.learning.build_federated_averaging_process(model_fn,
client_optimizer_fn=RMSprop(1e-4))`` + ``build_federated_evaluation``; 10 clients, 8 train / 2 test.
TFF 0.12 semantics reproduced:

* the server broadcasts its model; each client starts from it with a FRESH client optimizer,
  trains one local epoch over its dataset, and reports the delta of its TRAINABLE weights with
  weight = number of examples (a client whose delta is non-finite gets weight 0);
* the server applies the example-weighted mean delta with SGD(lr=1.0) (``server_optimizer_fn``);
* non-trainable weights (BN moving statistics) are not aggregated, unless
  ``average_bn_stats=True`` (documented deviation for BN backbones);
* metrics are example-weighted sums across clients, reported as OrderedDict(binary_accuracy, loss).

MI355X mapping: clients are assigned round-robin to ranks (one process per GPU);
each rank trains its clients back to back on ONE compiled model (the client's weights/optimizer
state are swapped into the flat arena — a device memcpy, no re-lowering); the per-rank partial
``[sum n_k*delta_k | sum n_k | metric sums]`` is combined with ONE packed all-reduce over RCCL.

``secure_aggregation="mask"`` (north-star config #5, secure FedAvg): each client's example-weighted
delta ``n_k * delta_k`` is quantised (one fixed-point scale per tensor) and masked with pairwise
Diffie-Hellman-keyed Philox masks (``secagg.MaskedAggregator``); the masks cancel in the int32
all-reduce, so the server learns only ``sum_k n_k * delta_k`` (example counts and metric sums stay
in the clear, as TFF reports them).  A client whose update is non-finite still takes part in the
masking with a zero vector and weight 0, so its peers' masks cancel.
"""
from __future__ import annotations

import collections
import os
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence

import torch

from ..parallel import comm


@dataclass
class ModelWeights:
    trainable: List[torch.Tensor]
    non_trainable: List[torch.Tensor]

    def clone(self):
        return ModelWeights([t.clone() for t in self.trainable], [t.clone() for t in self.non_trainable])


@dataclass
class ServerState:
    model: ModelWeights
    round_num: int = 0
    optimizer_state: dict = field(default_factory=dict)


def state_with_new_model_weights(state: ServerState, trainable_weights, non_trainable_weights) -> ServerState:
    """``tff.learning.state_with_new_model_weights`` (``fed_model.py:219-223``)."""
    dev = state.model.trainable[0].device if state.model.trainable else "cpu"
    tw = [torch.as_tensor(w, dtype=torch.float32).to(dev) for w in trainable_weights]
    nw = [torch.as_tensor(w, dtype=torch.float32).to(dev) for w in non_trainable_weights]
    for a, b in zip(tw, state.model.trainable):
        if a.shape != b.shape:
            raise ValueError("trainable weight shape mismatch")
    return ServerState(ModelWeights(tw, nw), state.round_num, state.optimizer_state)


def broadcast_server_state(state: ServerState, src: int = 0) -> ServerState:
    """Make every rank's server state rank ``src``'s (one process per GPU: the server model must
    be identical everywhere before clients start from it)."""
    if comm.world_size() > 1:
        for t in list(state.model.trainable) + list(state.model.non_trainable):
            comm.broadcast_(t, src)
        rn = torch.tensor([state.round_num], dtype=torch.int64,
                          device=state.model.trainable[0].device if state.model.trainable else "cpu")
        comm.broadcast_(rn, src)
        state.round_num = int(rn.item())
    return state


def save_server_state(state: ServerState, path: str, extra: Optional[dict] = None) -> None:
    """Federated resume point (SURVEY §5 checkpoint/resume): server model, round counter, server
    optimizer state and the host RNG; written to a temporary file and renamed into place."""
    import os
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    blob = {"trainable": [t.detach().cpu() for t in state.model.trainable],
            "non_trainable": [t.detach().cpu() for t in state.model.non_trainable],
            "round_num": int(state.round_num),
            "optimizer_state": {k: v.detach().cpu() for k, v in state.optimizer_state.items()
                                if isinstance(v, torch.Tensor)},
            "rng_cpu": torch.get_rng_state(),
            "extra": {k: v for k, v in (extra or {}).items() if isinstance(v, (int, float, str, bool))}}
    tmp = f"{path}.tmp"
    torch.save(blob, tmp)
    os.replace(tmp, path)


def load_server_extra(path: str) -> dict:
    """The ``extra`` dict saved with a server state (config fingerprint), without loading it."""
    blob = torch.load(path, map_location="cpu", weights_only=True)
    return dict(blob.get("extra", {}))


def load_server_state(path: str, device=None) -> ServerState:
    blob = torch.load(path, map_location="cpu", weights_only=True)
    dev = torch.device(device) if device is not None else torch.device("cpu")
    state = ServerState(ModelWeights([t.to(dev) for t in blob["trainable"]],
                                     [t.to(dev) for t in blob["non_trainable"]]),
                        int(blob["round_num"]), {k: v.to(dev) for k, v in blob.get("optimizer_state", {}).items()})
    if "rng_cpu" in blob:
        torch.set_rng_state(blob["rng_cpu"])
    return state


def assign_clients(num_clients: int, rank: int, world: int) -> List[int]:
    """ClientScheduler: client k -> rank k % world (8 train clients <-> 8 GPUs)."""
    return [k for k in range(num_clients) if k % world == rank]


class FedAvgProcess:
    def __init__(self, model_fn: Callable, client_optimizer_fn: Callable,
                 server_optimizer_fn: Optional[Callable] = None, average_bn_stats: bool = False,
                 local_epochs: int = 1, loss="binary_crossentropy", metrics=("binary_accuracy",),
                 secure_aggregation: Optional[str] = None, backend: str = "auto",
                 concurrent_clients: int = 1, client_batching: Optional[bool] = None):
        self.model_fn = model_fn
        # client batching (fed/grouped.py): a rank's clients advance in lockstep through ONE
        # grouped program, every launch covering all of them (default on, IDC_CLIENT_BATCHING=0
        # or client_batching=False: one client at a time / `concurrent_clients` worker threads)
        if client_batching is None:
            client_batching = os.environ.get("IDC_CLIENT_BATCHING", "1") != "0"
        self.client_batching = bool(client_batching)
        self._grouped = None
        # ClientScheduler: a rank trains up to `concurrent_clients` of its clients at
        # once, each on its own worker model and HIP stream (small-batch client steps leave most
        # of an MI355X idle); aggregation still runs in client order
        self.concurrent = max(1, int(concurrent_clients))
        self._more_workers = []
        self.client_optimizer_fn = client_optimizer_fn
        self.server_lr = 1.0
        if server_optimizer_fn is not None:
            opt = server_optimizer_fn()
            self.server_lr = float(getattr(opt, "learning_rate", 1.0))
        self.average_bn_stats = average_bn_stats
        self.local_epochs = local_epochs
        self.loss = loss
        self.metric_names = list(metrics)
        self._worker = None
        if secure_aggregation not in (None, "none", "mask"):
            raise ValueError(f"unknown secure aggregation mode {secure_aggregation!r}")
        self.secure = secure_aggregation == "mask"
        self._agg = None
        self.backend = backend

    # -------------------------------------------------------------- worker model
    def worker(self):
        if self._worker is None:
            m = self.model_fn()
            m.compile(self.client_optimizer_fn(), self.loss, list(self.metric_names), backend=self.backend)
            self._worker = m
        return self._worker

    def workers(self, n: int):
        """``n`` worker models: the primary one plus independently built copies.  With n > 1 they
        run concurrently on one device: their programs must not use a persistent launch order that
        assumes the device to itself (Builder.shared_device)."""
        while len(self._more_workers) < n - 1:
            m = self.model_fn()
            m.compile(self.client_optimizer_fn(), self.loss, list(self.metric_names), backend=self.backend)
            self._more_workers.append(m)
        ws = [self.worker()] + self._more_workers[:n - 1]
        if n > 1:
            for m in ws:
                impl = m.impl
                if impl is not None and not getattr(impl, "shared_device", False):
                    impl.shared_device = True
                    if getattr(impl, "progs", None):  # built for exclusive use: rebuild
                        impl.sync_to_module()
                        impl.close()
        return ws

    def _train_client(self, m, state: "ServerState", ds):
        """Local training of one client from the server weights: returns its flat trainable
        weights, flat non-trainable weights, example count and last-epoch logs."""
        self._load(m, state.model)
        m.reset_optimizer()
        if hasattr(m.impl, "reset_stats_shift"):
            m.impl.reset_stats_shift()
        h = m.fit(ds, epochs=self.local_epochs, verbose=0)
        n_k = float(len(ds.ds) if hasattr(ds, "ds") else len(ds))
        m.impl.sync_to_module()
        tr, ntr = self._tensors(m)
        flat = torch.cat([t.detach().reshape(-1) for t in tr])
        flat_ntr = torch.cat([t.detach().reshape(-1) for t in ntr]) if ntr else None
        return flat, flat_ntr, n_k, {k2: v[-1] for k2, v in h.history.items()}

    def _grouped_trainer(self, n_clients: int, batch: int):
        from .grouped import GroupedClientTrainer
        g = self._grouped
        if g is None or g.k < n_clients or g.B != batch:
            # a region stays reserved for the whole process (runtime/grouped.py _KEEP_ALIVE): the
            # old one stops allocating and the re-creation is reported (idle copies cost compute,
            # so the group is not over-sized speculatively; it only grows, never shrinks for a
            # smaller round)
            k = n_clients if g is None else max(n_clients, g.k)
            if g is not None:
                g.region.close()
                import warnings
                warnings.warn(f"client batching: re-creating the grouped trainer (K {g.k}->{k}, batch "
                              f"{g.B}->{batch}); the old {g.k} x {g.region.stride >> 20} MiB region stays reserved")
            m = self.worker()
            g = GroupedClientTrainer(self.model_fn, self.client_optimizer_fn, self.loss, self.metric_names,
                                     k, batch, m.device)
            self._grouped = g
        return g

    def _train_clients(self, mine, state, data):
        """Train this rank's clients: all at once through one grouped program (client batching),
        sequentially, or `concurrent` at a time on worker threads, each with its own model and
        current HIP stream (torch's current stream is per thread, so the clients' staging, metrics
        and kernels never order each other)."""
        if self.client_batching and len(mine) > 0 and self.local_epochs == 1:
            from .grouped import eligible
            from ..runtime.builder import PersistentLaunchError, disable_persistent
            sets = [data[k] for k in mine]
            if eligible(sets, self.worker()):
                g = self._grouped_trainer(len(mine), sets[0].batch_size)
                try:
                    res = g.train(lambda m: self._load(m, state.model), sets)
                    return dict(zip(mine, res))
                except PersistentLaunchError as e:
                    # a client copy's persistent launch gave up: its skipped steps make the round
                    # wrong, so the round is re-run on a grouped program without persistent
                    # launches (IDC_DS_ON_FAIL=raise: propagate)
                    if os.environ.get("IDC_DS_ON_FAIL", "fallback") == "raise":
                        raise
                    disable_persistent(str(e))
                    g.region.close()
                    self._grouped = None
                    g = self._grouped_trainer(len(mine), sets[0].batch_size)
                    res = g.train(lambda m: self._load(m, state.model), sets)
                    return dict(zip(mine, res))
        W = min(self.concurrent, len(mine))
        if W <= 1 or not torch.cuda.is_available() or self.worker().device.type != "cuda":
            return {k: self._train_client(self.worker(), state, data[k]) for k in mine}
        import threading
        models = self.workers(W)
        dev = models[0].device
        out, errs = {}, []

        def run(w):
            try:
                with torch.cuda.device(dev):
                    s = torch.cuda.Stream(dev)
                    s.wait_stream(torch.cuda.default_stream(dev))
                    with torch.cuda.stream(s):
                        for k in mine[w::W]:
                            out[k] = self._train_client(models[w], state, data[k])
                    s.synchronize()
            except BaseException as e:  # surfaced on the calling thread
                errs.append(e)

        # a worker whose program is not built yet builds (and autotunes) it on this thread, one
        # worker at a time, with its first client: tile timings taken while another client's
        # kernels share the GPU would be picked under contention
        queues = [list(mine[w::W]) for w in range(W)]
        for w in range(W):
            if queues[w] and not getattr(models[w].impl, "progs", {1: 1}):
                k = queues[w].pop(0)
                out[k] = self._train_client(models[w], state, data[k])

        def run_queue(w):
            try:
                with torch.cuda.device(dev):
                    s = torch.cuda.Stream(dev)
                    s.wait_stream(torch.cuda.default_stream(dev))
                    with torch.cuda.stream(s):
                        for k in queues[w]:
                            out[k] = self._train_client(models[w], state, data[k])
                    s.synchronize()
            except BaseException as e:  # surfaced on the calling thread
                errs.append(e)
        run = run_queue

        torch.cuda.current_stream(dev).synchronize()  # server weights final before the workers read
        threads = [threading.Thread(target=run, args=(w,), daemon=True) for w in range(W)]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if errs:
            raise errs[0]
        return out

    def _tensors(self, m):
        tr = [p for p in m.net.trainable_weights]
        ntr = [t for t in m.net.non_trainable_weights]
        return tr, ntr

    def initialize(self) -> ServerState:
        m = self.worker()
        tr, ntr = self._tensors(m)
        state = ServerState(ModelWeights([t.detach().clone() for t in tr], [t.detach().clone() for t in ntr]))
        return broadcast_server_state(state)

    def _load(self, m, weights: ModelWeights):
        _load_into(m, weights)

    # -------------------------------------------------------------- round
    def next(self, state: ServerState, federated_train_data: Sequence, participating=None):
        """One round.  ``participating``: indices of the clients that report this round (default
        all) — absent clients simply carry no weight, as in TFF's sampled rounds."""
        m = self.worker()
        rank, world = comm.rank(), comm.world_size()
        K = len(federated_train_data)
        mine = assign_clients(K, rank, world)
        parts = sorted(int(k) for k in participating) if participating is not None else list(range(K))
        keep = set(parts)
        mine = [k for k in mine if k in keep]
        masked = {}  # secure mode: client -> n_k * [delta | bn stats]
        dev = state.model.trainable[0].device if state.model.trainable else m.device
        flat_server = torch.cat([w.reshape(-1) for w in state.model.trainable]).to(m.device)
        delta_sum = torch.zeros_like(flat_server)
        ntr_sum = None
        if self.average_bn_stats and state.model.non_trainable:
            ntr_sum = torch.zeros(sum(w.numel() for w in state.model.non_trainable), device=m.device)
        n_sum = torch.zeros(1, device=m.device, dtype=torch.float64)
        met = torch.zeros(1 + len(self.metric_names), device=m.device, dtype=torch.float64)
        results = self._train_clients(mine, state, federated_train_data)
        for k in mine:  # aggregation in client order, however the clients were scheduled
            flat, flat_ntr, n_k, logs = results[k]
            delta = flat - flat_server
            # TFF gives a client weight 0 when its update is non-finite; the BatchNorm statistics
            # that get averaged too (average_bn_stats) must be finite as well, or they would poison
            # the mean (plain) or the masked segment ranges (secure).  The decision stays on the
            # device (a 0/1 weight, NaNs replaced by where()): no host sync per client -- the round
            # reads its totals once, after the all-reduce
            fin = torch.isfinite(delta).all()
            if flat_ntr is not None and ntr_sum is not None:
                fin = fin & torch.isfinite(flat_ntr).all()
            w = fin.to(torch.float64)
            zero = delta.new_zeros(())
            if self.secure:
                v = [n_k * delta] + ([n_k * flat_ntr] if ntr_sum is not None else [])
                masked[k] = torch.where(fin, torch.cat(v), zero)
            else:
                delta_sum += torch.where(fin, n_k * delta, zero)
                if ntr_sum is not None:
                    ntr_sum += torch.where(fin, n_k * flat_ntr, zero)
            n_sum += n_k * w
            # a diverged client's metrics are usually non-finite too (NaN * 0 = NaN): select, not
            # multiply, so its loss never reaches the round's metrics
            zero64 = met.new_zeros(())
            met[0] += torch.where(fin, torch.as_tensor(n_k * logs.get("loss", 0.0), dtype=met.dtype,
                                                       device=met.device), zero64)
            for i, name in enumerate(self.metric_names):
                v = logs.get(name if name in logs else "accuracy", 0.0)
                met[1 + i] += torch.where(fin, torch.as_tensor(n_k * v, dtype=met.dtype, device=met.device), zero64)
        if self.secure:
            # the weighted deltas cross ranks only masked; counts and metrics in the clear
            if self._agg is None or self._agg.K != K:
                from .secagg import MaskedAggregator
                self._agg = MaskedAggregator(K, assign_clients(K, rank, world), m.device)
            sizes = [w.numel() for w in state.model.trainable]
            if ntr_sum is not None:
                sizes += [w.numel() for w in state.model.non_trainable]
            s = self._agg.masked_sum(masked, sizes, state.round_num, parts)
            delta_sum.copy_(s[:delta_sum.numel()])
            if ntr_sum is not None:
                ntr_sum.copy_(s[delta_sum.numel():])
            clear = [n_sum, met]
        else:
            clear = [delta_sum, n_sum, met] + ([ntr_sum] if ntr_sum is not None else [])
        # packed all-reduces of [delta sums | bn sums] and [n | metrics] (clear parts), one per
        # dtype: the float64 example counts and metric sums stay exact across ranks
        if world > 1:
            comm.all_reduce_packed_(clear)
        total = float(n_sum.item())
        if total > 0:
            mean_delta = delta_sum / total
            new_flat = flat_server + self.server_lr * mean_delta
        else:
            new_flat = flat_server
        # the new server weights are VIEWS of one fresh flat buffer each (trainable / statistics):
        # a per-tensor clone was ~600 copy launches per DenseNet-121 round
        new_flat = new_flat.to(dev)
        tr_w = state.model.trainable
        new_tr = [t.view(w.shape) for t, w in zip(new_flat.split([w.numel() for w in tr_w]), tr_w)]
        if ntr_sum is not None and total > 0:
            flat_ntr_new = (ntr_sum / total).to(dev)
        else:
            flat_ntr_new = torch.cat([w.reshape(-1) for w in state.model.non_trainable]) \
                if state.model.non_trainable else None
        ntr_w = state.model.non_trainable
        new_ntr = [t.view(w.shape).to(w.dtype)
                   for t, w in zip(flat_ntr_new.split([w.numel() for w in ntr_w]), ntr_w)] if ntr_w else []
        metrics = collections.OrderedDict()
        for i, name in enumerate(self.metric_names):
            metrics[name] = float(met[1 + i].item() / total) if total else 0.0
        metrics["loss"] = float(met[0].item() / total) if total else 0.0
        return ServerState(ModelWeights(new_tr, new_ntr), state.round_num + 1, state.optimizer_state), metrics


def build_federated_averaging_process(model_fn, client_optimizer_fn, server_optimizer_fn=None, **kw):
    """``tff.learning.build_federated_averaging_process`` equivalent."""
    return FedAvgProcess(model_fn, client_optimizer_fn, server_optimizer_fn, **kw)


class FederatedEvaluation:
    """``tff.learning.build_federated_evaluation``: example-weighted metrics over test clients."""

    def __init__(self, model_fn: Callable, loss="binary_crossentropy", metrics=("binary_accuracy",)):
        self.model_fn = model_fn
        self.loss = loss
        self.metric_names = list(metrics)
        self._m = None

    def __call__(self, model_weights: ModelWeights, federated_test_data: Sequence):
        from ..engine.optimizers import SGD
        if self._m is None:
            self._m = self.model_fn()
            self._m.compile(SGD(0.0), self.loss, list(self.metric_names))
        m = self._m
        _load_into(m, model_weights)
        rank, world = comm.rank(), comm.world_size()
        mine = assign_clients(len(federated_test_data), rank, world)
        acc = torch.zeros(2 + len(self.metric_names), dtype=torch.float64, device=m.device)
        for k in mine:
            ds = federated_test_data[k]
            logs = m.evaluate(ds, return_dict=True)
            n_k = float(len(ds.ds) if hasattr(ds, "ds") else len(ds))
            acc[0] += n_k
            acc[1] += n_k * logs["loss"]
            for i, name in enumerate(self.metric_names):
                acc[2 + i] += n_k * logs.get(name if name in logs else "accuracy", 0.0)
        if world > 1:
            a32 = acc.float()
            comm.all_reduce_(a32)
            acc = a32.double()
        n = float(acc[0].item())
        out = collections.OrderedDict()
        for i, name in enumerate(self.metric_names):
            out[name] = float(acc[2 + i].item() / n) if n else 0.0
        out["loss"] = float(acc[1].item() / n) if n else 0.0
        return out


def _load_into(m, weights: ModelWeights):
    tr = list(m.net.trainable_weights)
    ntr = list(m.net.non_trainable_weights)
    with torch.no_grad():
        # multi-tensor copies (a handful of launches instead of one per tensor: ~600 for DenseNet)
        pairs = list(zip(tr, weights.trainable)) + list(zip(ntr, weights.non_trainable))
        dst = [t for t, _ in pairs]
        src = [w.to(t.device, t.dtype) for t, w in pairs]
        if hasattr(torch, "_foreach_copy_"):
            torch._foreach_copy_(dst, src)
        else:  # pragma: no cover - older torch
            for t, w in zip(dst, src):
                t.copy_(w)
    if m.impl is not None:
        m.impl.sync_from_module()


def build_federated_evaluation(model_fn, **kw):
    return FederatedEvaluation(model_fn, **kw)
