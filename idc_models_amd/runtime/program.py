"""A lowered, executable training/eval program and the ``fused`` Model backend.

``FusedProgram`` = one static plan for (model, batch, training, input dtype):
  segment ``fwd``  input staging -> convs/pools (fused BN/act) -> head loss -> BN moving update
  segment ``bwd``  grad-arena memset -> head bwd -> dgrad/wgrad/BN-bwd in reverse order
  segment ``opt``  fused RMSprop over the flat arena -> bf16 weight re-cast (ONE launch each)
Each segment is captured into a HIP graph on first use and replayed afterwards.  Under data
parallelism the backward segment is split at bucket boundaries so each bucket's RCCL all-reduce
is launched while the remaining backward segments run.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import torch

from ..engine.losses import BinaryCrossentropy, CategoricalCrossentropy, SparseCategoricalCrossentropy
from ..engine.optimizers import RMSprop
from ..ops import _native as nat
from ..utils import trace
from .builder import Builder


def _lowering_for(net):
    from ..models import Sequential
    from ..models.densenet import DenseNet
    from ..models.mobilenet_v2 import MobileNetV2
    from ..models.vgg import VGG16

    from ..models.tiny_cnn import TinyCNN
    if isinstance(net, TinyCNN):
        from .lower_tiny import lower_tiny, tiny_supported
        return lower_tiny if tiny_supported(net) else None
    if not isinstance(net, Sequential):
        return None
    base = net.base
    if isinstance(base, DenseNet):
        from .lower_densenet import lower_densenet
        return lower_densenet
    if isinstance(base, VGG16):
        from .lower_vgg import lower_vgg
        return lower_vgg
    if isinstance(base, MobileNetV2):
        from .lower_mobilenet import lower_mobilenet
        return lower_mobilenet
    return None


def fused_supported(net, loss) -> bool:
    if _lowering_for(net) is None:
        return False
    if not isinstance(loss, (BinaryCrossentropy, CategoricalCrossentropy, SparseCategoricalCrossentropy)):
        return False
    if not getattr(loss, "from_logits", True):
        return False
    if net.num_outputs > 16:
        return False
    return nat.available()


def persistent_allowed(model, training: bool) -> bool:
    """Whether a program may build persistent (work-queue) launches.  A persistent launch that
    gives up leaves stale stage outputs and relies on the step's update being skipped through the
    step guard word: only the fused RMSprop reads that word (a host optimizer would apply the stale
    update), and only the native communicator's guard all-reduce makes every replica skip
    together (the torch bucketer path and central storage would let the other replicas apply
    gradients that include the stale contribution).  Evaluation programs are unaffected."""
    if not training or not model.arena.params:
        return True
    opt = model.optimizer
    host_opt = not isinstance(opt, RMSprop) or bool(opt.momentum) or bool(opt.centered)
    st = model.strategy
    unguarded_dp = st.active and (getattr(st, "native_comm", None) is None
                                  or getattr(st, "central_storage", False))
    return not (host_opt or unguarded_dp)


def place_buckets(ops, bwd_marks, buckets) -> Dict[int, List[Tuple[int, int]]]:
    """Where each gradient bucket's all-reduce goes in a lowered op list: ``{i: [(start, end)]}``
    = the buckets issued right before ``ops[i]`` (``i`` may be the first op after the backward
    segment, or ``len(ops)``, for buckets no mark released).

    ``bwd_marks``: ``(op index, lowest arena parameter index whose gradient is final before that
    op)`` from the lowering (``Builder.mark_grads_ready``); ``buckets``: ``(param ids, start, end)``
    of ``GradBucketer``.  A bucket is released at the first mark whose lowest-ready index is at or
    below its lowest parameter (gradients become final in reverse parameter order).  Every bucket
    is placed exactly once, at or before the end of the backward segment."""
    mark_at: Dict[int, int] = {}
    for pos, lo in bwd_marks:
        mark_at[pos] = min(lo, mark_at.get(pos, lo))
    pending = sorted(((min(ids), s0, s1) for ids, s0, s1 in buckets), reverse=True)
    out: Dict[int, List[Tuple[int, int]]] = {}
    cur = None
    for i, op in enumerate(ops):
        seg = op[0]
        if seg != cur:
            if cur == "bwd" and pending:
                out.setdefault(i, []).extend((s0, s1) for _, s0, s1 in pending)
                pending = []
            cur = seg
        if cur == "bwd" and i in mark_at:
            while pending and pending[0][0] >= mark_at[i]:
                _, s0, s1 = pending.pop(0)
                out.setdefault(i, []).append((s0, s1))
    if pending:
        out.setdefault(len(ops), []).extend((s0, s1) for _, s0, s1 in pending)
    return out


class FusedProgram:
    def __init__(self, model, batch: int, training: bool, input_dtype, grad_scale: float = 1.0,
                 use_graphs: bool = True, skip_nonfinite: bool = False, group=None,
                 grad_weight: float = 1.0):
        """``group``: a ``runtime.grouped.GroupRegion`` — the program is built inside copy 0 of the
        region and every launch runs its K copies (client-batched federated training).
        ``grad_weight``: this rank's weight in an uneven split of a global batch; it scales the
        loss head's gradient seed, i.e. the LOCAL gradient before any all-reduce, while
        ``grad_scale`` (the optimizer's factor on the reduced sum) is the same on every rank."""
        nat.require()
        self.group = group
        self.model = model
        self.training = training
        self.batch = batch
        net = model.net
        self.U = net.num_outputs
        b = Builder(net, model.arena, model.device, batch, training)
        b.grouped = group is not None
        b.shared_device = bool(getattr(getattr(model, "impl", None), "shared_device", False))
        b.grad_weight = float(grad_weight)
        b.persist_ok = persistent_allowed(model, training)
        _lowering_for(net)(b, net, self.U, input_dtype)
        if b.has_wgrad_batch():  # a lowering that returned early (frozen layers) mid-batch
            b.segment = "bwd"
            b.flush_wgrad_batch()
        if b.pending_sums:  # BatchNorm gradient slot copies no apply kernel folded
            b.segment = "bwd"
            b.flush_grad_sums()
        if training and b.ops:
            # statistics shifts advance after the step's last statistics consumer
            b.segment = b.ops[-1][0]
            b.emit_stats_shift()
        self.b = b
        self.xin = b.xin
        self.io = b.io
        # the input stage (OP_INPUT) becomes the program's first op and is issued directly (never
        # captured): each step points it at the caller's own x / y tensors, so staging the inputs
        # costs one launch and no copies (FusedStep._stage_inputs)
        self.input_op = None
        k = next((i for i, op in enumerate(b.ops) if op[1] == nat.OP_INPUT), None)
        if k is not None and all(op[0] == "fwd" and op[1] == nat.OP_MEMSET for op in b.ops[:k]) \
                and b.ops[k][0] == "fwd" and not any(pos <= k for pos, _ in b.bwd_marks):
            seg, kind, raw, ints, floats, longs, ptrs, lane = b.ops.pop(k)
            ints = list(ints) + [0] * (8 - len(ints))
            ints[6], ints[7] = 0, self.U
            ptrs = list(ptrs) + [0] * (4 - len(ptrs))
            ptrs[2], ptrs[3] = 0, self.io.labels.data_ptr()
            b.ops.insert(0, (seg, kind, raw, ints, floats, longs, ptrs, lane))
            self.input_op = 0
        b.finalize_casts()
        b.finalize_moving()
        strategy = model.strategy
        if training and model.arena.params and b.step_flag is None and getattr(strategy, "native_comm", None) is not None \
                and strategy.active and not getattr(strategy, "central_storage", False):
            # every rank's program carries the step-guard all-reduce (below) and its optimizer reads
            # the summed word, whether or not its own lowering built persistent launches: the
            # ranks' collective sequences match and a give-up on any rank skips the step on all
            b.step_flag = b._stats_floats(4).view(torch.int32)
        # optimizer segment
        self.nonfinite_status = None
        if training and model.arena.params:
            opt = model.optimizer
            self.host_optimizer = not isinstance(opt, RMSprop) or bool(opt.momentum) or bool(opt.centered)
            flag = 0
            # persistent dense-stage launches OR 2 into the step guard word when they give up
            # (csrc/kernels/persist.h note_fail): RMSprop then skips the step's update, so stale
            # stage outputs never reach the weights.  The word lives in the stats arena, which every
            # training step zeroes first.
            guard = b.step_flag.data_ptr() if b.step_flag is not None else 0
            if guard and not self.host_optimizer:
                flag = guard
            if skip_nonfinite and not self.host_optimizer:
                # non-finite guard: the gradient arena is checked at the end of the
                # backward; RMSprop skips the whole update when anything is inf/nan
                # (opt segment: under data parallelism it runs after the all-reduce, so every
                # replica sees the same reduced gradients and makes the same decision)
                if not flag:
                    flag = b.alloc((4,), torch.int32).data_ptr()
                self.nonfinite_status = b.alloc((4,), torch.int32)
            b.segment = "opt"
            if skip_nonfinite and flag:
                b.emit(nat.OP_FINITE_CHECK, ints=(0,), longs=(model.arena.numel,),
                       ptrs=(model.arena.grad.data_ptr(), flag))
            if not self.host_optimizer:
                ms = opt.ms
                hflag = 0
                if flag and flag == guard and not b.grouped and torch.cuda.is_available():
                    # a skip caused by a give-up on any rank raises this rank's host flag too
                    if not b.host_flag:
                        from .builder import _host_flag_slot
                        b.host_flag = _host_flag_slot()
                    hflag = b.host_flag
                b.emit(nat.OP_RMSPROP, floats=(opt.learning_rate, opt.rho, opt.epsilon, grad_scale),
                       longs=(model.arena.numel,),
                       ptrs=(model.arena.data.data_ptr(), model.arena.grad.data_ptr(), ms.data_ptr(), flag,
                             hflag))
            if b.cast_tr_n:
                b.emit(nat.OP_CAST, ints=(b.cast_tr_n,), longs=(b.cast_tr_total,),
                       ptrs=(b.cast_tr_dev.data_ptr(), b.cast_tr_map.data_ptr()))
            if skip_nonfinite and flag:
                b.emit(nat.OP_FINITE_CHECK, ints=(1,), ptrs=(0, flag, self.nonfinite_status.data_ptr()))
        else:
            self.host_optimizer = False
        self.plan = nat.load().Plan()
        # side-lane ops are issued in batches every IDC_SIDE_FLUSH main ops (plan.cpp: issue).
        # Batching saves host calls where the backward is many short kernels (DenseNet: 128 main
        # ops; 3-4 measured best, 4.27-4.34 ms/step vs 4.30-4.43 at 6-8 and 4.42 at 2; MobileNetV2,
        # 89 main ops: 2.47 ms/step at 4 vs 2.56 at 0, 3 A/B pairs in round 3); a backward of few
        # long kernels (VGG16: 20 main ops of 45-220 us) forks every side op at once (0), or its
        # weight gradients would wait for the next dgrads to finish before starting
        # round 4 (DenseNet-121: 97 main backward ops after the persistent stage-4 backward):
        # 2 -> 3.894-3.901 ms/step, 3 -> 3.915-3.923, 4 -> 3.953-3.964; MobileNetV2 (73 ops): 2 ->
        # 2.394-2.395, 3 -> 2.318, 4 -> 2.322-2.329
        n_bwd_main = sum(1 for op in b.ops if op[0] == "bwd" and op[7] == 0)
        # grouped (client-batched) DenseNet: secure FedAvg 0.410-0.414 s/round at 0 vs 0.416 at 2,
        # 0.418 at 4; grouped MobileNetV2 FedAvg keeps 4 (0.220-0.222 vs 0.223 at 0)
        # IDC_SIDE_CUS=N (plan.cpp ensure_side: the side lane on a CU-masked queue of N CUs) is
        # opt-in: round 5, 64 / 128 / 192 CUs against the unmasked default, ms/step: MobileNetV2
        # 2.609 / 2.739 / 2.722 vs 2.311, VGG16 2.467 / 2.448 / 2.461 vs 2.388, DenseNet-121
        # 3.942 / 3.931 / 3.865 vs 3.702
        big = n_bwd_main >= 90
        default_flush = "0" if b.grouped and big else "2" if big else "4" if n_bwd_main >= 64 else "0"
        self.plan.set_side_flush(int(os.environ.get("IDC_SIDE_FLUSH", default_flush)))
        self.seg: Dict[str, Tuple[int, int]] = {}
        self.rms_index = None
        op_index = 0
        self.bwd_marks = []
        mark_at = {}
        for pos, lo in b.bwd_marks:
            mark_at.setdefault(pos, []).append(lo)
        # Data parallelism over the strategy's native RCCL communicator: every gradient bucket's
        # all-reduce becomes a plan op (OP_ALLREDUCE, comm lane) placed at the first backward mark
        # after which all of its parameters' gradients are final (place_buckets), so the C++
        # executor issues the whole backward + collectives in one call.
        self.native_comm = None
        placed: Dict[int, List[Tuple[int, int]]] = {}
        if training and model.arena.params and getattr(strategy, "native_comm", None) is not None \
                and strategy.active and not getattr(strategy, "central_storage", False):
            from ..parallel.buckets import GradBucketer
            self.native_comm = strategy.native_comm
            gb = GradBucketer(model.arena, strategy.bucket_bytes)
            placed = place_buckets(b.ops, b.bwd_marks, [(bk.param_ids, bk.start, bk.end) for bk in gb.buckets])
        self.n_comm_ops = 0

        def add_buckets(i: int):
            nonlocal op_index
            for s0, s1 in placed.get(i, ()):
                self.plan.add(nat.OP_ALLREDUCE, b"", [0, 0], [], [s1 - s0],
                              [model.arena.grad.data_ptr() + 4 * s0], 0)
                op_index += 1
                self.n_comm_ops += 1

        # under data parallelism a give-up on ONE rank must skip the update on EVERY rank (the
        # stale gradients were all-reduced into everyone's): the step guard word is summed over
        # the ranks at the end of the backward, after every persistent launch of the step
        guard_ar = self.native_comm is not None and b.step_flag is not None

        def add_guard_allreduce():
            nonlocal op_index, guard_ar
            if guard_ar:
                self.plan.add(nat.OP_ALLREDUCE, b"", [2, 0], [], [1], [b.step_flag.data_ptr()], 0)
                op_index += 1
                self.n_comm_ops += 1
                guard_ar = False

        cur, start = None, 0
        for i, (seg, kind, raw, ints, floats, longs, ptrs, lane) in enumerate(b.ops):
            if seg != cur:
                if cur == "bwd":
                    add_buckets(i)  # buckets no mark released (params without gradient)
                    add_guard_allreduce()
                if cur is not None:
                    self.seg[cur] = (start, op_index)
                cur, start = seg, op_index
            if i in mark_at:
                self.bwd_marks.append((op_index, min(mark_at[i])))
                if cur == "bwd":
                    add_buckets(i)
            if kind == "MOVING":
                if b.moving_dev is None:
                    continue
                kind, ints, ptrs = nat.OP_BN_MOVING, [len(b.moving), b.moving_maxc], [b.moving_dev.data_ptr()]
            if kind == nat.OP_MEMSET and ptrs[0] == b.stats_arena.data_ptr():
                longs = [max(b._stats_size, 4) * 4]
            if kind == nat.OP_RMSPROP:
                self.rms_index = op_index
            self.plan.add(kind, raw, ints, floats, longs, ptrs, lane)
            op_index += 1
        if cur == "bwd":
            add_buckets(len(b.ops))
            add_guard_allreduce()
        if cur is not None:
            self.seg[cur] = (start, op_index)
        if self.native_comm is not None:
            self.plan.set_comm(self.native_comm.c)
        self.use_graphs = use_graphs and os.environ.get("IDC_NO_GRAPHS", "0") != "1"
        # Which segments replay as HIP graphs.  The backward is issued directly by default: one
        # captured fork/join graph loses the side lane's concurrency under ROCm's graph executor
        # (4.93 vs 4.45 ms/step direct on DenseNet-121), and the opt-in IDC_DUAL_GRAPH=1 (main-
        # and side-lane graphs joined by event nodes, plan.cpp capture_dual) is exact but slower
        # still (6.1 ms/step: ROCm runs graphs holding event nodes node by node)
        self.dual_graphs = os.environ.get("IDC_DUAL_GRAPH", "0") == "1"
        default_graphs = "fwd,bwd,opt" if self.dual_graphs else "fwd,opt"
        self.graph_segments = set(os.environ.get("IDC_GRAPH_SEGMENTS", default_graphs).split(","))
        # opt-in: measured slower than direct issue on DenseNet-121 bs256 (4.62-5.0 vs 4.45-4.53
        # ms/step at 4-16 chunks): the side lane then waits for whole main chunks
        self.bwd_chunks = int(os.environ.get("IDC_BWD_CHUNKS", "0")) if self.use_graphs else 0
        if self.dual_graphs or "bwd" in self.graph_segments:
            self.bwd_chunks = 0  # the older whole-segment graph forms were asked for
        self._bwd_graphs = None
        self.graphs: Dict[Tuple[int, int], int] = {}
        self.grad_scale = grad_scale
        # stream priorities are opt-in (IDC_MAIN_PRIO=high, IDC_SIDE_PRIO=low in plan.cpp): measured
        # neutral on DenseNet-121 bs256 (4.90-4.96 vs 4.92-5.01 ms/step), and 1.2 ms/step slower
        # under rocprofv3 kernel tracing
        main_prio = -1 if os.environ.get("IDC_MAIN_PRIO", "normal") == "high" else 0
        self.stream = torch.cuda.Stream(device=model.device, priority=main_prio)
        self.comm_stream = torch.cuda.Stream(device=model.device)  # issues the gradient all-reduces
        # initial bf16 weight casts (all convs, frozen ones included)
        if b.cast_all_n:
            cast = nat.load().Plan()
            cast.add(nat.OP_CAST, b"", [b.cast_all_n], [], [b.cast_all_total],
                     [b.cast_all_dev.data_ptr(), b.cast_all_map.data_ptr()])
            self._cast_all_plan = cast
        else:
            self._cast_all_plan = None
        self.recast_all()
        if group is not None:
            # every pointer of the plan must lie in copy 0 of the region (the kernels reach copy g
            # by adding g * stride); the other copies start as replicas of copy 0, so that even
            # the autotuner's grouped trial launches only ever read well-formed data
            group.validate_program(self)
            group.replicate(self.stream)
            self.plan.set_groups(group.k, group.stride)
            if self._cast_all_plan is not None:
                self._cast_all_plan.set_groups(group.k, group.stride)
        # autotuning picks tiles by timing, which may differ from run to run: a deterministic
        # program keeps the fixed default tiles (and no split-K)
        if os.environ.get("IDC_AUTOTUNE", "1") != "0" and not b.det:
            from .autotune import autotune_plan
            autotune_plan(self.plan, self.stream, verbose=os.environ.get("IDC_TUNE_VERBOSE") == "1",
                          reset_tickets=b.reset_tickets, slab_floats=b.SLAB_FLOATS)
        b.reset_tickets()  # split-K tickets count modulo the op's split: start every op aligned

    # ------------------------------------------------------------------ execution
    def _sh(self):
        return self.stream.cuda_stream

    def recast_all(self):
        # the masters (and, right after lowering, the zero-fills of every freshly allocated
        # buffer) were written on the caller's stream: order the plan stream after them
        self.stream.wait_stream(torch.cuda.current_stream(self.model.device))
        if self._cast_all_plan is not None:
            with torch.cuda.stream(self.stream):
                self._cast_all_plan.run(0, -1, self._sh())

    def reset_stats_shift(self):
        """Zero every statistics shift (the state the first step starts from): comparisons that
        replay one program on several inputs as if each were a first step use it."""
        for st in self.b.all_stats:
            if st.shift is not None:
                st.shift.zero_()

    def run_range(self, lo: int, hi: int, graph: Optional[bool] = None, join: bool = True):
        """Issue ops [lo, hi).  ``join=False`` (direct issue only) leaves the side lane running
        past the end of the range: use ``side_ready_on`` to order a consumer after it."""
        if hi <= lo:
            return
        if graph is None:
            graph = self.use_graphs and self._graph_for(lo)
        if graph and self.dual_graphs and self.plan.has_side(lo, hi) and not self.plan.has_comm_ops(lo, hi):
            # main-lane and side-lane graphs joined by external events (plan.cpp capture_dual)
            g = self.graphs.get(("dual", lo, hi))
            if g is None:
                g = self.plan.capture_dual(lo, hi, self._sh())
                self.graphs[("dual", lo, hi)] = g
            self.plan.launch_dual(g, self._sh(), join)
        elif graph:
            g = self.graphs.get((lo, hi))
            if g is None:
                g = self.plan.capture(lo, hi, self._sh())
                self.graphs[(lo, hi)] = g
            self.plan.launch(g, self._sh())
        else:
            self.plan.run(lo, hi, self._sh(), join)

    def side_ready_on(self, stream: torch.cuda.Stream):
        """``stream`` waits for the main lane so far AND every side-lane op issued so far."""
        stream.wait_stream(self.stream)
        self.plan.wait_side(stream.cuda_stream)

    def _graph_for(self, lo: int) -> bool:
        for name, (a, b) in self.seg.items():
            if a <= lo < b:
                return name in self.graph_segments
        return True

    # ---- backward as lane-split chunk graphs (plan.cpp capture_lane) ----------------------
    def _bwd_chunks(self, nchunks: int):
        lo, hi = self.seg["bwd"]
        n_main = self.plan.count_lane(lo, hi, 0)
        per = max(1, -(-n_main // max(1, nchunks)))
        bounds, start, count = [], lo, 0
        for i in range(lo, hi):
            if self.plan.lane(i) == 0 and self.plan.kind(i) != nat.OP_ALLREDUCE:
                count += 1
                if count == per:
                    bounds.append((start, i + 1))
                    start, count = i + 1, 0
        if start < hi:
            bounds.append((start, hi))
        return bounds

    def run_bwd(self):
        """The backward segment.  Default (IDC_BWD_CHUNKS=N, N>0): N chunks, each replayed as a
        main-lane graph on the plan stream plus a side-lane (weight-gradient) graph forked after
        it, so a chunk's weight gradients overlap the next chunk's data gradients; collectives of
        a chunk (native data parallelism) follow its side graph on the comm stream.  N=0: direct
        issue of every op with per-batch side forks (plan.cpp issue)."""
        lo, hi = self.seg["bwd"]
        if self.bwd_chunks <= 0:
            # whole-segment forms (IDC_DUAL_GRAPH=1 / "bwd" in IDC_GRAPH_SEGMENTS) replay graphs,
            # everything else issues directly
            self.run_range(lo, hi, graph=None if self.use_graphs else False)
            return
        plan, sh = self.plan, self._sh()
        if self._bwd_graphs is None:
            self._bwd_graphs = [(a, b2, plan.capture_lane(a, b2, 0, sh), plan.capture_lane(a, b2, 1, sh))
                                for a, b2 in self._bwd_chunks(self.bwd_chunks)]
        for a, b2, gm, gs in self._bwd_graphs:
            if gm >= 0:
                plan.launch(gm, sh)
            if gs >= 0:
                plan.fork_side(sh)
                plan.launch_side(gs)
            if self.native_comm is not None:
                plan.comm_range(a, b2, sh)
        plan.join_side(sh)
        plan.join_comm(sh)

    def run_segment(self, name: str):
        if name in self.seg:
            with trace.range("seg:" + name):
                lo, hi = self.seg[name]
                if name == "fwd" and self.input_op == lo:
                    # direct issue with this step's operands, then back to the program's own
                    # buffers (a later forward without staging reads xin, as before)
                    self.plan.run(lo, lo + 1, self._sh(), True)
                    self.plan.set_ptr(lo, 0, self.xin.data_ptr())
                    self.plan.set_ptr(lo, 2, 0)
                    self.plan.set_int(lo, 6, 0)
                    lo += 1
                self.run_range(lo, hi)

    def set_lr(self, lr: float):
        if self.rms_index is not None:
            self.plan.set_float(self.rms_index, 0, float(lr))
            self.plan.clear_graphs()
            self.graphs = {}
            self._bwd_graphs = None

    def close(self):
        self.plan.clear_graphs()


_LABEL_CODES = {torch.float32: 1, torch.int64: 2, torch.int32: 3, torch.uint8: 4}


def _direct_input_codes(p: "FusedProgram", x, y):
    """None: stage through copies.  Else the input op's label code (0: no labels) for reading the
    caller's x / y in place: same device, dtype and shape as the program's input, contiguous;
    labels as the head takes them (U == 1: [B]; U > 1: [B] class ids or an [B, U] fp32 matrix)."""
    if p.input_op is None or p.group is not None or not isinstance(x, torch.Tensor):
        return None
    xin = p.xin
    if x.device != xin.device or x.dtype != xin.dtype or x.shape != xin.shape or not x.is_contiguous():
        return None
    if y is None:
        return 0
    if not isinstance(y, torch.Tensor) or y.device != xin.device or not y.is_contiguous():
        return None
    code = _LABEL_CODES.get(y.dtype)
    if code is None:
        return None
    B, U = xin.shape[0], p.U
    if U == 1 or code != 1:
        return code if y.numel() == B else None
    return code if tuple(y.shape) == (B, U) else None


def _labels_to(io_labels: torch.Tensor, y: torch.Tensor, U: int):
    y = y.to(io_labels.device, non_blocking=True)
    if U == 1:
        io_labels.copy_(y.reshape(-1))  # one conversion kernel (no float temporary)
    elif y.dim() == 2 and y.shape[1] == U:
        io_labels.copy_(y)
    else:
        io_labels.zero_()
        io_labels.scatter_(1, y.reshape(-1, 1).long(), 1.0)


class FusedStep:
    """``engine.Model`` backend that runs the lowered MI355X program."""

    name = "fused"

    def __init__(self, model, use_graphs: bool = True, skip_nonfinite: Optional[bool] = None):
        self.m = model
        self.use_graphs = use_graphs
        if skip_nonfinite is None:
            skip_nonfinite = os.environ.get("IDC_SKIP_NONFINITE", "0") == "1"
        self.skip_nonfinite = skip_nonfinite
        self.progs: Dict[tuple, FusedProgram] = {}
        self._lr = model.optimizer.learning_rate if model.optimizer else None
        self.group = None  # runtime.grouped.GroupRegion: programs run K copies (grouped.py)
        self.shared_device = False  # other programs run concurrently on the device (fedavg workers)

    def _prog(self, batch: int, training: bool, dtype) -> FusedProgram:
        from ..parallel.strategy import current_replica_weight
        w = current_replica_weight[0] if training else 1.0  # uneven split of a global batch
        key = (batch, training, dtype) if w == 1.0 else (batch, training, dtype, w)
        p = self.progs.get(key)
        if p is None:
            # the share weight w scales this rank's gradient seed (before the all-reduce); the
            # reduced sum is scaled by the same 1/N on every rank, so replicas stay identical
            gs = 1.0 / self.m.strategy.num_replicas_in_sync
            p = FusedProgram(self.m, batch, training, dtype, grad_scale=gs, use_graphs=self.use_graphs,
                             skip_nonfinite=self.skip_nonfinite, group=self.group, grad_weight=w)
            self.progs[key] = p
        return p

    def _stage_inputs(self, p: FusedProgram, x, y):
        cur = torch.cuda.current_stream(self.m.device)
        p.stream.wait_stream(cur)
        code = _direct_input_codes(p, x, y)
        if code is not None:
            # the input op reads x and y where they are (one launch, no copies); they stay
            # allocated until it has run on the program stream
            p.plan.set_ptr(p.input_op, 0, x.data_ptr())
            x.record_stream(p.stream)
            if code:
                p.plan.set_ptr(p.input_op, 2, y.data_ptr())
                p.plan.set_int(p.input_op, 6, code)
                y.record_stream(p.stream)
            return
        with torch.cuda.stream(p.stream):
            p.xin.copy_(x.to(p.xin.device, non_blocking=True).to(p.xin.dtype))
            if y is not None:
                _labels_to(p.io.labels, y, p.U)

    def _validate(self, p, where):
        """IDC_VALIDATE=1 debugging aid: after a segment, every program buffer and the master
        weights must be finite and bounded; report the first offending buffer."""
        torch.cuda.synchronize(self.m.device)
        named = [("arena.data", self.m.arena.data), ("arena.grad", self.m.arena.grad)]
        named += [(f"keep[{i}]{tuple(t.shape)}", t) for i, t in enumerate(p.b.keep) if t.is_floating_point()]
        named.append(("stats_arena", p.b.stats_arena))
        bad = []
        err = getattr(p.b, "dense_err", None)
        if err is not None and int(err[0].item()):
            bad.append(f"dense_err={int(err[0].item())} (a persistent dense-stage launch timed out)")
        for name, t in named:
            if t.numel() and (not bool(torch.isfinite(t).all()) or t.float().abs().max().item() > 1e8):
                bad.append(f"{name} max={t.float().abs().max().item():.3g}")
        if bad:
            print(f"[validate] {where}: {len(bad)} bad buffers: " + "; ".join(bad[:40]), flush=True)
        return not bad

    # ---- fail-safe of the persistent dense-stage launches -----------------------------------
    def check_persistent(self) -> int:
        """Poll the programs' pinned host give-up flags (no device synchronisation).  A set flag
        means a persistent dense-stage launch of an already finished step gave up on a wait: that
        step's weight update was skipped on the device (step guard word, csrc/kernels/persist.h).
        Policy IDC_DS_ON_FAIL: ``fallback`` (default) switches persistent launches off for the
        process and rebuilds the programs with per-layer kernels; ``raise`` raises
        PersistentLaunchError.  Returns the number of programs that reported a give-up."""
        import ctypes
        from .builder import PersistentLaunchError, disable_persistent
        hit = []
        for key, p in self.progs.items():
            hf = getattr(p.b, "host_flag", 0)
            if hf and ctypes.c_int.from_address(hf).value:
                ctypes.c_int.from_address(hf).value = 0
                hit.append(key)
        if not hit:
            return 0
        policy = os.environ.get("IDC_DS_ON_FAIL", "fallback")
        msg = (f"a persistent dense-stage launch gave up on a wait in program(s) {hit}; the "
               "affected step(s) skipped their weight update")
        if policy == "raise":
            raise PersistentLaunchError(msg)
        disable_persistent(msg)
        torch.cuda.current_stream(self.m.device).wait_stream(next(iter(self.progs.values())).stream)
        for p in self.progs.values():
            p.stream.synchronize()
            p.close()
        self.progs = {}
        return len(hit)

    def train_step(self, x, y):
        """One training step.  Returns (loss, logits) as VIEWS of the program's output buffers:
        the next step of the same program overwrites them (clone() them to keep them; see
        _outputs)."""
        with trace.range("train_step"):
            if self.progs:
                self.check_persistent()
            return self._train_step(x, y)

    def _train_step(self, x, y):
        m = self.m
        dtype = torch.uint8 if x.dtype == torch.uint8 else torch.float32
        p = self._prog(x.shape[0], True, dtype)
        if p.native_comm is not None:
            # a failure the watchdog acted on since the last step surfaces as CommFailure here,
            # before anything is enqueued on the aborted communicator
            p.native_comm.check()
        self._stage_inputs(p, x, y)
        validate = os.environ.get("IDC_VALIDATE") == "1"
        if validate:
            self._validate(p, "before fwd")
        p.run_segment("fwd")
        if validate:
            self._validate(p, "after fwd")
        strategy = m.strategy
        active = strategy.active
        if active and getattr(strategy, "central_storage", False):
            return self._central_storage_step(p, validate)
        if "bwd" in p.seg:
            trace.push("seg:bwd")
            lo, hi = p.seg["bwd"]
            bucketer = strategy.bucketer(m.arena) if active and p.native_comm is None else None
            if p.native_comm is not None or bucketer is None:
                # the plan itself issues every bucket all-reduce on the communicator's stream and
                # joins it back into the main lane at the end of the range
                p.run_bwd()
                if p.native_comm is not None:
                    p.native_comm.step_issued()  # watchdog progress mark (parallel/watchdog.py)
            elif bucketer is not None and p.bwd_marks:
                # backward in bucket-aligned segments: each bucket's all-reduce is issued from
                # the comm stream as soon as its gradients are final — the comm stream waits for
                # the main lane AND the side-lane weight gradients issued so far, while the main
                # lane itself runs on without joining the side lane (plan.cpp run(join=False))
                cs = p.comm_stream
                pos = lo
                for mark, low_param in p.bwd_marks:
                    if mark <= pos:
                        continue
                    p.run_range(pos, mark, join=False)
                    pos = mark
                    p.side_ready_on(cs)
                    with torch.cuda.stream(cs), trace.range("allreduce:from_param%d" % low_param):
                        bucketer.launch_range(low_param, None)
                p.run_range(pos, hi)
                cs.wait_stream(p.stream)
                with torch.cuda.stream(cs):
                    bucketer.finish()
                p.stream.wait_stream(cs)
            else:
                p.run_range(lo, hi)
                with torch.cuda.stream(p.stream):
                    bucketer.finish()
            trace.pop()
        if p.host_optimizer:
            with torch.cuda.stream(p.stream):
                m.optimizer.step(m.arena, grad_scale=p.grad_scale)
        if validate:
            self._validate(p, "after bwd")
        p.run_segment("opt")
        if validate:
            self._validate(p, "after opt")
        torch.cuda.current_stream(m.device).wait_stream(p.stream)
        return self._outputs(p)

    @staticmethod
    def _outputs(p: FusedProgram):
        """(loss, logits) as VIEWS of the program's output buffers, ordered after the step on the
        caller's stream and valid until the next step of the same program (copies would add two
        dependent launches to every step; Model.fit consumes them before the next step is issued)."""
        return p.io.loss.reshape(()), p.io.logits

    def _central_storage_step(self, p: FusedProgram, validate: bool):
        """CentralStorageStrategy (``dist_model_tf_dense.py:24``): gradients are reduced to rank 0,
        only rank 0 owns optimizer state and applies RMSprop, the updated fp32 parameters are
        broadcast and every rank re-casts its bf16 kernel copies."""
        m = self.m
        st = m.strategy
        p.run_segment("bwd")
        st.reduce_to_root(m.arena.grad, p.stream)
        if "opt" in p.seg:
            lo, hi = p.seg["opt"]  # [finite check] rmsprop | cast [flag reset]
            if p.host_optimizer:
                if st.rank == 0:
                    with torch.cuda.stream(p.stream):
                        m.optimizer.step(m.arena, grad_scale=1.0 / st.world)
                cast_lo = lo
            else:
                if st.rank == 0:
                    p.run_range(lo, p.rms_index + 1, graph=False)
                cast_lo = p.rms_index + 1
            st.broadcast_from_root(m.arena.data, p.stream)
            p.run_range(cast_lo, hi, graph=False)
        torch.cuda.current_stream(m.device).wait_stream(p.stream)
        return self._outputs(p)

    def persistent_failures(self) -> int:
        """Persistent dense-stage launches (forward or backward) of this backend's programs that
        gave up on a wait: their outputs are stale (one small device read per call)."""
        n = 0
        for p in self.progs.values():
            err = getattr(p.b, "dense_err", None)
            if err is not None:
                n += int(err[0].item())
        return n

    def skipped_steps(self) -> int:
        """Training steps whose update was skipped for non-finite gradients (skip_nonfinite)."""
        n = 0
        for p in self.progs.values():
            if p.nonfinite_status is not None:
                n += int(p.nonfinite_status[1].item())
        return n

    def eval_step(self, x, y):
        """One inference step.  Returns (loss, logits) as VIEWS of the program's output buffers,
        like train_step: the next step of the same program overwrites them (clone() to keep)."""
        if self.progs:
            self.check_persistent()
        dtype = torch.uint8 if x.dtype == torch.uint8 else torch.float32
        p = self._prog(x.shape[0], False, dtype)
        self._stage_inputs(p, x, y)
        p.run_segment("fwd")
        torch.cuda.current_stream(self.m.device).wait_stream(p.stream)
        return self._outputs(p)

    def reset_stats_shift(self):
        """Every program back to a first step's statistics shifts (a federated client starts
        from the same state whichever worker model, and whatever client before it, it runs on)."""
        for p in self.progs.values():
            p.reset_stats_shift()

    def sync_from_module(self):
        # weights were overwritten on the module side (set_weights / load_weights): re-cast
        for p in self.progs.values():
            p.recast_all()

    def sync_to_module(self):
        # the programs' own streams, not the device: concurrent federated clients on other
        # worker models keep running (the side lane joins the main stream inside every step)
        for p in self.progs.values():
            p.stream.synchronize()
            p.comm_stream.synchronize()
        torch.cuda.current_stream(self.m.device).synchronize()

    def close(self):
        for p in self.progs.values():
            p.close()
        self.progs = {}
