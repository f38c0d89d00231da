"""Failure detection of the native RCCL communicator (``parallel/watchdog.py``,
``parallel/native_comm.py``), on the CPU:

* the watchdog policy against a fake communicator (stalled collectives, asynchronous errors, no
  marks on an aborted communicator, ``wait_with_watchdog``);
* end to end in a real gloo world of 2: a peer that never joins a collective is detected by the
  watchdog and surfaces as ``CommFailure`` on the waiting rank instead of a hang;
* one native communicator per rank: the strategy's buckets and the secure-aggregation ring share it
  (and its watchdog); releasing it closes it for every holder;
* packed all-reduces keep float64 accumulators exact (FedAvg example counts and metric sums).

Reference: the implicit collective timeouts of ``tf.distribute`` around the NCCL all-reduce
(``/root/reference/dist_model_tf_vgg.py:115-117``); the secure round's aggregation
(``/root/reference/secure_fed_model.py:224-233``).
"""
import threading
import time

import numpy as np
import pytest
import torch

from idc_models_amd.parallel.launch import spawn


class _WdComm:
    def __init__(self):
        self.age = 0.0
        self.async_err = None
        self.aborted = 0
        self.marks = 0

    def check_async(self):
        if self.async_err:
            raise RuntimeError(self.async_err)

    def mark_age(self):
        return self.age

    def mark(self):
        self.marks += 1

    def abort(self):
        self.aborted += 1


def test_watchdog_aborts_on_stalled_collectives():
    from idc_models_amd.parallel.watchdog import CommFailure, CommWatchdog
    c = _WdComm()
    wd = CommWatchdog(c, timeout_s=5.0)
    wd.mark()
    assert c.marks == 1
    c.age = 4.0
    assert wd.poll_once() is None and c.aborted == 0
    wd.raise_if_failed()
    c.age = 6.0
    reason = wd.poll_once()
    assert reason is not None and "no progress" in reason and c.aborted == 1
    with pytest.raises(CommFailure):
        wd.raise_if_failed()
    wd.poll_once()  # sticky: no second abort
    assert c.aborted == 1
    wd.mark()
    assert c.marks == 1  # no marks on an aborted communicator


def test_watchdog_aborts_on_async_error_from_its_thread():
    from idc_models_amd.parallel.watchdog import CommFailure, CommWatchdog
    c = _WdComm()
    wd = CommWatchdog(c, timeout_s=100.0, poll_s=0.01).start()
    try:
        time.sleep(0.05)
        assert c.aborted == 0
        c.async_err = "remote process exited"
        t0 = time.time()
        while wd.error is None and time.time() - t0 < 5:
            time.sleep(0.01)
        assert c.aborted == 1 and "remote process exited" in wd.error
        with pytest.raises(CommFailure):
            wd.raise_if_failed()
    finally:
        wd.stop()


def test_wait_with_watchdog_raises_when_aborted():
    from idc_models_amd.parallel.watchdog import CommFailure, CommWatchdog, wait_with_watchdog
    c = _WdComm()
    wd = CommWatchdog(c, timeout_s=0.5, poll_s=0.01).start()
    try:
        wd.mark()
        c.age = 1.0  # the mark never completes
        with pytest.raises(CommFailure):
            wait_with_watchdog(wd, lambda: False, poll_s=0.01, timeout_s=10)
    finally:
        wd.stop()


def test_mark_never_reaches_an_aborted_communicator():
    """mark() re-checks the failure under the watchdog lock: a poll that aborts the communicator
    while the training thread is about to mark it wins, and the mark is dropped."""
    from idc_models_amd.parallel.watchdog import CommWatchdog
    c = _WdComm()
    wd = CommWatchdog(c, timeout_s=1.0)
    entered, release = threading.Event(), threading.Event()
    orig_abort = c.abort

    def slow_abort():
        entered.set()
        release.wait(5)
        orig_abort()
    c.abort = slow_abort
    c.age = 2.0
    t = threading.Thread(target=wd.poll_once)
    t.start()
    entered.wait(5)
    marker = threading.Thread(target=wd.mark)  # blocks on the lock until the abort is recorded
    marker.start()
    time.sleep(0.05)
    release.set()
    t.join(5)
    marker.join(5)
    assert c.aborted == 1 and c.marks == 0 and wd.error is not None


# ---------------------------------------------------------------------------------------------
# end to end over a real gloo world


class _GlooComm:
    """The watchdog's duck-typed communicator over gloo: mark() starts an asynchronous all-reduce
    (the 'step's collectives'); its age grows until every rank has joined it."""

    def __init__(self):
        self.work, self.t0, self.aborted = None, 0.0, 0
        self.buf = torch.ones(4)

    def check_async(self):
        pass

    def mark(self):
        import torch.distributed as dist
        self.work = dist.all_reduce(self.buf, async_op=True)
        self.t0 = time.monotonic()

    def mark_age(self):
        if self.work is None or self.work.is_completed():
            return 0.0
        return time.monotonic() - self.t0

    def abort(self):
        self.aborted += 1


def _hang_worker(rank, world):
    import torch.distributed as dist
    from torch.distributed import distributed_c10d as c10d
    from idc_models_amd.parallel.watchdog import CommFailure, CommWatchdog, wait_with_watchdog
    store = c10d._get_default_store()
    if rank == 0:
        c = _GlooComm()
        wd = CommWatchdog(c, timeout_s=0.5, poll_s=0.05, name="gloo rank 0").start()
        wd.mark()  # rank 1 is "hung": it does not join this collective
        t0 = time.monotonic()
        try:
            wait_with_watchdog(wd, c.work.is_completed, poll_s=0.02, timeout_s=60)
            raised = None
        except CommFailure as e:
            raised = str(e)
        waited = time.monotonic() - t0
        wd.stop()
        store.set("detected", "1")  # let the peer join so both processes exit cleanly
        c.work.wait()
        return {"raised": raised, "aborted": c.aborted, "waited": waited}
    store.wait(["detected"])
    dist.all_reduce(torch.ones(4))
    return None


def test_watchdog_detects_a_hung_peer_in_a_gloo_world():
    res = spawn(_hang_worker, 2)[0]
    assert res["raised"] is not None and "no progress" in res["raised"], res
    assert res["aborted"] == 1
    assert 0.4 < res["waited"] < 30, res


def _packed_worker(rank, world):
    from idc_models_amd.parallel import comm
    big = torch.tensor([2.0 ** 30 + 1 + rank, 1e-9 * (rank + 1)], dtype=torch.float64)
    f32 = torch.tensor([0.5 + rank], dtype=torch.float32)
    comm.all_reduce_packed_([f32, big])
    return big.numpy().copy(), f32.numpy().copy()


def test_packed_all_reduce_keeps_float64_exact():
    """FedAvg's [delta sums | n | metrics] reduction (fed/fedavg.py): one packed all-reduce per
    dtype; a float64 count above 2^24 (not representable in float32) survives exactly."""
    res = spawn(_packed_worker, 2)
    for big, f32 in res:
        assert big[0] == 2.0 ** 31 + 3  # (2^30 + 1) + (2^30 + 2)
        assert big[1] == pytest.approx(3e-9, rel=1e-12)
        assert f32[0] == 2.0


# ---------------------------------------------------------------------------------------------
# one communicator per rank


class _FakeComm:
    made = []

    def __init__(self, rank, world, uid, device, init_timeout_s=0.0):
        self.closed = 0
        self.stream = 0
        _FakeComm.made.append(self)

    @staticmethod
    def make_unique_id():
        return bytes(128)

    def close(self):
        self.closed += 1


class _FakeExt:
    Communicator = _FakeComm


def test_shared_communicator_is_reused_and_released():
    from idc_models_amd.parallel import native_comm as ncm
    _FakeComm.made.clear()
    dev = torch.device("cuda", 0)
    a = ncm.shared_communicator(0, 1, dev, ext=_FakeExt(), watchdog=False)
    b = ncm.shared_communicator(0, 1, dev, ext=_FakeExt(), watchdog=False)
    assert a is b and len(_FakeComm.made) == 1
    ncm.release_shared(a)
    assert a.c is None and _FakeComm.made[0].closed == 1
    c = ncm.shared_communicator(0, 1, dev, ext=_FakeExt(), watchdog=False)
    assert c is not a and len(_FakeComm.made) == 2  # a closed one is replaced
    ncm.release_shared(c)
    assert not ncm._SHARED


def test_ring_and_strategy_use_the_shared_communicator():
    """The secure ring no longer builds its own communicator (a second RCCL context without a
    watchdog): it asks for the rank's shared one, created with the watchdog default."""
    import inspect
    from idc_models_amd.parallel import comm, strategy
    assert "shared_communicator" in inspect.getsource(comm._native_ring)
    assert "watchdog=False" not in inspect.getsource(comm._native_ring)
    assert "shared_communicator" in inspect.getsource(strategy.MirroredStrategy.__init__)
