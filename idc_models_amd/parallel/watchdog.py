"""Host watchdog for the native RCCL communicator (SURVEY §5 "failure detection").

A data-parallel step enqueues its gradient all-reduces on the communicator's stream from inside
the C++ plan (``parallel/native_comm.py``, ``csrc/runtime/plan.cpp`` OP_ALLREDUCE).  If a peer rank
dies, those collectives never complete: every surviving rank would block forever in its next
device synchronisation.  The watchdog turns that into an error:

* after each step the runtime calls ``mark()``: the communicator records an event on its stream
  behind the step's collectives (``Communicator::mark``; an outstanding older mark is kept, so the
  age measured is that of the oldest unfinished one);
* a daemon thread polls every ``poll_s`` seconds: RCCL's asynchronous error state
  (``check_async``) and the age of the outstanding mark (``mark_age``);
* on an asynchronous error, or a mark older than ``timeout_s``, it aborts the communicator
  (``ncclCommAbort``: the stuck collective kernels exit, so a blocked synchronisation returns) and
  records the failure; ``raise_if_failed()`` raises ``CommFailure`` on the training thread.  The
  fused runtime calls it at the top of every data-parallel step (``NativeCommunicator.check`` in
  ``FusedStep._train_step``) and again after issuing the step's collectives (``step_issued``).

The reference's equivalent is implicit: TF's collective executor timeouts around the NCCL
all-reduce of ``MirroredStrategy`` (``/root/reference/dist_model_tf_vgg.py:115-117,135-138``).
The policy is written against a duck-typed communicator (``check_async``, ``mark_age``,
``abort``) so it is unit-tested on the CPU with a fake (``tests/test_watchdog.py``), and a real
gloo world of 2 on the CPU checks the abort-on-hang path end to end (same file).
"""
from __future__ import annotations

import threading
import time
from typing import Optional


class CommFailure(RuntimeError):
    """The communicator was aborted: a peer failed or a collective made no progress."""


class CommWatchdog:
    def __init__(self, comm, timeout_s: float = 300.0, poll_s: float = 1.0, name: str = "rccl"):
        self.comm = comm
        self.timeout_s = float(timeout_s)
        self.poll_s = float(poll_s)
        self.name = name
        self.error: Optional[str] = None
        self._stop = threading.Event()
        self._lock = threading.Lock()
        self._thread: Optional[threading.Thread] = None

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> "CommWatchdog":
        if self._thread is None:
            self._thread = threading.Thread(target=self._run, name=f"{self.name}-watchdog", daemon=True)
            self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        t, self._thread = self._thread, None
        if t is not None and t is not threading.current_thread():
            t.join(timeout=max(1.0, 2 * self.poll_s))

    # ------------------------------------------------------------------ policy
    def poll_once(self) -> Optional[str]:
        """One watchdog check (the thread's loop body; tests call it directly).  Returns the
        failure it detected and acted on, or None."""
        with self._lock:
            if self.error is not None or self.comm is None:
                return self.error
            reason = None
            try:
                self.comm.check_async()
            except Exception as e:  # RCCL reported a peer / proxy failure
                reason = f"asynchronous communicator error: {e}"
            if reason is None:
                age = float(self.comm.mark_age())
                if age > self.timeout_s:
                    reason = (f"collectives made no progress for {age:.0f} s "
                              f"(timeout {self.timeout_s:.0f} s): a peer rank is gone or hung")
            if reason is not None:
                try:
                    self.comm.abort()
                finally:
                    self.error = reason
            return reason

    def _run(self):
        while not self._stop.wait(self.poll_s):
            if self.poll_once() is not None:
                return

    # ------------------------------------------------------------------ training-thread side
    def mark(self):
        # checked under the lock: poll_once may abort the communicator between a check made
        # outside it and the mark (marking an aborted communicator raises a generic error)
        with self._lock:
            if self.error is None and self.comm is not None:
                self.comm.mark()

    def raise_if_failed(self):
        if self.error is not None:
            raise CommFailure(f"{self.name}: {self.error}")


def wait_with_watchdog(wd: CommWatchdog, done, poll_s: float = 0.05, timeout_s: Optional[float] = None):
    """Block until ``done()`` is true, raising CommFailure as soon as the watchdog aborts (a host
    wait on device work that depends on collectives, e.g. before reading a metric)."""
    t0 = time.monotonic()
    while not done():
        wd.raise_if_failed()
        if timeout_s is not None and time.monotonic() - t0 > timeout_s:
            raise TimeoutError("wait_with_watchdog: timed out")
        time.sleep(poll_s)
    wd.raise_if_failed()
