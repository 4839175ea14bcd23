"""One cross-rank-agreed issue order for every GPU collective of a process.

mivod has two producers of GPU collectives: *direct* calls that every rank
makes at the same program point without negotiation (the static gradient
schedule issued from backward hooks, ``broadcast_parameters``, barriers) and
*named* ops (``hvd.allreduce_async(...)`` and friends) that the background
engine negotiates through the coordinator.  Both go to ONE communicator on ONE
HIP stream, so every rank must issue them in the same global order — two
communicators with unordered issue is the classic RCCL/NCCL deadlock.

Protocol (all ranks run the same program):

* ``Q`` counts the GPU collectives this rank has issued (direct and named).
* A direct collective is not issued while this rank has a named GPU op that it
  submitted but has not yet received the coordinator's response for (it
  blocks; the engine cycle is a few ms).
* Every negotiation cycle reports this rank's ``Q``; the coordinator attaches
  ``E = max_r Q_r`` to its response list.  A named response runs when the local
  ``Q`` reaches ``E`` — immediately if it already has, otherwise right after the
  direct collective that brings ``Q`` to ``E`` (drained by the thread that issued
  it).

Why it is safe: a rank that submitted op A is frozen at its ``Q`` until A's
response arrives, and the same program point has the same ``Q`` on every rank,
so ``E`` is exactly that common ``Q`` and every rank runs A between the same two
direct collectives.  Named ops never wait for the end of a step, so
``hvd.allreduce`` between ``loss.backward()`` and ``optimizer.step()`` — or inside
a backward hook — cannot deadlock against the bucket schedule.

Parity: the role of horovod 0.18.1's single background-thread issue loop
(``operations.cc`` RunLoopOnce), without negotiating the
static gradient schedule every step.
"""
from __future__ import annotations

import contextlib
import threading
from typing import Callable, List, Tuple


class IssueOrder:
    def __init__(self):
        self.cv = threading.Condition(threading.RLock())
        self.q = 0                 # GPU collectives issued by this rank
        self.pending = 0           # named GPU ops submitted, response not yet received
        self.deferred: List[Tuple[int, int, Callable[[], None]]] = []
        self._seq = 0
        self._draining = False
        self.enabled = False       # multi-rank GPU world only
        self.waits = 0             # direct issues that had to wait for a response (stats)
        # called with the new Q after every issue (the native engine loop reports
        # it to the coordinator each cycle without taking this lock)
        self.on_position = None

    def reset(self, enabled: bool):
        with self.cv:
            self.q = 0
            self.pending = 0
            self.deferred = []
            self.enabled = enabled
            self.waits = 0
            if self.on_position is not None:
                self.on_position(0)

    # -------------------------------------------------------------- direct
    @contextlib.contextmanager
    def issue(self, negotiated: bool = False):
        """Bracket ONE logical GPU collective.  Direct (un-negotiated) issues wait
        until this rank has no named op outstanding at the coordinator."""
        if not self.enabled:
            yield
            return
        with self.cv:
            if not negotiated and self.pending > 0:
                self.waits += 1
                while self.pending > 0:
                    self.cv.wait()
            yield
            self.q += 1
            if self.on_position is not None:
                self.on_position(self.q)
            self._drain()

    # --------------------------------------------------------------- named
    def submitted(self, n: int = 1):
        if not self.enabled or n <= 0:
            return
        with self.cv:
            self.pending += n

    def position(self) -> int:
        with self.cv:
            return self.q

    def responded(self, exec_at: int, n_gpu: int, fns: List[Callable[[], None]]):
        """Responses for ``n_gpu`` named GPU tensors arrived with ``E = exec_at``;
        ``fns`` execute them (each issues its collectives through ``issue``)."""
        if not self.enabled:
            for fn in fns:
                fn()
            return
        with self.cv:
            self.pending -= n_gpu
            if self.pending < 0:
                self.pending = 0
            for fn in fns:
                self._seq += 1
                self.deferred.append((exec_at, self._seq, fn))
            self.deferred.sort(key=lambda x: (x[0], x[1]))
            self._drain()
            self.cv.notify_all()

    def _drain(self):
        if self._draining:
            return
        self._draining = True
        try:
            while self.deferred and self.deferred[0][0] <= self.q:
                _, _, fn = self.deferred.pop(0)
                fn()
        finally:
            self._draining = False


ORDER = IssueOrder()
