"""Fault injection for failure-path tests (SURVEY.md §5 "Failure detection").

``MIVOD_FAULT="<rank>:<step>:<kind>[,...]"`` makes rank <rank> misbehave when
its DistributedOptimizer finishes step <step> (1-based):
``crash`` (exit 17 without cleanup), ``hang`` (sleep forever), ``raise``
(RuntimeError).  Used to check that the job ends instead of hanging: the
launcher tears every rank down when one exits non-zero; with
``HOROVOD_STALL_SHUTDOWN_TIME_SECONDS`` set, the surviving ranks' collectives
time out — the CPU ring's per-step I/O timeout, and on GPU the RCCL watchdog
thread of ``mivod._mvcomm`` (csrc/comm/comm.cc: ncclCommGetAsyncError polling +
ncclCommAbort of a collective older than the limit) — so they exit non-zero
and the launcher reaps the hung rank (tests/test_checkpoint_faults_autotune.py).
"""
from __future__ import annotations

import os
import time

_PLAN = None


def _plan():
    global _PLAN
    if _PLAN is None:
        _PLAN = []
        for item in os.environ.get("MIVOD_FAULT", "").split(","):
            item = item.strip()
            if not item:
                continue
            r, s, k = item.split(":")
            _PLAN.append((int(r), int(s), k))
    return _PLAN


def maybe_inject(rank: int, step: int) -> None:
    for r, s, k in _plan():
        if r == rank and s == step:
            if k == "crash":
                os._exit(17)
            if k == "hang":
                while True:
                    time.sleep(3600)
            if k == "raise":
                raise RuntimeError(f"mivod injected fault on rank {rank} at step {step}")
