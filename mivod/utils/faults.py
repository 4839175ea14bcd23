"""Fault injection for failure-path tests (SURVEY.md §5 "Failure detection").

``MIVOD_FAULT="<rank>:<step>:<kind>[,...]"`` makes rank <rank> misbehave when
its DistributedOptimizer finishes step <step> (1-based):
``crash`` (exit 17 without cleanup), ``hang`` (sleep forever), ``raise``
(RuntimeError).  Used to check that the launcher tears the job down and that
the stall inspector / RCCL watchdog report instead of hanging silently.
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
