"""Bucket-size autotuning for the static gradient schedule (``HOROVOD_AUTOTUNE=1``).

Parity target: horovod's parameter manager, which tunes
the fusion threshold / cycle time by Bayesian optimisation on measured bytes/s.
On MI355X the knob that matters for the hook path is the bucket geometry
(first bucket vs. the rest: how early xGMI traffic starts vs. how many RCCL
launches): a small grid is enough.  Each candidate runs ``warmup`` + ``trial``
steps; rank 0 scores the median step time and broadcasts the winner so every
rank re-plans at the same step.  ``HOROVOD_AUTOTUNE_LOG`` gets one CSV row per
trial.
"""
from __future__ import annotations

import os
import statistics
import time
from typing import List, Optional, Tuple

DEFAULT_GRID: List[Tuple[float, float]] = [(2.0, 32.0), (1.0, 16.0), (4.0, 64.0), (2.0, 128.0),
                                           (8.0, 8.0)]


class BucketAutotuner:
    def __init__(self, grid=None, warmup: int = 2, trial: int = 5, log_path: str = ""):
        self.grid = list(grid or DEFAULT_GRID)
        self.warmup = warmup
        self.trial = trial
        self.log_path = log_path
        self.idx = 0
        self.times: List[float] = []
        self.results: List[Tuple[Tuple[float, float], float]] = []
        self.step_in_trial = 0
        self.last = None
        self.done = False
        self.best: Optional[Tuple[float, float]] = None

    def current(self) -> Tuple[float, float]:
        return self.grid[self.idx]

    def on_step_end(self, sync_fn) -> Optional[Tuple[float, float]]:
        """Called after every synchronize().  Returns a new (first_mb, bucket_mb)
        when the plan must change, else None.  ``sync_fn`` waits for the GPU."""
        if self.done:
            return None
        sync_fn()
        now = time.perf_counter()
        if self.last is not None and self.step_in_trial > self.warmup:
            self.times.append(now - self.last)
        self.last = now
        self.step_in_trial += 1
        if self.step_in_trial < self.warmup + self.trial + 1:
            return None
        med = statistics.median(self.times) if self.times else float("inf")
        self.results.append((self.current(), med))
        self._log(self.current(), med)
        self.times, self.step_in_trial, self.last = [], 0, None
        self.idx += 1
        if self.idx < len(self.grid):
            return self.current()
        self.done = True
        self.best = min(self.results, key=lambda r: r[1])[0]
        return self.best

    def _log(self, cand, med):
        if not self.log_path:
            return
        new = not os.path.exists(self.log_path)
        with open(self.log_path, "a") as f:
            if new:
                f.write("first_bucket_mb,bucket_mb,median_step_s\n")
            f.write(f"{cand[0]},{cand[1]},{med:.6f}\n")
