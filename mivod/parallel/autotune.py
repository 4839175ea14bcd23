"""Bucket-size autotuning for the static gradient schedule (``HOROVOD_AUTOTUNE=1``).

Parity: horovod's parameter manager (``common/parameter_manager.cc`` +
``optim/bayesian_optimization.cc`` / ``gaussian_process.cc``, SURVEY.md §2.2
U14), which tunes the fusion threshold and cycle time by Bayesian optimisation
of measured throughput.  On MI355X the knobs that matter for the hook path are
the bucket geometry — the first bucket (how early xGMI traffic starts) and the
body bucket size (how many RCCL launches vs. how much exposed tail) — so the
search space is (log2 first_bucket_mb, log2 bucket_mb).

Procedure: a fixed seed design (``DEFAULT_GRID``), then ``bo_iters`` rounds of
Gaussian-process regression (RBF kernel on the log2 box, noise term,
standardised targets) with the expected-improvement acquisition maximised over
a dense lattice of the box; the winner is the best *measured* candidate.  Each
candidate runs ``warmup`` + ``trial`` steps and is scored by its median step
time.  Everything is deterministic, and rank 0's decision is broadcast so all
ranks re-plan at the same step.  ``HOROVOD_AUTOTUNE_LOG`` gets one CSV row per
trial.

``tune_rccl_ctas`` is the communicator half: at ``hvd.init()`` (HOROVOD_AUTOTUNE=1,
mivod RCCL transport, >1 rank) it builds one communicator per candidate CTA count
(``ncclConfig_t.minCTAs = maxCTAs``: the number of channels, i.e. rings over the 7
xGMI links, a collective spreads over), times the allreduce of the schedule's
bucket sizes on each, MAX-reduces the time over ranks (so every rank picks the same
winner without a broadcast) and keeps the fastest communicator.
"""
from __future__ import annotations

import math
import os
import statistics
import time
from typing import Callable, List, Optional, Tuple

import numpy as np

DEFAULT_GRID: List[Tuple[float, float]] = [(2.0, 32.0), (1.0, 16.0), (4.0, 64.0), (2.0, 128.0),
                                           (8.0, 8.0)]
# search box in log2(MB): first bucket 0.5..16 MB, body bucket 4..256 MB
BOX = ((-1.0, 4.0), (2.0, 8.0))


class GaussianProcess:
    """GP regression with an RBF kernel (fixed length scales on the log2 box)."""

    def __init__(self, length_scale=(1.0, 1.0), noise: float = 1e-2):
        self.ls = np.asarray(length_scale, dtype=np.float64)
        self.noise = noise

    def _k(self, a, b):
        d = (a[:, None, :] - b[None, :, :]) / self.ls
        return np.exp(-0.5 * (d ** 2).sum(-1))

    def fit(self, x, y):
        self.x = np.asarray(x, dtype=np.float64)
        y = np.asarray(y, dtype=np.float64)
        self.mu, self.sd = y.mean(), (y.std() if y.std() > 0 else 1.0)
        yn = (y - self.mu) / self.sd
        K = self._k(self.x, self.x) + self.noise * np.eye(len(self.x))
        self.L = np.linalg.cholesky(K)
        self.alpha = np.linalg.solve(self.L.T, np.linalg.solve(self.L, yn))
        return self

    def predict(self, xq):
        xq = np.asarray(xq, dtype=np.float64)
        ks = self._k(xq, self.x)
        mean = ks @ self.alpha
        v = np.linalg.solve(self.L, ks.T)
        var = np.clip(1.0 - (v ** 2).sum(0), 1e-12, None)
        return mean * self.sd + self.mu, np.sqrt(var) * self.sd


def expected_improvement(mean, std, best, xi: float = 0.01):
    """EI for MINIMISATION of the objective (step time)."""
    z = (best - mean - xi) / std
    cdf = 0.5 * (1.0 + np.vectorize(math.erf)(z / math.sqrt(2.0)))
    pdf = np.exp(-0.5 * z ** 2) / math.sqrt(2.0 * math.pi)
    return (best - mean - xi) * cdf + std * pdf


def _lattice(step: float = 0.25):
    a = np.arange(BOX[0][0], BOX[0][1] + 1e-9, step)
    b = np.arange(BOX[1][0], BOX[1][1] + 1e-9, step)
    return np.array([(u, v) for u in a for v in b])


class BucketAutotuner:
    def __init__(self, grid=None, warmup: int = 2, trial: int = 5, log_path: str = "",
                 bo_iters: int = 5, clock: Callable[[], float] = time.perf_counter):
        self.seed = list(grid or DEFAULT_GRID)
        self.warmup = warmup
        self.trial = trial
        self.log_path = log_path
        self.bo_iters = bo_iters
        self.clock = clock
        self.cand: Tuple[float, float] = self.seed[0]
        self.n_tried = 0
        self.times: List[float] = []
        self.results: List[Tuple[Tuple[float, float], float]] = []
        self.step_in_trial = 0
        self.last = None
        self.done = False
        self.best: Optional[Tuple[float, float]] = None
        self.last_ei = float("nan")

    def current(self) -> Tuple[float, float]:
        return self.cand

    # ------------------------------------------------------------------ search
    def _next_candidate(self) -> Optional[Tuple[float, float]]:
        if self.n_tried < len(self.seed):
            return self.seed[self.n_tried]
        if self.n_tried >= len(self.seed) + self.bo_iters:
            return None
        x = np.array([(math.log2(f), math.log2(b)) for (f, b), _ in self.results])
        y = np.array([t for _, t in self.results])
        gp = GaussianProcess().fit(x, y)
        q = _lattice()
        mean, std = gp.predict(q)
        ei = expected_improvement(mean, std, y.min() if len(y) else 0.0)
        tried = {(round(u, 3), round(v, 3)) for u, v in x}
        for i in np.argsort(-ei, kind="stable"):
            u, v = q[i]
            if (round(u, 3), round(v, 3)) not in tried:
                self.last_ei = float(ei[i])
                return (float(2.0 ** u), float(2.0 ** v))
        return None

    def on_step_end(self, sync_fn) -> Optional[Tuple[float, float]]:
        """Called after every synchronize().  Returns a new (first_mb, bucket_mb)
        when the plan must change, else None.  ``sync_fn`` waits for the GPU."""
        if self.done:
            return None
        sync_fn()
        now = self.clock()
        if self.last is not None and self.step_in_trial > self.warmup:
            self.times.append(now - self.last)
        self.last = now
        self.step_in_trial += 1
        if self.step_in_trial < self.warmup + self.trial + 1:
            return None
        med = statistics.median(self.times) if self.times else float("inf")
        self.results.append((self.cand, med))
        self._log(self.cand, med)
        self.times, self.step_in_trial, self.last = [], 0, None
        self.n_tried += 1
        nxt = self._next_candidate()
        if nxt is not None:
            self.cand = nxt
            return nxt
        self.done = True
        self.best = min(self.results, key=lambda r: r[1])[0]
        self.cand = self.best
        return self.best

    def _log(self, cand, med):
        if not self.log_path:
            return
        new = not os.path.exists(self.log_path)
        phase = "seed" if self.n_tried < len(self.seed) else "bayes"
        with open(self.log_path, "a") as f:
            if new:
                f.write("first_bucket_mb,bucket_mb,median_step_s,phase,expected_improvement\n")
            f.write(f"{cand[0]:.4g},{cand[1]:.4g},{med:.6f},{phase},{self.last_ei:.4g}\n")


# CTA (channel) counts tried by tune_rccl_ctas; 0 = RCCL's own choice
CTA_CANDIDATES: Tuple[int, ...] = (0, 4, 8, 16, 32)


def tune_rccl_ctas(make_comm: Callable[[int], object], time_fn: Callable[[object], float],
                   candidates=CTA_CANDIDATES, log_path: str = ""):
    """Pick the CTA count whose communicator runs the bucket allreduces fastest.

    ``make_comm(c)`` builds a communicator with minCTAs = maxCTAs = c (0: default) —
    collectively, on every rank; ``time_fn(comm)`` returns this schedule's allreduce
    time in seconds on that communicator, already MAX-reduced over ranks.  Returns
    (best_comm, best_c, [(c, seconds)]); the other communicators are closed."""
    results: List[Tuple[int, float]] = []
    best = None
    for c in candidates:
        comm = make_comm(c)
        t = float(time_fn(comm))
        results.append((c, t))
        if log_path:
            new = not os.path.exists(log_path)
            with open(log_path, "a") as f:
                if new:
                    f.write("rccl_ctas,allreduce_s\n")
                f.write(f"{c},{t:.6e}\n")
        if best is None or t < best[2]:
            if best is not None:
                best[0].close()
            best = (comm, c, t)
        else:
            comm.close()
    return best[0], best[1], results
