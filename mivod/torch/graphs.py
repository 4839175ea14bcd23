"""HIP-graph capture of a whole data-parallel training step.

``make_graphed_step(step_fn, optimizer)`` captures forward, backward, the
bucketed gradient allreduce (RCCL on the comm stream, forked from and joined
back into the capture stream by events) and the fused optimizer update into ONE
HIP graph, then replays it: one graph launch per step instead of ~700 kernel
launches (ResNet-50) plus the Python work of autograd, the backward hooks and
the bucket schedule.  This is mivod's answer to a tracing compiler: the step's
kernels (the hand-written gfx950 ones plus MIOpen / hipBLASLt) are frozen into a
graph — no Triton, no torch.compile.

What makes a replay equal to an eager step:

* **Device-side hyperparameters.**  While the step is captured the fused
  optimizer kernels are launched with a 16-byte device block per arena,
  ``[lr, first, bias_correction1, bias_correction2]`` (``dyn`` in
  csrc/kernels/mv_kernels.hip), instead of baked launch arguments.  Before
  every replay the host refills it from the param groups — so LR warmup and
  schedules keep working — through a ring of pinned staging buffers (async
  H2D; a slot is reused only after its copy has completed).
* **Host bookkeeping replayed in Python.**  Arena step counters (Adam bias
  correction, SGD momentum seeding), the DistributedOptimizer step count and
  the fused BatchNorm modules' step counters advance per replay exactly as an
  eager step advances them; what the capture itself advanced is rolled back.
* **Static inputs / outputs.**  Tensors the step reads (images, labels) are
  captured by address: refill them in place (``x.copy_(batch)``) between
  replays.  ``step_fn``'s return value is a static output that every replay
  overwrites.
* **Warmup first.**  ``warmup`` eager steps (real training steps) run on a side
  stream before capture, so MIOpen's find, chunk tables, workspaces and RCCL
  communicators exist; nothing inside the step may synchronize the host.

The bucket schedule is frozen by the capture (autotuning is switched off) and
every replay is a full step, so ``backward_passes_per_step`` must be 1.

Measured (1x MI355X, ROCm 7): ResNet-50 replays are correct but not faster than
eager at bs 128-1024 — the step is GPU-bound and ROCm replays the two-stream
graph DAG (compute + comm stream) ~15 us/node slower; see GraphedStep.__init__.
Graph mode pays off for launch-bound steps (small models / small batches).
Eager steps after the capture remain valid (they use the scalar arguments).
Parity: horovod 0.18.1 has no graph mode — an MI355X-native addition
("HIP graphs for launch overhead").
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional

import torch

from ..optim.fused import FusedOptimizer


class _DynRing:
    """Pinned host staging for the per-arena dyn blocks: slot k is rewritten only
    after the H2D copy issued from it has completed."""

    def __init__(self, n_floats: int, depth: int = 4):
        self.bufs = [torch.empty(max(n_floats, 1), dtype=torch.float32).pin_memory()
                     for _ in range(depth)]
        self.events: List[Optional[torch.cuda.Event]] = [None] * depth
        self.k = 0

    def acquire(self):
        k = self.k
        self.k = (k + 1) % len(self.bufs)
        if self.events[k] is not None:
            self.events[k].synchronize()
        return k, self.bufs[k]

    def release(self, k: int):
        ev = torch.cuda.Event()
        ev.record()
        self.events[k] = ev


def dyn_values(a) -> List[float]:
    """[lr, first, bc1, bc2] of arena ``a`` for its current ``a.step``."""
    g = a.group
    bc1 = bc2 = 1.0
    betas = g.get("betas")
    if betas is not None:
        bc1 = 1.0 - float(betas[0]) ** a.step
        bc2 = 1.0 - float(betas[1]) ** a.step
    return [float(g["lr"]), 1.0 if a.step == 1 else 0.0, bc1, bc2]


class GraphedStep:
    """A captured training step; calling it replays the step and returns the
    static outputs of ``step_fn``."""

    _force_fork = False     # tests: keep the comm-stream fork even with one rank
    _side_warmup = os.environ.get("MIVOD_GRAPH_SIDE_WARMUP", "0") == "1"

    def __init__(self, step_fn: Callable, optimizer, model: Optional[torch.nn.Module] = None,
                 warmup: int = 3, pool=None):
        from .optimizer import _DistributedOptimizerMixin
        if not torch.cuda.is_available():
            raise RuntimeError("make_graphed_step needs a GPU (HIP graphs)")
        if not isinstance(optimizer, FusedOptimizer):
            raise TypeError("make_graphed_step needs a mivod.optim.Fused* optimizer (optionally "
                            "wrapped in DistributedOptimizer): its kernels read the per-step "
                            "hyperparameters from device memory during replays")
        if warmup < 1:
            raise ValueError("make_graphed_step needs at least one eager warmup step")
        self.dist = isinstance(optimizer, _DistributedOptimizerMixin)
        if self.dist:
            if getattr(optimizer, "_mvd_guard", False):
                raise ValueError("make_graphed_step: the fp16-wire overflow guard reads its flag "
                                 "on the host between steps; pass overflow_guard=False")
            if optimizer._mvd_bpps != 1:
                raise ValueError("graph mode needs backward_passes_per_step == 1")
            optimizer._mvd_autotune = None         # the captured bucket plan is final
        self.step_fn = step_fn
        self.opt = optimizer
        self.bns = [m for m in (model.modules() if model is not None else [])
                    if hasattr(m, "_mv_steps")]

        # 1. eager warmup (real training steps)
        if self._side_warmup:
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(warmup):
                    step_fn()
            torch.cuda.current_stream().wait_stream(side)
        else:
            for _ in range(warmup):
                step_fn()
        torch.cuda.synchronize()

        self.arenas = optimizer._mv_build()
        for a in self.arenas:
            if a.dyn is None:
                a.dyn = torch.zeros(4, dtype=torch.float32, device=a.device)
        self.ring = _DynRing(4 * len(self.arenas))

        # 2. capture with dyn-reading optimizer kernels; roll back host bookkeeping
        steps0 = [a.step for a in self.arenas]
        bn0 = [m._mv_steps for m in self.bns]
        mvd0 = optimizer._mvd_steps if self.dist else 0
        self.graph = torch.cuda.CUDAGraph()
        optimizer._mv_graph = True
        # The bucket launches fork onto the comm stream inside the capture (the same
        # schedule as eager).  Measured on ROCm 7 / MI355X: that two-stream DAG
        # replays every node ~15 us slower than a one-stream chain (ResNet-50 bs512:
        # eager 48.2 ms, graph 59.1 ms/step; a one-stream fwd+bwd graph replays at
        # eager speed, scripts/debug/graph_speed.py).  A one-rank capture with the
        # updates inline on the capture stream (MIVOD_GRAPH_INLINE=1) replays at
        # 47.1 ms but produced non-finite MIOpen weight gradients from the second
        # replay on (scripts/debug/graph_alloc.py), so it stays opt-in.
        inline = (self.dist and getattr(optimizer, "_mvd_size", 1) == 1
                  and os.environ.get("MIVOD_GRAPH_INLINE", "0") == "1"
                  and not self._force_fork)
        if inline:
            optimizer._mvd_inline = True
        try:
            with torch.cuda.graph(self.graph, pool=pool):
                self.outputs = step_fn()
        finally:
            optimizer._mv_graph = False
            if inline:
                optimizer._mvd_inline = False
        self.bn_incr = [m._mv_steps - s for m, s in zip(self.bns, bn0)]
        for a, s in zip(self.arenas, steps0):
            a.step = s
        for m, s in zip(self.bns, bn0):
            m._mv_steps = s
        if self.dist:
            optimizer._mvd_steps = mvd0
            optimizer._mvd_synchronized = False
        self.replays = 0

    def __call__(self):
        k, host = self.ring.acquire()
        vals = []
        for a in self.arenas:
            a.sync_master_if_modified()      # params edited in place since the last step
            a.step += 1
            vals.extend(dyn_values(a))
        host.copy_(torch.tensor(vals, dtype=torch.float32))
        for i, a in enumerate(self.arenas):
            a.dyn.copy_(host[4 * i:4 * i + 4], non_blocking=True)
        self.ring.release(k)
        self.graph.replay()
        self.opt._mv_end_step()
        for m, inc in zip(self.bns, self.bn_incr):
            m._mv_steps += inc
        if self.dist:
            self.opt._mvd_steps += 1
        self.replays += 1
        return self.outputs


def make_graphed_step(step_fn: Callable, optimizer, model: Optional[torch.nn.Module] = None,
                      warmup: int = 3, pool=None) -> GraphedStep:
    """Capture ``step_fn`` — forward, ``loss.backward()``, ``optimizer.step()``
    (and ``zero_grad``), returning e.g. the loss — into a HIP graph after
    ``warmup`` eager steps, and return a callable that replays it.

    ``model`` (optional) lets mivod's fused BatchNorm modules keep their step
    counters exact across replays.  Inputs are static: refill the tensors
    ``step_fn`` reads in place between calls."""
    return GraphedStep(step_fn, optimizer, model=model, warmup=warmup, pool=pool)
