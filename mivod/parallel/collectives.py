"""Flat-buffer collectives — the data plane under both the static gradient
schedule (``mivod.torch.DistributedOptimizer``) and the negotiated named-op
engine.

GPU tensors ride mivod's own RCCL communicator (``transport.RcclTransport``,
csrc/comm) over xGMI on the caller's HIP stream (the comm stream); every GPU
collective is one entry of the cross-rank issue order (``order.ORDER``), so the
hook-driven bucket schedule and the engine's named ops can share ONE
communicator without deadlocking.  CPU tensors ride the native TCP ring
(csrc/engine/ring.cc) or gloo.  A collective never blocks the host for GPU
tensors (RCCL transport).

Horovod parity: allreduce (Sum / Average / Adasum, plus
pre-scale), hierarchical allreduce, allgather (first-dim concat, ragged
allowed), broadcast, alltoall, barrier.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from ..common import basics
from . import transport as T
from .order import ORDER

# horovod reduce ops (horovod/common/basics.py: Average / Sum / Adasum) + internal Max/Min
Average = 0
Sum = 1
Adasum = 2
Max = 3
Min = 4

_OP_NAMES = {Average: "Average", Sum: "Sum", Adasum: "Adasum", Max: "Max", Min: "Min"}
_TOP = {Average: T.AVG, Sum: T.SUM, Max: T.MAX, Min: T.MIN}


def op_name(op: int) -> str:
    return _OP_NAMES.get(op, str(op))


def _gloo_ok(dtype: torch.dtype) -> bool:
    return dtype not in (torch.bfloat16,)


def _gpu_transport(t: torch.Tensor, group=None):
    """The GPU transport serving ``t`` (None for CPU tensors / no GPU plane)."""
    if not t.is_cuda:
        return None
    if group is not None and hasattr(group, "allreduce_"):
        return group
    return basics.state().gpu


def _ring(t: torch.Tensor, group, engine: bool):
    """The native TCP ring (csrc/engine/ring.cc) serving CPU tensors of the whole
    world, or None (GPU tensor, sub-group, MIVOD_CPU_TRANSPORT=gloo)."""
    st = basics.state()
    if t.is_cuda or group is not None or not st.rings:
        return None
    from .tcp_ring import supported
    return st.rings[1 if engine else 0] if supported(t) else None


def group_for(t: torch.Tensor, engine: bool = False):
    st = basics.state()
    return st.engine_cpu_pg if engine else st.cpu_pg


def _flat(t: torch.Tensor) -> torch.Tensor:
    return t.view(-1) if t.is_contiguous() else t.contiguous().view(-1)


def allreduce_(t: torch.Tensor, op: int = Sum, group=None, engine: bool = False,
               adasum_table=None, prescale: float = 1.0) -> torch.Tensor:
    """In-place allreduce of a dense tensor.  ``Average`` divides by size
    (ncclAvg on GPU), ``prescale`` multiplies every rank's contribution first
    (ncclRedOpCreatePreMulSum).  Adasum needs a chunk table of the per-tensor
    segments (``ops.kernels.make_chunk_table``)."""
    st = basics.state()
    tr = _gpu_transport(t, group)
    if tr is not None:
        with ORDER.issue(negotiated=engine):
            flat = _flat(t)
            if op == Adasum:
                from .adasum import adasum_allreduce_
                if prescale != 1.0:
                    flat.mul_(prescale)
                adasum_allreduce_(flat, adasum_table, tr)
            elif (st.mesh is not None and group is None and op in (Average, Sum)
                  and st.mesh.accepts(flat, _TOP[op])):
                st.mesh.allreduce_(flat, _TOP[op], prescale)     # small bucket: one xGMI hop
            elif (st.config is not None and st.config.hierarchical_allreduce and group is None
                  and _hier_ok(flat, op, prescale)
                  and st.gpu_local is not None and st.gpu_cross is not None):
                _hierarchical_gpu_(flat, op, prescale)
            else:
                tr.allreduce_(flat, _TOP[op], prescale)
            if flat.data_ptr() != t.data_ptr():
                t.copy_(flat.view_as(t))
        return t
    if prescale != 1.0:
        t.mul_(prescale)
    if st.size == 1:
        return t
    pg = group or group_for(t, engine)
    if op == Adasum:
        from .adasum import adasum_allreduce_
        return adasum_allreduce_(t, adasum_table)
    if (st.config is not None and st.config.hierarchical_allreduce and op in (Average, Sum)
            and st.local_pg is not None and st.cross_pg is not None and group is None
            and not engine):
        return _hierarchical_cpu_(t, op)
    ring = _ring(t, group, engine)
    if ring is not None and op in (Average, Sum):
        return ring.allreduce_(t, average=(op == Average))
    rop = {Max: dist.ReduceOp.MAX, Min: dist.ReduceOp.MIN}.get(op, dist.ReduceOp.SUM)
    if _gloo_ok(t.dtype):
        dist.all_reduce(t, op=rop, group=pg)
        if op == Average:
            if t.dtype.is_floating_point:
                t.div_(st.size)
            else:
                t.floor_divide_(st.size)
        return t
    w = t.float()
    dist.all_reduce(w, op=rop, group=pg)
    if op == Average:
        w.div_(st.size)
    t.copy_(w)
    return t


def _hier_ok(t: torch.Tensor, op: int, prescale: float) -> bool:
    """Ops the two-level schedule computes exactly: Sum / Average (integer
    tensors only as an unscaled Sum — the scale is a floating-point pass)."""
    if op not in (Average, Sum):
        return False
    return t.dtype.is_floating_point or (op == Sum and prescale == 1.0)


def _hierarchical_gpu_(flat: torch.Tensor, op: int, prescale: float) -> None:
    """HOROVOD_HIERARCHICAL_ALLREDUCE on GPU (Sum / Average only): intra-node
    reduce-scatter (xGMI), cross-node allreduce of each 1/local_size shard (the
    network carries 1/L of the bytes), intra-node allgather — RCCL calls on
    ncclCommSplit comms, all IN PLACE on ``flat`` (no padded copy).  The average
    and ``prescale`` are one scale of the SHARD (1/L of the buffer) by mivod's
    flat-cast kernel after the cross-node sum (the sum is linear), not a pass
    over the whole buffer.  (Not RCCL PreMulSum: RCCL 2.26 leaves the last
    element of an odd-length 1-rank PreMulSum unscaled — tests/
    test_multirank_gpu.py::test_gpu_rccl_communicator_world1 caught it.)  The
    ``n % L`` tail elements that do not split evenly take one small allreduce on
    the world communicator.  Max / Min never come here (they run flat)."""
    from ..ops import kernels as K
    st = basics.state()
    L = st.gpu_local.size
    scale = float(prescale) / (st.size if op == Average else 1)
    n = flat.numel()
    m = n - n % L
    if m:
        body = flat[:m]
        c = m // L
        shard = body[st.gpu_local.rank * c:(st.gpu_local.rank + 1) * c]
        st.gpu_local.reduce_scatter(shard, body, T.SUM)       # in place (recvbuf in sendbuf)
        st.gpu_cross.allreduce_(shard, T.SUM)
        if scale != 1.0:
            K.flat_cast(shard, shard, scale)
        st.gpu_local.allgather_into(body, shard)              # in place (sendbuf in recvbuf)
    if m < n:
        tail = flat[m:]
        st.gpu.allreduce_(tail, T.SUM)
        if scale != 1.0:
            K.flat_cast(tail, tail, scale)


def _hierarchical_cpu_(t: torch.Tensor, op: int = Sum) -> torch.Tensor:
    """The same two-level structure on CPU/gloo (local allreduce + cross allreduce)."""
    st = basics.state()
    flat = _flat(t)
    work = flat if _gloo_ok(flat.dtype) else flat.float()
    dist.all_reduce(work, op=dist.ReduceOp.SUM, group=st.local_pg)
    dist.all_reduce(work, op=dist.ReduceOp.SUM, group=st.cross_pg)
    if work is not flat:
        flat.copy_(work)
    if op == Average:
        flat.div_(st.size)
    if flat.data_ptr() != t.data_ptr():
        t.copy_(flat.view_as(t))
    return t


def hierarchical_allreduce_(t: torch.Tensor, op: int = Sum) -> torch.Tensor:
    st = basics.state()
    if op not in (Average, Sum):
        return allreduce_(t, op)          # Max / Min: flat (see _hierarchical_gpu_)
    if t.is_cuda and st.gpu_local is not None and st.gpu_cross is not None \
            and _hier_ok(t, op, 1.0):
        with ORDER.issue():
            flat = _flat(t)
            _hierarchical_gpu_(flat, op, 1.0)
            if flat.data_ptr() != t.data_ptr():
                t.copy_(flat.view_as(t))
        return t
    return _hierarchical_cpu_(t, op)


def allgather(t: torch.Tensor, group=None, engine: bool = False) -> torch.Tensor:
    """Concatenate ``t`` from every rank along dim 0 (first dims may differ)."""
    st = basics.state()
    tr = _gpu_transport(t, group)
    if tr is not None and tr.size > 1:
        with ORDER.issue(negotiated=engine):
            src = (t if t.dim() > 0 else t.reshape(1)).contiguous()
            n = torch.tensor([src.shape[0]], dtype=torch.int64, device=t.device)
            sizes_t = torch.empty(tr.size, dtype=torch.int64, device=t.device)
            tr.allgather_into(sizes_t, n)
            sizes = sizes_t.tolist()
            rest = tuple(src.shape[1:])
            mx = max(sizes)
            if all(s == mx for s in sizes):
                out = torch.empty((mx * tr.size,) + rest, dtype=src.dtype, device=src.device)
                tr.allgather_into(out, src)
                return out
            pad = torch.zeros((mx,) + rest, dtype=src.dtype, device=src.device)
            pad[:src.shape[0]].copy_(src)
            outs = torch.empty((mx * tr.size,) + rest, dtype=src.dtype, device=src.device)
            tr.allgather_into(outs, pad)
            parts = outs.view((tr.size, mx) + rest)
            return torch.cat([parts[i, :s] for i, s in enumerate(sizes)], dim=0)
    if st.size == 1 or tr is not None:
        return t.clone()
    ring = _ring(t, group, engine)
    if ring is not None:
        return ring.allgather(t)
    pg = group or group_for(t, engine)
    n = torch.tensor([t.shape[0] if t.dim() > 0 else 1], dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(st.size)]
    dist.all_gather(sizes, n, group=pg)
    sizes = [int(s.item()) for s in sizes]
    src = t if t.dim() > 0 else t.reshape(1)
    rest = tuple(src.shape[1:])
    mx = max(sizes)
    work_dtype = src.dtype if _gloo_ok(src.dtype) else torch.float32
    pad = torch.zeros((mx,) + rest, dtype=work_dtype)
    pad[:src.shape[0]].copy_(src)
    outs = [torch.empty_like(pad) for _ in range(st.size)]
    dist.all_gather(outs, pad, group=pg)
    res = torch.cat([o[:s] for o, s in zip(outs, sizes)], dim=0)
    return res.to(t.dtype)


def broadcast_(t: torch.Tensor, root_rank: int, group=None, engine: bool = False) -> torch.Tensor:
    st = basics.state()
    tr = _gpu_transport(t, group)
    if tr is not None:
        if tr.size == 1:
            return t
        with ORDER.issue(negotiated=engine):
            work = t if t.is_contiguous() else t.contiguous()
            tr.broadcast_(work, root_rank)
            if work is not t:
                t.copy_(work)
        return t
    if st.size == 1:
        return t
    ring = _ring(t, group, engine)
    if ring is not None:
        return ring.broadcast_(t, root_rank)
    pg = group or group_for(t, engine)
    if _gloo_ok(t.dtype):
        if t.is_contiguous():
            dist.broadcast(t, src=root_rank, group=pg)
        else:
            c = t.contiguous()
            dist.broadcast(c, src=root_rank, group=pg)
            t.copy_(c)
        return t
    w = t.float().contiguous()
    dist.broadcast(w, src=root_rank, group=pg)
    t.copy_(w)
    return t


def alltoall(t: torch.Tensor, splits: Optional[List[int]] = None, group=None,
             engine: bool = False) -> torch.Tensor:
    st = basics.state()
    tr = _gpu_transport(t, group)
    size = tr.size if tr is not None else st.size
    if size == 1:
        return t.clone()
    n = t.shape[0]
    if splits is None:
        if n % size:
            raise ValueError("alltoall: first dim must divide by size when splits is None")
        splits = [n // size] * size
    if len(splits) != size or sum(splits) != n:
        raise ValueError("alltoall: splits must have one entry per rank summing to dim 0")
    if tr is not None:
        with ORDER.issue(negotiated=engine):
            sp = torch.tensor(splits, dtype=torch.int64, device=t.device)
            rsp = torch.empty_like(sp)
            tr.alltoallv(rsp, sp, [1] * size, [1] * size)
            rsplits = rsp.tolist()
            out = torch.empty((sum(rsplits),) + tuple(t.shape[1:]), dtype=t.dtype,
                              device=t.device)
            tr.alltoallv(out, t.contiguous(), list(splits), rsplits)
        return out
    pg = group or group_for(t, engine)
    sp = torch.tensor(splits, dtype=torch.int64)
    rsp = torch.empty_like(sp)
    dist.all_to_all_single(rsp, sp, group=pg)
    rsplits = rsp.tolist()
    out = torch.empty((sum(rsplits),) + tuple(t.shape[1:]), dtype=t.dtype)
    dist.all_to_all_single(out, t.contiguous(), rsplits, splits, group=pg)
    return out


def barrier(group=None):
    """Barrier over the world.  On a GPU world the GPU plane takes part too (a
    1-element allreduce on the current stream, then a stream sync), so every
    rank's previously enqueued GPU collectives have been issued in order."""
    st = basics.state()
    if st.size == 1:
        return
    if group is None and st.gpu is not None:
        with ORDER.issue():
            st.gpu.barrier(st.device)
        return
    if group is None and st.rings:
        st.rings[0].barrier()
        return
    dist.barrier(group=group or st.cpu_pg)


def max_over_ranks(x: float) -> float:
    """max of a host float over all ranks (CPU plane; used for timing)."""
    st = basics.state()
    if st.size == 1:
        return float(x)
    v = allgather(torch.tensor([float(x)], dtype=torch.float64))
    return float(v.max())


def gpu_stats() -> dict:
    """Cumulative calls / bytes of the GPU transport (+ mesh; empty without one)."""
    st = basics.state()
    out = dict(st.gpu.stats()) if st.gpu is not None else {}
    if st.mesh is not None:
        out.update(st.mesh.stats())
        out["calls"] = out.get("calls", 0) + out["mesh_calls"]
    return out
