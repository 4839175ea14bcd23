"""Flat-buffer collectives on the mivod process groups.

This is the data plane under both the static gradient schedule
(``mivod.torch.DistributedOptimizer``) and the negotiated named-op engine.
GPU tensors ride RCCL (torch.distributed backend "nccl" == RCCL on ROCm) over
xGMI; CPU tensors ride gloo.  Callers choose the HIP stream (the comm stream);
a collective here never blocks the host for GPU tensors.

Horovod parity: allreduce (Sum / Average / Adasum),
allgather (first-dim concat, ragged allowed), broadcast.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from ..common import basics

# horovod reduce ops (horovod/common/basics.py: Average / Sum / Adasum)
Average = 0
Sum = 1
Adasum = 2

_OP_NAMES = {Average: "Average", Sum: "Sum", Adasum: "Adasum"}


def op_name(op: int) -> str:
    return _OP_NAMES.get(op, str(op))


def _gloo_ok(dtype: torch.dtype) -> bool:
    return dtype not in (torch.bfloat16,)


def _native_gpu(t: torch.Tensor) -> bool:
    """GPU tensor on an RCCL world (False for MIVOD_TRANSPORT=gloo-gpu: GPU compute,
    gloo wire — the multi-rank-on-one-GPU test mode, which lacks AVG and bf16)."""
    return t.is_cuda and basics.state().backend != "gloo"


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
    if t.is_cuda:
        return st.engine_pg if engine else st.pg
    return st.engine_cpu_pg if engine else st.cpu_pg


def allreduce_(t: torch.Tensor, op: int = Sum, group=None, engine: bool = False,
               adasum_table=None) -> torch.Tensor:
    """In-place allreduce of a dense tensor.  ``Average`` divides by size
    (RCCL ncclAvg on GPU).  Adasum needs a chunk table of the per-tensor
    segments (``ops.kernels.make_chunk_table``)."""
    st = basics.state()
    if st.size == 1:
        return t
    pg = group or group_for(t, engine)
    if op == Adasum:
        from .adasum import adasum_allreduce_
        return adasum_allreduce_(t, adasum_table, pg)
    if (st.config is not None and st.config.hierarchical_allreduce and st.local_pg is not None
            and st.cross_pg is not None and group is None and not engine
            and t.is_cuda == (st.backend == "nccl")):
        return hierarchical_allreduce_(t, op)
    if t.is_cuda and st.backend != "gloo":
        rop = dist.ReduceOp.AVG if op == Average else dist.ReduceOp.SUM
        dist.all_reduce(t, op=rop, group=pg)
        return t
    ring = _ring(t, group, engine)
    if ring is not None:
        return ring.allreduce_(t, average=(op == Average))
    if _gloo_ok(t.dtype):
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=pg)
        if op == Average:
            if t.dtype.is_floating_point:
                t.div_(st.size)
            else:
                t.floor_divide_(st.size)
        return t
    w = t.float()
    dist.all_reduce(w, op=dist.ReduceOp.SUM, group=pg)
    if op == Average:
        w.div_(st.size)
    t.copy_(w)
    return t


def hierarchical_allreduce_(t: torch.Tensor, op: int = Sum) -> torch.Tensor:
    """HOROVOD_HIERARCHICAL_ALLREDUCE: intra-node reduce-scatter (xGMI), cross-node
    allreduce of each 1/local_size shard (the network carries 1/L of the bytes),
    intra-node allgather.  On CPU/gloo (no reduce-scatter) the same two-level
    structure runs as local allreduce + cross allreduce."""
    st = basics.state()
    L = st.local_size
    flat = t.view(-1) if t.is_contiguous() else t.contiguous().view(-1)
    if t.is_cuda:
        n = flat.numel()
        pad = (-n) % L
        work = flat if pad == 0 else torch.cat([flat, flat.new_zeros(pad)])
        shard = torch.empty(work.numel() // L, dtype=t.dtype, device=t.device)
        dist.reduce_scatter_tensor(shard, work, op=dist.ReduceOp.SUM, group=st.local_pg)
        dist.all_reduce(shard, op=dist.ReduceOp.SUM, group=st.cross_pg)
        dist.all_gather_into_tensor(work, shard, group=st.local_pg)
        if pad:
            flat.copy_(work[:n])
    else:
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


def allgather(t: torch.Tensor, group=None, engine: bool = False) -> torch.Tensor:
    """Concatenate ``t`` from every rank along dim 0 (first dims may differ)."""
    st = basics.state()
    if st.size == 1:
        return t.clone()
    ring = _ring(t, group, engine)
    if ring is not None:
        return ring.allgather(t)
    pg = group or group_for(t, engine)
    n = torch.tensor([t.shape[0] if t.dim() > 0 else 1], dtype=torch.int64,
                     device=t.device if t.is_cuda else "cpu")
    sizes = [torch.zeros_like(n) for _ in range(st.size)]
    dist.all_gather(sizes, n, group=pg)
    sizes = [int(s.item()) for s in sizes]
    src = t if t.dim() > 0 else t.reshape(1)
    rest = tuple(src.shape[1:])
    mx = max(sizes)
    work_dtype = src.dtype if (_native_gpu(t) or _gloo_ok(src.dtype)) else torch.float32
    pad = torch.zeros((mx,) + rest, dtype=work_dtype, device=src.device)
    pad[:src.shape[0]].copy_(src)
    outs = [torch.empty_like(pad) for _ in range(st.size)]
    dist.all_gather(outs, pad, group=pg)
    res = torch.cat([o[:s] for o, s in zip(outs, sizes)], dim=0)
    return res.to(t.dtype)


def broadcast_(t: torch.Tensor, root_rank: int, group=None, engine: bool = False) -> torch.Tensor:
    st = basics.state()
    if st.size == 1:
        return t
    ring = _ring(t, group, engine)
    if ring is not None:
        return ring.broadcast_(t, root_rank)
    pg = group or group_for(t, engine)
    if _native_gpu(t) or _gloo_ok(t.dtype):
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
    if st.size == 1:
        return t.clone()
    pg = group or group_for(t, engine)
    n = t.shape[0]
    if splits is None:
        if n % st.size:
            raise ValueError("alltoall: first dim must divide by size when splits is None")
        splits = [n // st.size] * st.size
    sp = torch.tensor(splits, dtype=torch.int64, device=t.device)
    rsp = torch.empty_like(sp)
    dist.all_to_all_single(rsp, sp, group=pg)
    rsplits = rsp.tolist()
    out = torch.empty((sum(rsplits),) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    dist.all_to_all_single(out, t.contiguous(), rsplits, splits, group=pg)
    return out


def barrier(group=None):
    st = basics.state()
    if st.size == 1:
        return
    dist.barrier(group=group or st.cpu_pg)
