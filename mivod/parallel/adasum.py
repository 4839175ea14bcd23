"""Adasum reduction (Maleki et al., "Scaling Distributed Training with Adaptive
Summation", MLSys 2021) — parity with horovod ``op=hvd.Adasum``.

For two gradients a, b of one tensor (layer):

    adasum(a, b) = (1 - a.b / (2|a|^2)) a + (1 - a.b / (2|b|^2)) b

applied per *tensor segment* of a fused buffer, and over 2^k ranks by
recursive doubling: at level d each rank exchanges its current vector with
``rank ^ 2^d`` and both partners compute the identical merge (the lower rank's
vector is always ``a``), so every rank ends with bit-identical results.

GPU math is the hand-written gfx950 kernels K8 (``seg_dot3`` — deterministic
two-pass segmented Gram terms — and ``adasum_combine``); the exchange is an
RCCL send/recv pair over xGMI.  ``MIVOD_ADASUM_HIERARCHICAL=1`` gives horovod's
GPU semantics instead (intra-node average, Adasum across nodes).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from ..common import basics
from ..ops import kernels as K


def _is_pow2(n: int) -> bool:
    return n > 0 and (n & (n - 1)) == 0


def _exchange(send: torch.Tensor, recv: torch.Tensor, peer: int, pg) -> None:
    grank = peer
    if pg is not None and pg is not dist.group.WORLD:
        grank = dist.get_global_rank(pg, peer)
    if send.is_cuda and basics.state().backend == "gloo":
        # gloo-gpu test transport: gloo point-to-point moves host tensors only
        s_h, r_h = send.cpu(), torch.empty(recv.shape, dtype=recv.dtype)
        _exchange(s_h, r_h, peer, pg)
        recv.copy_(r_h)
        return
    ops = [dist.P2POp(dist.isend, send, grank, group=pg),
           dist.P2POp(dist.irecv, recv, grank, group=pg)]
    for w in dist.batch_isend_irecv(ops):
        w.wait()


def adasum_pairwise_(buf: torch.Tensor, table: K.ChunkTable, pg=None, rank: int = None,
                     size: int = None, workspace: dict = None) -> torch.Tensor:
    """Recursive-doubling Adasum of ``buf`` (flat) among ``size`` ranks of ``pg``."""
    if size is None:
        size = dist.get_world_size(pg) if pg is not None else basics.size()
    if rank is None:
        rank = dist.get_rank(pg) if pg is not None else basics.rank()
    if size == 1:
        return buf
    if not _is_pow2(size):
        raise ValueError(f"Adasum requires a power-of-2 number of ranks, got {size}")
    ws = workspace if workspace is not None else {}
    wire = buf
    if not buf.is_cuda and buf.dtype == torch.bfloat16:
        wire = buf.float()   # CPU reference path computes in fp32
    other = torch.empty_like(wire)
    d = 1
    while d < size:
        peer = rank ^ d
        _exchange(wire, other, peer, pg)
        if rank < peer:
            a, b = wire, other
        else:
            a, b = other, wire
        dots = K.seg_dot3(a, b, table, ws)
        if rank < peer:
            K.adasum_combine(wire, other, table, dots)
        else:
            # result must equal combine(a=other, b=wire): compute into `other`, then swap
            K.adasum_combine(other, wire, table, dots)
            wire, other = other, wire
        d <<= 1
    if wire is not buf:
        buf.copy_(wire)
    return buf


def adasum_allreduce_(buf: torch.Tensor, table, pg=None) -> torch.Tensor:
    st = basics.state()
    if table is None:
        table = K.make_chunk_table([buf.numel()], buf.device)
    if os.environ.get("MIVOD_ADASUM_HIERARCHICAL", "0") == "1" and st.local_pg is not None:
        # horovod GPU semantics: average within the node, Adasum across nodes
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=st.local_pg)
        buf.div_(st.local_size)
        return adasum_pairwise_(buf, table, st.cross_pg, st.cross_rank, st.cross_size)
    return adasum_pairwise_(buf, table, pg)
