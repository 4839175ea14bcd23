"""Adasum reduction (Maleki et al., "Scaling Distributed Training with Adaptive
Summation", MLSys 2021) — parity with horovod ``op=hvd.Adasum`` (SURVEY.md §2.2
U11; BASELINE.json config 5: BERT-Large with fp16 compression + Adasum).

For two gradients a, b of one tensor (layer):

    adasum(a, b) = (1 - a.b / (2|a|^2)) a + (1 - a.b / (2|b|^2)) b

applied per *tensor segment* of a fused buffer, over 2^k ranks, with the
bandwidth-optimal **vector-halving / distance-doubling** schedule:

* reduce phase, level i (distance d = 2^i): partners r and r^d share the range
  they hold; the lower rank keeps the first half, the upper the second, and
  each sends the half it gives away (wire dtype) and receives the partner's
  copy of the half it keeps.  The per-tensor Gram terms (a.b, |a|^2, |b|^2) of
  that level are partial sums over the kept piece, so they are summed over the
  2^(i+1) ranks that jointly hold the two vectors being merged (recursive
  doubling inside that group: i+1 exchanges of nseg*3 fp32 — no world-wide
  traffic).  Then each rank merges its kept piece.
* allgather phase: the levels in reverse, each rank swaps its finished piece
  with its partner until everyone holds the whole result.

Per rank that is S(N-1)/N bytes out in each phase — 2·S·(N-1)/N in total, the
same as a ring allreduce — instead of S·log2(N) for full-vector recursive
doubling.  The running merge is kept in **fp32** (``f``); only the wire (what is
sent) is compressed to the bucket's dtype, so fp16 compression rounds each
transmitted value once per hop instead of re-rounding the merge at every level.
Every output element is computed by exactly one rank and then copied bitwise,
so all ranks end with identical buffers.

GPU math is the hand-written gfx950 kernels K8: ``seg_dot3`` (deterministic
two-pass segmented Gram terms, fp32 x wire mixed), ``adasum_fcombine`` (merge on
the fp32 running sum) and ``flat_cast`` (wire casts); the exchange is a grouped
RCCL send/recv on the comm stream.  ``MIVOD_ADASUM_HIERARCHICAL=1`` gives
horovod's GPU semantics instead (intra-node average, Adasum across nodes).
"""
from __future__ import annotations

import math
import os
from typing import Dict

import torch

from ..common import basics
from ..ops import kernels as K
from . import transport as T

ALIGN = 64

# bytes this rank sent in the last call (tests / bench comm record)
LAST = {"exchange_bytes": 0, "dot_bytes": 0, "levels": 0}

_WS: Dict[tuple, torch.Tensor] = {}


def _is_pow2(n: int) -> bool:
    return n > 0 and (n & (n - 1)) == 0


def _half(n: int) -> int:
    """Split point of a range of n elements (64-element aligned when possible,
    identical on both partners)."""
    h = n // 2
    if n >= 2 * ALIGN:
        h = h // ALIGN * ALIGN
    return h


def _scratch(name: str, numel: int, dtype: torch.dtype, device) -> torch.Tensor:
    key = (name, str(device), dtype)
    t = _WS.get(key)
    if t is None or t.numel() < numel:
        t = torch.empty(max(numel, 1), dtype=dtype, device=device)
        _WS[key] = t
    return t[:numel]


def _clipped(table: K.ChunkTable, lo: int, hi: int, device) -> K.ChunkTable:
    """Chunk table of ``table``'s segments clipped to [lo, hi) (segment ids kept).

    Cached on ``table`` itself (``ChunkTable.derived``): the clipped tables live
    and die with their parent, so a new table that happens to reuse a freed
    one's address can never be served the old segment boundaries."""
    key = ("adasum-clip", lo, hi, str(device))
    t = table.derived.get(key)
    if t is None:
        sizes, offs = [], []
        for off, n in zip(table.seg_offsets, table.seg_sizes):
            a, b = max(off, lo), min(off + n, hi)
            sizes.append(max(0, b - a))
            offs.append(a if b > a else lo)
        t = K.make_chunk_table(sizes, device, offs)
        table.derived[key] = t
    return t


def _group_sum_(part: torch.Tensor, tr, rank: int, level: int) -> int:
    """Sum ``part`` (a rank's [nseg, 3] Gram partial) over the 2^(level+1) ranks
    that share ``rank >> (level+1)`` — the ranks jointly holding the two vectors
    merged at this level — by recursive doubling inside that group (level+1
    send/recv exchanges of nseg*3 floats).  Traffic is independent of the world
    size (the old scheme allreduced a zero-padded [world/2^(level+1), nseg, 3]
    buffer over the whole world).  IEEE addition is commutative, so both sides
    of every exchange compute the same bits: the group ends bitwise identical.
    Returns the bytes this rank sent."""
    recv = torch.empty_like(part)
    sent = 0
    for j in range(level + 1):
        tr.sendrecv(part, recv, rank ^ (1 << j))
        part.add_(recv)
        sent += part.numel() * 4
    return sent


def adasum_vhdd_(buf: torch.Tensor, table: K.ChunkTable, tr) -> torch.Tensor:
    """Vector-halving / distance-doubling Adasum of the flat ``buf`` among the
    ``tr.size`` ranks of transport ``tr`` (in place)."""
    n_ranks, rank = tr.size, tr.rank
    if n_ranks == 1:
        return buf
    if not _is_pow2(n_ranks):
        raise ValueError(f"Adasum requires a power-of-2 number of ranks, got {n_ranks}")
    S = buf.numel()
    dev = buf.device
    es = buf.element_size()
    f = _scratch("f32", S, torch.float32, dev)
    sw = _scratch("send", S, buf.dtype, dev)
    rw = _scratch("recv", S, buf.dtype, dev)
    K.flat_cast(buf, f)
    nseg = table.nseg
    levels = int(math.log2(n_ranks))
    exch = dots_b = 0
    ranges = []
    lo, hi = 0, S
    for i in range(levels):
        d = 1 << i
        peer = rank ^ d
        mid = lo + _half(hi - lo)
        lower = (rank & d) == 0
        klo, khi = (lo, mid) if lower else (mid, hi)
        glo, ghi = (mid, hi) if lower else (lo, mid)
        ranges.append((lo, hi))
        if ghi > glo:
            K.flat_cast(f[glo:ghi], sw[glo:ghi])
        tr.sendrecv(sw[glo:ghi], rw[klo:khi], peer)
        exch += (ghi - glo) * es
        tk = _clipped(table, klo, khi, dev)
        part = K.seg_dot3(f, rw, tk)                   # (f.r, |f|^2, |r|^2)
        if not lower:
            part = part[:, [0, 2, 1]]                   # -> (a.b, |a|^2, |b|^2)
        part = part.contiguous()
        assert part.shape == (nseg, 3)
        dots_b += _group_sum_(part, tr, rank, i)
        K.adasum_fcombine(f, rw, tk, part, swap=not lower)
        lo, hi = klo, khi
    if hi > lo:
        K.flat_cast(f[lo:hi], buf[lo:hi])
    for i in reversed(range(levels)):
        d = 1 << i
        peer = rank ^ d
        plo, phi = ranges[i]
        mid = plo + _half(phi - plo)
        lower = (rank & d) == 0
        mine = (plo, mid) if lower else (mid, phi)
        theirs = (mid, phi) if lower else (plo, mid)
        tr.sendrecv(buf[mine[0]:mine[1]], buf[theirs[0]:theirs[1]], peer)
        exch += (mine[1] - mine[0]) * es
    LAST.update(exchange_bytes=exch, dot_bytes=dots_b, levels=levels)
    return buf


class _CpuGroup:
    """Adasum's two primitives over a gloo group for CPU tensors (test tier)."""

    def __init__(self, pg):
        import torch.distributed as dist
        self.dist = dist
        self.pg = pg
        self.rank = dist.get_rank(pg)
        self.size = dist.get_world_size(pg)

    def sendrecv(self, send, recv, peer):
        gpeer = self.dist.get_global_rank(self.pg, peer)
        s, r = send, recv
        if s.dtype in (torch.bfloat16, torch.float16):
            s, r = s.view(torch.int16), r.view(torch.int16)
        ops = []
        if s.numel():
            ops.append(self.dist.P2POp(self.dist.isend, s.contiguous(), gpeer, group=self.pg))
        if r.numel():
            ops.append(self.dist.P2POp(self.dist.irecv, r, gpeer, group=self.pg))
        if ops:
            for w in self.dist.batch_isend_irecv(ops):
                w.wait()

    def allreduce_(self, t, op=T.SUM, prescale=1.0):
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.pg)
        return t


def adasum_allreduce_(buf: torch.Tensor, table, tr=None) -> torch.Tensor:
    """Adasum of ``buf`` over the world (GPU: mivod's transport; CPU: gloo)."""
    st = basics.state()
    if table is None:
        table = K.make_chunk_table([buf.numel()], buf.device)
    if buf.is_cuda:
        tr = tr or st.gpu
        if os.environ.get("MIVOD_ADASUM_HIERARCHICAL", "0") == "1" and \
                st.gpu_local is not None and st.gpu_cross is not None:
            # horovod GPU semantics: average within the node, Adasum across nodes
            st.gpu_local.allreduce_(buf, T.AVG)
            return adasum_vhdd_(buf, table, st.gpu_cross)
        return adasum_vhdd_(buf, table, tr)
    if st.size == 1:
        return buf
    work = buf
    return adasum_vhdd_(work, table, tr or _CpuGroup(st.cpu_pg))


def adasum_reference(vectors, table: K.ChunkTable) -> torch.Tensor:
    """Full-vector recursive-doubling Adasum of a list of 2^k flat fp32 tensors
    (the pairing structure of horovod's algorithm) — the numerics reference the
    tests compare the vector-halving implementation against."""
    vs = [v.float().clone() for v in vectors]
    n = len(vs)
    d = 1
    while d < n:
        nxt = list(vs)
        for r in range(n):
            p = r ^ d
            a, b = (vs[r], vs[p]) if r < p else (vs[p], vs[r])
            out = a.clone()
            dots = K.seg_dot3(a, b, table)
            K.adasum_combine(out, b, table, dots)
            nxt[r] = out
        vs = nxt
        d <<= 1
    return vs[0]


def _peek_cache() -> int:
    return len(_WS)
