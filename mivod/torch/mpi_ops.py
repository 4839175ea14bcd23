"""Named collectives on torch tensors (parity: horovod/torch/mpi_ops.py,
SURVEY.md §2.2 U18/U22): ``allreduce[_][_async]``, ``allgather[_async]``,
``broadcast[_][_async]``, ``alltoall``, ``synchronize``, ``poll``.

Non-inplace ops are differentiable like horovod's: the gradient of allreduce is
an allreduce of the gradient (same op), of allgather the matching slice of an
allreduced gradient, of broadcast the gradient summed onto the root.
"""
from __future__ import annotations

import torch

from ..common import basics
from ..ops.compression import Compression
from ..parallel import collectives as C
from ..parallel.engine import ALLGATHER, ALLREDUCE, ALLTOALL, BROADCAST, HorovodInternalError

Average, Sum, Adasum = C.Average, C.Sum, C.Adasum


def _engine():
    st = basics.state()
    if not st.initialized or st.engine is None:
        raise ValueError(basics._NOT_INIT)
    return st.engine


def _resolve_op(average, op):
    if op is not None and average is not None:
        raise ValueError("The op parameter supersedes average. Please provide only one of them.")
    if op is None:
        op = Average if (average is None or average) else Sum
    return op


def handle_average_backwards_compatibility(op, average):
    return _resolve_op(average, op)


# ---------------------------------------------------------------- allreduce
def allreduce_async(tensor, average=None, name=None, op=None, prescale_factor=1.0,
                    postscale_factor=1.0, compression=Compression.none):
    op = _resolve_op(average, op)
    out = torch.empty_like(tensor, memory_format=torch.contiguous_format)
    return _engine().enqueue(ALLREDUCE, tensor, out, name, op, 0, compression, prescale_factor,
                             postscale_factor)


def allreduce_async_(tensor, average=None, name=None, op=None, prescale_factor=1.0,
                     postscale_factor=1.0, compression=Compression.none):
    op = _resolve_op(average, op)
    return _engine().enqueue(ALLREDUCE, tensor, tensor, name, op, 0, compression, prescale_factor,
                             postscale_factor)


class _AllreduceFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tensor, name, op, prescale, postscale, compression):
        ctx.op, ctx.pre, ctx.post, ctx.comp = op, prescale, postscale, compression
        h = allreduce_async(tensor, name=name, op=op, prescale_factor=prescale,
                            postscale_factor=postscale, compression=compression)
        return synchronize(h)

    @staticmethod
    def backward(ctx, grad):
        h = allreduce_async(grad.contiguous(), op=ctx.op, prescale_factor=ctx.pre,
                            postscale_factor=ctx.post, compression=ctx.comp)
        return synchronize(h), None, None, None, None, None


def allreduce(tensor, average=None, name=None, compression=Compression.none, op=None,
              prescale_factor=1.0, postscale_factor=1.0):
    """Returns the reduction of ``tensor`` over all ranks (Average by default)."""
    op = _resolve_op(average, op)
    if tensor.requires_grad and torch.is_grad_enabled():
        return _AllreduceFn.apply(tensor, name, op, prescale_factor, postscale_factor, compression)
    return synchronize(allreduce_async(tensor, name=name, op=op, prescale_factor=prescale_factor,
                                       postscale_factor=postscale_factor, compression=compression))


def allreduce_(tensor, average=None, name=None, op=None, prescale_factor=1.0,
               postscale_factor=1.0, compression=Compression.none):
    op = _resolve_op(average, op)
    return synchronize(allreduce_async_(tensor, name=name, op=op, prescale_factor=prescale_factor,
                                        postscale_factor=postscale_factor,
                                        compression=compression))


# ---------------------------------------------------------------- allgather
def allgather_async(tensor, name=None):
    return _engine().enqueue(ALLGATHER, tensor, None, name)


class _AllgatherFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tensor, name):
        ctx.dim0 = tensor.shape[0] if tensor.dim() > 0 else 1
        out = synchronize(allgather_async(tensor, name=name))
        sizes = synchronize(allgather_async(
            torch.tensor([ctx.dim0], dtype=torch.int64, device=tensor.device)))
        ctx.sizes = sizes.tolist()
        return out

    @staticmethod
    def backward(ctx, grad):
        g = synchronize(allreduce_async(grad.contiguous(), op=Sum))
        r = basics.rank()
        off = sum(ctx.sizes[:r])
        return g.narrow(0, off, ctx.dim0), None


def allgather(tensor, name=None):
    """Concatenation of ``tensor`` from all ranks along dim 0 (ragged allowed)."""
    if tensor.requires_grad and torch.is_grad_enabled():
        return _AllgatherFn.apply(tensor, name)
    return synchronize(allgather_async(tensor, name=name))


# ---------------------------------------------------------------- broadcast
def broadcast_async(tensor, root_rank, name=None):
    out = tensor.clone()
    return _engine().enqueue(BROADCAST, tensor, out, name, root=root_rank)


def broadcast_async_(tensor, root_rank, name=None):
    return _engine().enqueue(BROADCAST, tensor, tensor, name, root=root_rank)


class _BroadcastFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tensor, root_rank, name):
        ctx.root = root_rank
        return synchronize(broadcast_async(tensor, root_rank, name))

    @staticmethod
    def backward(ctx, grad):
        g = synchronize(allreduce_async(grad.contiguous(), op=Sum))
        if basics.rank() != ctx.root:
            g = g * 0
        return g, None, None


def broadcast(tensor, root_rank, name=None):
    if tensor.requires_grad and torch.is_grad_enabled():
        return _BroadcastFn.apply(tensor, root_rank, name)
    return synchronize(broadcast_async(tensor, root_rank, name))


def broadcast_(tensor, root_rank, name=None):
    return synchronize(broadcast_async_(tensor, root_rank, name))


# ---------------------------------------------------------------- alltoall
def alltoall_async(tensor, splits=None, name=None):
    if splits is not None and torch.is_tensor(splits):
        splits = [int(x) for x in splits.tolist()]
    return _engine().enqueue(ALLTOALL, tensor, None, name, splits=splits)


def alltoall(tensor, splits=None, name=None):
    return synchronize(alltoall_async(tensor, splits, name))


# ---------------------------------------------------------------- handles
def poll(handle) -> bool:
    return _engine().poll(handle)


def synchronize(handle):
    return _engine().synchronize(handle)


def join(device=-1):
    """Barrier across ranks (horovod >=0.20 ``join``); returns the last rank."""
    C.barrier()
    return basics.size() - 1


__all__ = ["allreduce", "allreduce_", "allreduce_async", "allreduce_async_", "allgather",
           "allgather_async", "broadcast", "broadcast_", "broadcast_async", "broadcast_async_",
           "alltoall", "alltoall_async", "poll", "synchronize", "join", "Average", "Sum", "Adasum",
           "HorovodInternalError"]
