"""``import mivod.tensorflow as hvd`` — the ``horovod.tensorflow`` API (SURVEY.md
§2.2 U18, §2.6) on mivod's PyTorch-ROCm substrate.

There is no TensorFlow in this stack, so the "graph" objects map as follows:

* a TF tensor / variable            -> a ``torch.Tensor`` / ``torch.nn.Parameter``
* ``tf.IndexedSlices``               -> :class:`IndexedSlices` or a sparse COO tensor
* ``tf.global_variables()``          -> every variable of every live ``mivod.kerasfw``
  model and its optimizer slots (:func:`global_variables`)
* ``tf.GradientTape``                -> :class:`GradientTape` (records nothing; torch
  autograd already holds the graph, ``gradient()`` is ``torch.autograd.grad``)
* ``tf.train.SessionRunHook``        -> :class:`BroadcastGlobalVariablesHook` with the
  same ``begin`` / ``after_create_session`` entry points

Semantics kept from horovod 0.18 ``horovod/tensorflow/__init__.py``:
``allreduce`` of sparse slices is an allgather of values and indices (values
divided by ``size()`` when averaging); dense tensors are compressed, summed
and decompressed, then divided by ``size()`` when averaging.
``DistributedOptimizer.compute_gradients`` averages the gradients only when
``size() > 1``, and ``DistributedGradientTape.gradient`` does the same.
The data plane is mivod's negotiated engine (fusion buffer + K1 pack kernel on
GPU, RCCL over xGMI; the native TCP ring on CPU).

The reference reaches these only through ``horovod.tensorflow.keras``
(/root/reference/tensorflow2_keras_mnist.py:18); this module is for users of
the lower-level TF API.
"""
from __future__ import annotations

from typing import Iterable, List, Optional

import torch

from ..common.basics import (cross_rank, cross_size, gloo_enabled, init, is_initialized,
                             local_rank, local_size, mpi_enabled, mpi_threads_supported,
                             nccl_built, rank, rocm_built, shutdown, size)
from ..ops.compression import Compression
from ..torch import mpi_ops as _ops
from ..torch.functions import broadcast_parameters as _broadcast_tensors

Average, Sum, Adasum = _ops.Average, _ops.Sum, _ops.Adasum


class IndexedSlices:
    """Stand-in for ``tf.IndexedSlices``: rows ``values[i]`` of a tensor of
    ``dense_shape`` at row ``indices[i]`` (duplicates add)."""

    def __init__(self, values: torch.Tensor, indices: torch.Tensor, dense_shape=None):
        self.values = values
        self.indices = indices
        self.dense_shape = tuple(dense_shape) if dense_shape is not None else None

    def to_dense(self) -> torch.Tensor:
        if self.dense_shape is None:
            raise ValueError("IndexedSlices.to_dense needs dense_shape")
        out = self.values.new_zeros(self.dense_shape)
        out.index_add_(0, self.indices.long(), self.values)
        return out


def _is_sparse(t) -> bool:
    return isinstance(t, IndexedSlices) or (torch.is_tensor(t) and t.is_sparse)


def allreduce(tensor, average=None, device_dense: str = "", device_sparse: str = "",
              compression=Compression.none, op=None, name: Optional[str] = None):
    """Reduce ``tensor`` over all ranks (Average by default).

    Sparse input (:class:`IndexedSlices` or a sparse COO tensor) is allgathered
    (values and indices), as horovod does for ``tf.IndexedSlices``; the result
    keeps the input's sparse type.  ``device_dense`` / ``device_sparse`` are
    accepted for signature compatibility: placement follows the tensor."""
    op = _ops._resolve_op(average, op)
    if op == Adasum and _is_sparse(tensor):
        raise NotImplementedError("Adasum does not support sparse tensors")
    if isinstance(tensor, IndexedSlices):
        values = _ops.allgather(tensor.values.contiguous(),
                                name=None if name is None else f"{name}.values")
        indices = _ops.allgather(tensor.indices.contiguous(),
                                 name=None if name is None else f"{name}.indices")
        if op == Average:
            values = values / size()
        return IndexedSlices(values, indices, tensor.dense_shape)
    if torch.is_tensor(tensor) and tensor.is_sparse:
        sl = tensor.coalesce()
        out = allreduce(IndexedSlices(sl.values(), sl.indices().t().contiguous(), sl.shape),
                        op=op, name=name)
        return torch.sparse_coo_tensor(out.indices.t(), out.values, sl.shape).coalesce()
    compressed, ctx = compression.compress(tensor)
    summed = _ops.allreduce(compressed, name=name, op=Sum if op == Average else op)
    summed = compression.decompress(summed, ctx)
    if op == Average:
        summed = summed / size() if summed.dtype.is_floating_point else summed // size()
    return summed


def allgather(tensor, name: Optional[str] = None):
    """Concatenate ``tensor`` from all ranks along the first dimension."""
    return _ops.allgather(tensor, name=name)


def broadcast(tensor, root_rank: int, name: Optional[str] = None):
    """``tensor`` of ``root_rank`` on every rank (a new tensor)."""
    return _ops.broadcast(tensor, root_rank, name=name)


def alltoall(tensor, splits=None, name: Optional[str] = None):
    return _ops.alltoall(tensor, splits, name=name)


# ------------------------------------------------------------ global variables
def _models():
    """Live ``mivod.kerasfw`` models in creation order (registered by Model.__init__)."""
    from ..kerasfw.models import _LIVE_MODELS
    return sorted(_LIVE_MODELS, key=lambda m: m._mvd_seq)


def global_variables() -> List[torch.Tensor]:
    """Every variable of every live Keras-front-end model plus its optimizer's
    slot variables (the ``tf.global_variables()`` collection), in creation order."""
    out, seen = [], set()
    for m in _models():
        vs = list(m.variables)
        opt = getattr(m, "optimizer", None)
        if opt is not None and hasattr(opt, "variables"):
            vs += list(opt.variables())
        for v in vs:
            if id(v) not in seen:
                seen.add(id(v))
                out.append(v)
    return out


def broadcast_variables(variables: Iterable[torch.Tensor], root_rank: int = 0) -> None:
    """Assign ``root_rank``'s value to every variable in place (one fused broadcast)."""
    _broadcast_tensors([v for v in variables if torch.is_tensor(v)], root_rank)


def broadcast_global_variables(root_rank: int = 0) -> None:
    """Broadcast :func:`global_variables` (and each optimizer's step counter and
    learning rate) from ``root_rank``."""
    from ..keras import broadcast_global_variables as _keras_bcast
    for m in _models():
        if getattr(m, "optimizer", None) is not None:
            _keras_bcast(root_rank, model=m)     # variables + optimizer slots/step/lr
        else:
            broadcast_variables(m.variables, root_rank)


class BroadcastGlobalVariablesHook:
    """``tf.train.SessionRunHook`` equivalent: broadcasts the global variables
    once, when the session is created (``begin`` + ``after_create_session``)."""

    def __init__(self, root_rank: int, device: str = ""):
        self.root_rank = root_rank
        self.device = device
        self._done = False

    def begin(self):
        self._done = False

    def after_create_session(self, session=None, coord=None):
        if not self._done:
            broadcast_global_variables(self.root_rank)
            self._done = True

    def before_run(self, run_context=None):
        return None

    def after_run(self, run_context=None, run_values=None):
        return None

    def end(self, session=None):
        return None


# ------------------------------------------------------------------ optimizers
def _reduce_grads(grads, name, device_dense, device_sparse, compression, sparse_as_dense, op):
    if size() <= 1:
        return list(grads)
    out, handles = [], []
    for i, g in enumerate(grads):
        if g is None:
            handles.append(None)
            continue
        if sparse_as_dense and _is_sparse(g):
            g = g.to_dense()
        if _is_sparse(g) or op == Adasum:
            handles.append(("sync", allreduce(g, op=op, compression=compression,
                                              name=f"{name}_Allreduce/{i}")))
            continue
        # dense: one async submit per gradient so the engine fuses them into one
        # collective per dtype (fusion buffer + K1 pack kernel on GPU)
        c, ctx = compression.compress(g.contiguous())
        handles.append(("async", _ops.allreduce_async(c, op=op, name=f"{name}_Allreduce/{i}"),
                        ctx))
    for h in handles:
        if h is None:
            out.append(None)
        elif h[0] == "sync":
            out.append(h[1])
        else:
            out.append(compression.decompress(_ops.synchronize(h[1]), h[2]))
    return out


class DistributedOptimizer:
    """Wraps an optimizer with ``compute_gradients`` / ``apply_gradients``
    (``mivod.kerasfw`` optimizers, or any object offering ``apply_gradients``):
    ``compute_gradients`` averages the gradients across ranks before they are
    returned; everything else is delegated to the wrapped optimizer."""

    def __init__(self, optimizer, name: Optional[str] = None, use_locking: bool = False,
                 device_dense: str = "", device_sparse: str = "",
                 compression=Compression.none, sparse_as_dense: bool = False, op=Average):
        self._optimizer = optimizer
        self._name = name or f"Distributed{type(optimizer).__name__}"
        self._device_dense = device_dense
        self._device_sparse = device_sparse
        self._compression = compression
        self._sparse_as_dense = sparse_as_dense
        self._op = op

    def compute_gradients(self, loss, var_list, *args, **kwargs):
        var_list = list(var_list)
        if hasattr(self._optimizer, "compute_gradients"):
            gv = list(self._optimizer.compute_gradients(loss, var_list, *args, **kwargs))
            grads, variables = [g for g, _ in gv], [v for _, v in gv]
        elif hasattr(self._optimizer, "get_gradients"):
            grads, variables = list(self._optimizer.get_gradients(loss, var_list)), var_list
        else:
            grads = list(torch.autograd.grad(loss, var_list, allow_unused=True))
            variables = var_list
        grads = _reduce_grads(grads, self._name, self._device_dense, self._device_sparse,
                              self._compression, self._sparse_as_dense, self._op)
        return list(zip(grads, variables))

    def apply_gradients(self, grads_and_vars, *args, **kwargs):
        return self._optimizer.apply_gradients(grads_and_vars, *args, **kwargs)

    def minimize(self, loss, var_list):
        return self.apply_gradients(self.compute_gradients(loss, var_list))

    def get_slot(self, *args, **kwargs):
        return self._optimizer.get_slot(*args, **kwargs)

    def get_slot_names(self, *args, **kwargs):
        return self._optimizer.get_slot_names(*args, **kwargs)

    def variables(self, *args, **kwargs):
        return self._optimizer.variables(*args, **kwargs)

    def __getattr__(self, item):
        return getattr(self.__dict__["_optimizer"], item)


class GradientTape:
    """``tf.GradientTape`` on torch autograd: the graph is already recorded by
    the tensors themselves, so the tape only scopes ``torch.enable_grad``."""

    def __init__(self, persistent: bool = False, watch_accessed_variables: bool = True):
        self._persistent = persistent
        self._ctx = None

    def __enter__(self):
        self._ctx = torch.enable_grad()
        self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        return self._ctx.__exit__(*exc)

    def watch(self, tensor):
        pass

    def gradient(self, target, sources, output_gradients=None):
        single = torch.is_tensor(sources)
        srcs = [sources] if single else list(sources)
        grads = torch.autograd.grad(target, srcs, grad_outputs=output_gradients,
                                    retain_graph=self._persistent, allow_unused=True)
        return grads[0] if single else list(grads)


class _DistributedGradientTape:
    def __init__(self, tape, device_dense, device_sparse, compression, sparse_as_dense, op):
        self._tape = tape
        self._args = (device_dense, device_sparse, compression, sparse_as_dense, op)

    def __enter__(self):
        self._tape.__enter__()
        return self

    def __exit__(self, *exc):
        return self._tape.__exit__(*exc)

    def watch(self, tensor):
        return self._tape.watch(tensor)

    def gradient(self, target, sources, output_gradients=None):
        single = torch.is_tensor(sources)
        grads = self._tape.gradient(target, sources, output_gradients)
        grads = _reduce_grads([grads] if single else grads, "DistributedGradientTape",
                              *self._args)
        return grads[0] if single else grads


def DistributedGradientTape(gradtape, device_dense: str = "", device_sparse: str = "",
                            compression=Compression.none, sparse_as_dense: bool = False,
                            op=Average):
    """Wrap a :class:`GradientTape` so ``gradient()`` returns rank-averaged gradients."""
    return _DistributedGradientTape(gradtape, device_dense, device_sparse, compression,
                                    sparse_as_dense, op)


__all__ = ["init", "shutdown", "is_initialized", "size", "local_size", "rank", "local_rank",
           "cross_rank", "cross_size", "mpi_threads_supported", "mpi_enabled", "gloo_enabled",
           "nccl_built", "rocm_built", "allreduce", "allgather", "broadcast", "alltoall",
           "broadcast_variables", "broadcast_global_variables", "global_variables",
           "BroadcastGlobalVariablesHook", "DistributedOptimizer", "DistributedGradientTape",
           "GradientTape", "IndexedSlices", "Compression", "Average", "Sum", "Adasum"]
