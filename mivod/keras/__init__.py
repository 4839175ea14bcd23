"""``import mivod.keras as hvd`` — horovod.keras-compatible API for the Keras
front end (``mivod.kerasfw``).

Parity: horovod 0.18.1 ``horovod/keras`` + ``horovod/_keras`` (SURVEY.md §2.2
U20/U21, §2.6), as used by /root/reference/mnist_keras.py:20,30,87,97 and
/root/reference/tensorflow2_keras_mnist.py:18,25,58,71-82.

``DistributedOptimizer(opt)`` returns an instance of a dynamically created
subclass of the optimizer's own class (same class name, so saved models load
with the plain ``load_model`` as the reference does at mnist_keras.py:124),
re-instantiated from ``opt.get_config()``, whose ``get_gradients`` averages the
gradients across ranks when ``size() > 1``, on a STATIC schedule checked across
ranks once (no per-step negotiation).  On GPU the averaging OVERLAPS the
backward pass (``_static.OverlappedGradientReducer``): tensor hooks armed
during ``torch.autograd.grad`` pack each completed bucket (K1 kernel) and the
high-priority comm stream reduces it over RCCL while autograd continues; the
result is zero-copy views into the reduced buckets.  On CPU, or with gradient
clipping, ``_static.StaticGradientReducer`` packs, reduces once per (device,
dtype) group (native TCP ring / gloo) and unpacks after the backward.
``MIVOD_KERAS_OVERLAP=0/1`` forces the choice.
``MIVOD_KERAS_NEGOTIATED=1`` submits every gradient to the negotiated engine under
``<Name>_Allreduce/<i>`` instead (horovod's per-tensor protocol).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..common.basics import (cross_rank, cross_size, init, is_initialized, local_rank,
                             local_size, mpi_threads_supported, rank, shutdown, size)
from ..ops.compression import Compression
from ..torch import mpi_ops as _ops
from ..torch.functions import broadcast_optimizer_state, broadcast_parameters
from . import callbacks  # noqa: F401

Average, Sum, Adasum = _ops.Average, _ops.Sum, _ops.Adasum


class _DistributedOptimizerMixin:
    def _hvd_setup(self, name, device_dense, device_sparse, compression, sparse_as_dense, op):
        self._hvd_name = name or f"Distributed{type(self).__mro__[2].__name__}"
        self._hvd_compression = compression
        self._hvd_sparse_as_dense = sparse_as_dense
        self._hvd_op = op
        from ._static import OverlappedGradientReducer, StaticGradientReducer
        self._hvd_static = StaticGradientReducer(self._hvd_name, op, compression)
        self._hvd_overlap = OverlappedGradientReducer(self._hvd_name, op, compression)

    def _hvd_overlappable(self, params) -> bool:
        env = os.environ.get("MIVOD_KERAS_OVERLAP", "")
        if env == "0" or os.environ.get("MIVOD_KERAS_NEGOTIATED", "0") == "1":
            return False
        if self.clipnorm is not None or self.clipvalue is not None:
            return False        # Keras clips the LOCAL gradients before the average
        return env == "1" or (len(params) > 0 and params[0].is_cuda)

    def get_gradients(self, loss, params):
        if size() <= 1:
            return super().get_gradients(loss, params)
        params = list(params)
        if self._hvd_overlappable(params):
            # the reduction overlaps the backward pass (hooks + comm stream)
            return self._hvd_overlap(loss, params)
        grads = super().get_gradients(loss, params)
        if os.environ.get("MIVOD_KERAS_NEGOTIATED", "0") != "1":
            return self._hvd_static(grads)
        handles = []
        for i, g in enumerate(grads):
            if g is None:
                handles.append(None)
                continue
            handles.append(_ops.allreduce_async(g.contiguous(), name=f"{self._hvd_name}_Allreduce/{i}",
                                                op=self._hvd_op, compression=self._hvd_compression))
        return [None if h is None else _ops.synchronize(h) for h in handles]


def DistributedOptimizer(optimizer, name=None, device_dense="", device_sparse="",
                         compression=Compression.none, sparse_as_dense=False, op=Average):
    """Wrap a ``mivod.kerasfw`` optimizer so gradients are averaged across ranks."""
    base = type(optimizer)
    cls = type(base.__name__, (_DistributedOptimizerMixin, base), {"__module__": base.__module__})
    obj = cls.from_config(optimizer.get_config())
    obj._hvd_setup(name, device_dense, device_sparse, compression, sparse_as_dense, op)
    return obj


def broadcast_variables(variables, root_rank: int = 0):
    """Broadcast a list of tensors (model variables / optimizer variables) in place."""
    # Parameters themselves (broadcast_parameters unwraps .data and bumps the
    # Parameter's own version counter, which a fused optimizer's master copy tracks)
    ts = [v for v in variables if torch.is_tensor(v)]
    broadcast_parameters(ts, root_rank)


def broadcast_global_variables(root_rank: int = 0, model=None):
    """Broadcast every model variable and optimizer slot from ``root_rank``.

    TF1's version walks ``tf.global_variables()``; mivod has no global graph,
    so the model whose variables to broadcast is passed (the callback does)."""
    if model is None:
        raise ValueError("mivod.keras.broadcast_global_variables needs the model")
    broadcast_variables(model.variables, root_rank)
    opt = getattr(model, "optimizer", None)
    if opt is not None:
        from ..common import basics
        it = torch.tensor([float(opt.iterations), float(opt.lr)], dtype=torch.float64)
        from ..parallel import collectives as C
        C.broadcast_(it, root_rank, group=basics.state().cpu_pg)
        opt.iterations = int(it[0].item())
        opt.lr.value = float(it[1].item())
        if getattr(opt, "_impl", None) is not None:
            broadcast_optimizer_state(opt._impl, root_rank)


def allreduce(value, name=None, average=True):
    """numpy/scalar in, numpy out (horovod.keras.allreduce)."""
    t = torch.as_tensor(np.asarray(value, dtype=np.float64 if np.isscalar(value) else None))
    out = _ops.allreduce(t, name=name, op=Average if average else Sum)
    return out.numpy()


def allgather(value, name=None):
    return _ops.allgather(torch.as_tensor(np.asarray(value)), name=name).numpy()


def broadcast(value, root_rank, name=None):
    return _ops.broadcast(torch.as_tensor(np.asarray(value)), root_rank, name=name).numpy()


def load_model(filepath, custom_optimizers=None, custom_objects=None,
               compression=Compression.none):
    """Load a saved model and re-wrap its optimizer in ``DistributedOptimizer``."""
    from ..kerasfw import load_model as _load
    from ..kerasfw import optimizers as O

    def wrap(cls):
        def make(**cfg):
            return DistributedOptimizer(cls(**cfg), compression=compression)
        make.from_config = lambda cfg: make(**cfg)
        return make

    objs = {}
    for n, c in O.OPTIMIZERS.items():
        objs[n] = type(n, (), {"from_config": staticmethod(lambda cfg, c=c: wrap(c)(**cfg))})
    for c in custom_optimizers or []:
        objs[c.__name__] = type(c.__name__, (), {"from_config":
                                                 staticmethod(lambda cfg, c=c: wrap(c)(**cfg))})
    objs.update(custom_objects or {})
    return _load(filepath, custom_objects=objs)
