"""State broadcast helpers (parity: horovod/torch/__init__.py
``broadcast_parameters`` / ``broadcast_optimizer_state`` / ``broadcast_object``,
SURVEY.md §3.5; the reference's ``BroadcastGlobalVariablesCallback(0)`` at
/root/reference/mnist_keras.py:97 and tensorflow2_keras_mnist.py:71).

MI355X design: all tensors of a dtype are packed into ONE flat buffer by the
hand-written multi-tensor pack kernel (K1), broadcast with a single RCCL call,
and unpacked (K2) — one collective per dtype instead of one per tensor.
"""
from __future__ import annotations

import io
import pickle
from typing import Dict, List

import torch

from ..common import basics
from ..ops import kernels as K
from ..parallel import collectives as C


def _fused_broadcast_(tensors: List[torch.Tensor], root_rank: int) -> None:
    st = basics.state()
    if st.size == 1 or not tensors:
        return
    groups: Dict[tuple, List[torch.Tensor]] = {}
    for t in tensors:
        groups.setdefault((t.dtype, t.device), []).append(t)
    for (dt, dev), ts in groups.items():
        dense = [t for t in ts if K.is_dense(t)]
        other = [t for t in ts if not K.is_dense(t)]
        for t in other:
            C.broadcast_(t, root_rank)
        if not dense:
            continue
        floaty = dt in (torch.float32, torch.float16, torch.bfloat16)
        offs, o = [], 0
        for t in dense:
            offs.append(o)
            o += (t.numel() + 63) // 64 * 64
        flat = torch.zeros(o, dtype=dt, device=dev)
        if floaty:
            K.pack(dense, flat, offs)
        else:
            for t, off in zip(dense, offs):
                flat[off:off + t.numel()].copy_(K._raw_flat(t))
        C.broadcast_(flat, root_rank)
        if floaty:
            K.unpack(dense, flat, offs)
        else:
            for t, off in zip(dense, offs):
                K._raw_flat(t).copy_(flat[off:off + t.numel()])


def broadcast_parameters(params, root_rank: int = 0) -> None:
    """Broadcast parameters (``model.state_dict()``, ``model.named_parameters()``
    or a list of tensors / (name, tensor) pairs) from ``root_rank`` in place."""
    if isinstance(params, dict):
        items = sorted(params.items())
    elif isinstance(params, list) or hasattr(params, "__iter__"):
        items = list(params)
        if items and not isinstance(items[0], tuple):
            items = [(str(i), t) for i, t in enumerate(items)]
    else:
        raise ValueError("invalid params of type: %s" % type(params))
    tensors = []
    for _name, p in items:
        if p is None:
            continue
        if not torch.is_tensor(p):
            raise ValueError(f"broadcast_parameters expects tensors, got {type(p)}")
        tensors.append(p.data if isinstance(p, torch.nn.Parameter) else p)
    with torch.no_grad():
        _fused_broadcast_(tensors, root_rank)
    if basics.state().size > 1:
        # the pack/unpack kernels write through raw pointers: bump the version
        # counters so in-place edits are visible — a fused optimizer re-seeds its
        # fp32 master copy of bf16 params from the broadcast values
        # (Arena.sync_master_if_modified) instead of keeping its own rank's init.
        # Bump the caller's tensor itself: a Parameter's ``.data`` has its own counter.
        for _name, p in items:
            if torch.is_tensor(p):
                torch.autograd.graph.increment_version(p)
    # no host synchronisation: pack, broadcast and unpack are all enqueued on the
    # caller's current stream (transport.py), so later work on it is ordered after them


def broadcast_optimizer_state(optimizer, root_rank: int = 0) -> None:
    """Broadcast an optimizer's state (tensors and scalar hyper-parameters)."""
    from ..optim.fused import FusedOptimizer
    from .optimizer import _DistributedOptimizerMixin
    if isinstance(optimizer, torch.optim.LBFGS):
        raise ValueError("cannot broadcast torch.optim.LBFGS state")
    if isinstance(optimizer, FusedOptimizer):
        optimizer._mv_build()
    state_dict = optimizer.state_dict()
    if len(state_dict["state"]) == 0 and not isinstance(optimizer, FusedOptimizer):
        # Newly created optimizer: materialise its state with a zero-gradient
        # step of the *base* optimizer (horovod does the same).
        for group in optimizer.param_groups:
            for p in group["params"]:
                if p.requires_grad and p.grad is None:
                    p.grad = torch.zeros_like(p)
        saved = [{k: v for k, v in g.items() if k != "params"} for g in optimizer.param_groups]
        for g in optimizer.param_groups:
            if "lr" in g:
                g["lr"] = 0.0
            if "weight_decay" in g:
                g["weight_decay"] = 0.0
        base = optimizer.__class__
        if isinstance(optimizer, _DistributedOptimizerMixin):
            base = optimizer.__class__.__mro__[2]
        base.step(optimizer)
        for g, s in zip(optimizer.param_groups, saved):
            g.update(s)
        optimizer.zero_grad()
        state_dict = optimizer.state_dict()

    # scalar hyper-parameters in the param groups, broadcast as one fp64 vector
    scalars = []
    for g in state_dict["param_groups"]:
        for k in sorted(g):
            if k == "params":
                continue
            v = g[k]
            if isinstance(v, bool) or v is None:
                continue
            if isinstance(v, (int, float)):
                scalars.append((g, k, type(v)))
            elif isinstance(v, tuple) and all(isinstance(x, (int, float)) for x in v):
                scalars.append((g, k, tuple))
    if scalars:
        vals = []
        for g, k, ty in scalars:
            vals.extend(list(g[k]) if ty is tuple else [g[k]])
        vec = torch.tensor(vals, dtype=torch.float64)
        C.broadcast_(vec, root_rank)
        it = iter(vec.tolist())
        for (g, k, ty), pg in zip(scalars, [None] * len(scalars)):
            if ty is tuple:
                g[k] = tuple(next(it) for _ in g[k])
            else:
                g[k] = ty(next(it))
        # write back into the live param groups (state_dict() returned copies)
        for live, sd in zip(optimizer.param_groups, state_dict["param_groups"]):
            for k, v in sd.items():
                if k != "params":
                    live[k] = v

    tensors, scalar_state = [], []
    for pid in sorted(state_dict["state"]):
        st = state_dict["state"][pid]
        for k in sorted(st):
            v = st[k]
            if torch.is_tensor(v):
                if v.dim() == 0 and not v.is_cuda:
                    scalar_state.append((pid, k, v))
                else:
                    tensors.append(v)
            elif isinstance(v, (int, float)):
                scalar_state.append((pid, k, v))
    with torch.no_grad():
        _fused_broadcast_(tensors, root_rank)
    if scalar_state:
        vec = torch.tensor([float(v) for _, _, v in scalar_state], dtype=torch.float64)
        C.broadcast_(vec, root_rank)
        for (pid, k, v), nv in zip(scalar_state, vec.tolist()):
            if torch.is_tensor(v):
                v.fill_(nv)
            else:
                state_dict["state"][pid][k] = type(v)(nv)
    if isinstance(optimizer, FusedOptimizer):
        # state views alias the flat arenas: already updated in place; sync step counters
        for a in optimizer._mv_arenas:
            for p in a.params:
                s = optimizer.state[p].get("step")
                if torch.is_tensor(s):
                    a.step = int(s.item())
                    break
            # the exact fp32 master was just broadcast: keep it.  Without this the
            # version bump of a preceding broadcast_parameters makes the next step
            # re-seed the master from the (bf16) model copy on every rank.
            a.versions = [p._version for p in a.params]
    else:
        optimizer.load_state_dict(state_dict)
    # stream-ordered like broadcast_parameters: no host synchronisation


def broadcast_object(obj, root_rank: int = 0, name=None):
    """Broadcast a picklable Python object from ``root_rank`` (objects produced
    by this program only; never used on untrusted files)."""
    st = basics.state()
    if st.size == 1:
        return obj
    if st.rank == root_rank:
        b = io.BytesIO()
        pickle.dump(obj, b)
        data = torch.frombuffer(bytearray(b.getvalue()), dtype=torch.uint8)
        n = torch.tensor([data.numel()], dtype=torch.int64)
    else:
        n = torch.zeros(1, dtype=torch.int64)
    C.broadcast_(n, root_rank, group=st.cpu_pg)
    if st.rank != root_rank:
        data = torch.zeros(int(n.item()), dtype=torch.uint8)
    C.broadcast_(data, root_rank, group=st.cpu_pg)
    if st.rank == root_rank:
        return obj
    return pickle.loads(data.numpy().tobytes())


def allgather_object(obj, name=None):
    st = basics.state()
    if st.size == 1:
        return [obj]
    b = pickle.dumps(obj)
    data = torch.frombuffer(bytearray(b), dtype=torch.uint8)
    gathered = C.allgather(data, group=st.cpu_pg)
    sizes = C.allgather(torch.tensor([data.numel()], dtype=torch.int64), group=st.cpu_pg).tolist()
    out, o = [], 0
    for s in sizes:
        out.append(pickle.loads(gathered[o:o + s].numpy().tobytes()))
        o += s
    return out
