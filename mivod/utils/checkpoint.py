"""Checkpoint / resume for the PyTorch path (SURVEY.md §5 "Checkpoint / resume").

The reference saves ``checkpoint-{epoch}.h5`` on rank 0 only
(/root/reference/mnist_keras.py:100-104) and relies on the initial broadcast to
make restored runs consistent (:94-96); it has no resume logic.  mivod:

* ``save_checkpoint`` — rank 0 writes ONE safetensors file atomically (model
  state, optimizer tensors incl. fp32 master weights of fused optimizers) with
  the epoch, optimizer param-groups and scalar state as JSON metadata;
* ``load_checkpoint`` — rank 0 reads, every rank receives the model and
  optimizer state by broadcast (fused K1/K2 pack + one RCCL broadcast per
  dtype), so only rank 0 needs the file;
* ``resume_from(dir)`` — finds the newest ``checkpoint-<epoch>`` on rank 0
  and agrees on it across ranks; returns the epoch to start from.
"""
from __future__ import annotations

import json
import os
import re
from typing import Optional

import torch

from ..common import basics


def _rank0() -> bool:
    return not basics.is_initialized() or basics.rank() == 0


def _flatten_optimizer(opt):
    sd = opt.state_dict()
    tensors, scalars = {}, {}
    for pid, st in sd["state"].items():
        for k, v in st.items():
            key = f"optimizer.state.{pid}.{k}"
            if torch.is_tensor(v):
                tensors[key] = v.detach().contiguous().cpu()
            else:
                scalars[key] = v
    groups = []
    for g in sd["param_groups"]:
        groups.append({k: (list(v) if isinstance(v, tuple) else v) for k, v in g.items()})
    return tensors, scalars, groups


def save_checkpoint(path: str, model: torch.nn.Module, optimizer=None, epoch: Optional[int] = None,
                    extra: Optional[dict] = None) -> Optional[str]:
    """Rank 0 writes ``path`` (atomically); other ranks return None."""
    if not _rank0():
        return None
    from safetensors.torch import save_file
    tensors = {f"model.{k}": v.detach().contiguous().cpu() for k, v in model.state_dict().items()}
    meta = {"format": _FORMAT, "epoch": json.dumps(epoch),
            "extra": json.dumps(extra or {})}
    if optimizer is not None:
        ot, osc, groups = _flatten_optimizer(optimizer)
        tensors.update(ot)
        meta["optimizer.scalars"] = json.dumps(osc)
        meta["optimizer.param_groups"] = json.dumps(groups)
        meta["optimizer.class"] = type(optimizer).__name__
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    save_file(tensors, tmp, metadata=meta)
    os.replace(tmp, path)
    return path


def load_checkpoint(path: str, model: torch.nn.Module, optimizer=None, broadcast: bool = True,
                    map_location=None) -> dict:
    """Restore model (+ optimizer) from ``path`` read on rank 0 and broadcast.
    Returns ``{"epoch": ..., "extra": ...}`` on every rank."""
    from ..torch.functions import (broadcast_object, broadcast_optimizer_state,
                                   broadcast_parameters)
    info = None
    if _rank0():
        from safetensors import safe_open
        from safetensors.torch import load_file
        with safe_open(path, framework="pt") as f:
            meta = f.metadata() or {}
        t = load_file(path)
        msd = {k[len("model."):]: v for k, v in t.items() if k.startswith("model.")}
        model.load_state_dict(msd)
        if optimizer is not None and "optimizer.param_groups" in meta:
            state = {}
            for k, v in t.items():
                if k.startswith("optimizer.state."):
                    _, _, pid, name = k.split(".", 3)
                    state.setdefault(int(pid), {})[name] = v
            for k, v in json.loads(meta.get("optimizer.scalars", "{}")).items():
                _, _, pid, name = k.split(".", 3)
                state.setdefault(int(pid), {})[name] = v
            groups = json.loads(meta["optimizer.param_groups"])
            for g in groups:
                for k, v in list(g.items()):
                    if isinstance(v, list) and k != "params":
                        g[k] = tuple(v)
            optimizer.load_state_dict({"state": state, "param_groups": groups})
        info = {"epoch": json.loads(meta.get("epoch", "null")),
                "extra": json.loads(meta.get("extra", "{}"))}
    if broadcast and basics.is_initialized() and basics.size() > 1:
        broadcast_parameters(model.state_dict(), root_rank=0)
        if optimizer is not None:
            broadcast_optimizer_state(optimizer, root_rank=0)
        info = broadcast_object(info, root_rank=0)
    return info


_CKPT_RE = re.compile(r"checkpoint-(\d+)\.safetensors$")
_FORMAT = "mivod.checkpoint/1"


def _is_mivod_checkpoint(path: str) -> bool:
    """Only files this module wrote (safetensors with our format tag) — Keras
    ``checkpoint-{epoch}.h5`` files or foreign files in the same directory are
    never picked up by resume."""
    try:
        from safetensors import safe_open
        with safe_open(path, framework="pt") as f:
            return (f.metadata() or {}).get("format") == _FORMAT
    except Exception:
        return False


def latest_checkpoint(directory: str) -> Optional[str]:
    if not os.path.isdir(directory):
        return None
    cands = []
    for f in os.listdir(directory):
        m = _CKPT_RE.search(f)
        if m:
            cands.append((int(m.group(1)), os.path.join(directory, f)))
    for _ep, path in sorted(cands, reverse=True):
        if _is_mivod_checkpoint(path):
            return path
    return None


def resume_from(directory: str, model, optimizer=None) -> int:
    """Load the newest checkpoint in ``directory`` (if any); return the epoch
    to start from (0 when there is nothing to resume)."""
    from ..torch.functions import broadcast_object
    path = latest_checkpoint(directory) if _rank0() else None
    if basics.is_initialized() and basics.size() > 1:
        path = broadcast_object(path, root_rank=0)
    if path is None:
        return 0
    info = load_checkpoint(path, model, optimizer)
    ep = info.get("epoch") if info else None
    return int(ep) + 1 if ep is not None else 0
