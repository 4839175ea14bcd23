"""Fused multi-tensor optimizers on flat parameter arenas.

MI355X design: every param group's parameters (per dtype) live in ONE flat,
64-element-aligned arena laid out in *backward order* (reverse registration
order), and each ``Parameter`` is a strided view into it (channels_last
preserved).  Gradients are packed into a flat grad arena of the same layout,
so a gradient bucket is simply a contiguous range ``[lo, hi)`` of the arena and
one kernel launch updates the whole bucket: grad read once, fp32 master and
optimizer state read+written once, the bf16 model copy written in the same
pass.  ``mivod.torch.DistributedOptimizer`` launches that kernel on the comm
stream right after the bucket's RCCL allreduce, overlapped with the rest of
backward.

Reference parity: the optimizers the reference trains with — Keras ``Adadelta``
(/root/reference/mnist_keras.py:84) and ``tf.optimizers.Adam``
(/root/reference/tensorflow2_keras_mnist.py:55) — plus SGD-momentum (ResNet-50)
and LARS (large-batch ResNet), per BASELINE.json north star.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch

from ..ops import kernels as K

ALIGN = 64  # elements; keeps every slot 16-byte aligned for bf16/fp16/fp32


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


class Arena:
    """A flat arena for the params of one (param_group, dtype)."""

    def __init__(self, group: dict, group_index: int, params: List[torch.nn.Parameter],
                 state_names: List[str], grad_dtype: Optional[torch.dtype] = None):
        assert params
        self.group = group
        self.group_index = group_index
        self.params = params                      # arena (backward) order
        self.dtype = params[0].dtype
        self.device = params[0].device
        self.offsets: List[int] = []
        o = 0
        for p in params:
            if not K.is_dense(p):
                raise ValueError("fused optimizers need dense parameters")
            self.offsets.append(o)
            o += _align(p.numel())
        self.numel = o
        self.index = {id(p): i for i, p in enumerate(params)}
        # model arena: params become views into it
        self.model = torch.zeros(self.numel, dtype=self.dtype, device=self.device)
        with torch.no_grad():
            for p, off in zip(params, self.offsets):
                view = torch.as_strided(self.model, p.size(), p.stride(), off)
                view.copy_(p.data)
                p.data = view
        self.low_precision = self.dtype != torch.float32
        self.master = self.model.float() if self.low_precision else self.model
        self.grad_dtype = grad_dtype or self.dtype
        self.grad = torch.zeros(self.numel, dtype=self.grad_dtype, device=self.device)
        self.state: Dict[str, torch.Tensor] = {
            n: torch.zeros(self.numel, dtype=torch.float32, device=self.device) for n in state_names}
        self.step = 0
        self.versions = [p._version for p in params]
        self.tables: Dict[tuple, K.ChunkTable] = {}
        self.workspace: Dict[str, torch.Tensor] = {}
        self.dyn: Optional[torch.Tensor] = None   # [lr, first, bc1, bc2] for graph replays

    # -- views ---------------------------------------------------------------
    def slot(self, flat: torch.Tensor, i: int) -> torch.Tensor:
        p = self.params[i]
        return torch.as_strided(flat, p.size(), p.stride(), self.offsets[i])

    def range_of(self, i0: int, i1: int):
        """Element range covering params [i0, i1) (aligned)."""
        lo = self.offsets[i0]
        hi = self.offsets[i1] if i1 < len(self.params) else self.numel
        return lo, hi

    def sync_master_if_modified(self):
        """Params modified in place outside the optimizer (broadcast_parameters,
        load_state_dict, manual edits) re-seed their fp32 master slot."""
        if not self.low_precision:
            return
        for i, p in enumerate(self.params):
            v = p._version
            if v != self.versions[i]:
                lo = self.offsets[i]
                n = p.numel()
                with torch.no_grad():
                    self.master[lo:lo + n].copy_(self.model[lo:lo + n])
                self.versions[i] = v

    def table(self, i0: int, i1: int) -> K.ChunkTable:
        key = (i0, i1)
        t = self.tables.get(key)
        if t is None:
            lo = self.offsets[i0]
            sizes = [self.params[i].numel() for i in range(i0, i1)]
            offs = [self.offsets[i] - lo for i in range(i0, i1)]
            t = K.make_chunk_table(sizes, self.device, offs)
            self.tables[key] = t
        return t


class FusedOptimizer(torch.optim.Optimizer):
    """Base class: arena management, standalone ``step()``, state-dict views."""

    _state_names: List[str] = []

    def __init__(self, params, defaults, grad_dtype: Optional[torch.dtype] = None):
        super().__init__(params, defaults)
        self._mv_arenas: Optional[List[Arena]] = None
        self._mv_grad_dtype = grad_dtype
        self._mv_external_grads = False   # True when DistributedOptimizer packs grads
        self._mv_graph = False            # True while a HIP graph captures the step
        self._mv_skip = None              # device int32 skip flag (overflow guard)

    # ---- layout ----------------------------------------------------------
    def _mv_build(self, grad_dtype_for=None) -> List[Arena]:
        if self._mv_arenas is not None:
            return self._mv_arenas
        arenas = []
        for gi, g in enumerate(self.param_groups):
            params = [p for p in g["params"] if p.requires_grad]
            by_dtype: Dict[torch.dtype, List[torch.nn.Parameter]] = {}
            for p in reversed(params):                # backward order
                by_dtype.setdefault(p.dtype, []).append(p)
            for dt, ps in by_dtype.items():
                gdt = self._mv_grad_dtype
                if grad_dtype_for is not None:
                    gdt = grad_dtype_for(dt)
                arenas.append(Arena(g, gi, ps, self._state_names, gdt))
        self._mv_arenas = arenas
        self._mv_expose_state()
        return arenas

    def _mv_expose_state(self):
        """Per-param state entries are views into the flat state arenas, so
        ``state_dict()`` / ``broadcast_optimizer_state`` work unchanged."""
        for a in self._mv_arenas:
            for i, p in enumerate(a.params):
                st = self.state[p]
                for n, flat in a.state.items():
                    st[n] = a.slot(flat, i)
                if a.low_precision:
                    st["master_param"] = a.slot(a.master, i)
                st["step"] = torch.tensor(float(a.step))

    def _mv_begin_step(self):
        for a in self._mv_build():
            a.sync_master_if_modified()
            a.step += 1

    def _mv_end_step(self):
        for a in self._mv_arenas or []:
            a.versions = [p._version for p in a.params]

    def state_dict(self):
        for a in self._mv_arenas or []:
            for p in a.params:
                self.state[p]["step"] = torch.tensor(float(a.step))
        return super().state_dict()

    # ---- the fused update of a bucket ------------------------------------
    def _mv_apply(self, a: Arena, i0: int, i1: int, gscale: float = 1.0):
        raise NotImplementedError

    def _mv_dyn(self, a: Arena):
        """Device hyperparameter block for graph capture (None in eager mode)."""
        if not self._mv_graph:
            return None
        if a.dyn is None:
            a.dyn = torch.zeros(4, dtype=torch.float32, device=a.device)
        return a.dyn

    def _mv_slices(self, a: Arena, i0: int, i1: int):
        lo, hi = a.range_of(i0, i1)
        model = a.model[lo:hi] if a.low_precision else None
        st = {n: f[lo:hi] for n, f in a.state.items()}
        return a.grad[lo:hi], a.master[lo:hi], st, model

    # ---- standalone step (no DistributedOptimizer) -------------------------
    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        arenas = self._mv_build()
        self._mv_begin_step()
        for a in arenas:
            if not self._mv_external_grads:
                grads, offs = [], []
                for i, p in enumerate(a.params):
                    if p.grad is None:
                        lo = a.offsets[i]
                        a.grad[lo:lo + p.numel()].zero_()
                        continue
                    g = p.grad
                    if g.stride() != p.stride():
                        g = torch.empty_like(p).copy_(g)
                    grads.append(g)
                    offs.append(a.offsets[i])
                by_dt: Dict[torch.dtype, tuple] = {}
                for g, o in zip(grads, offs):
                    by_dt.setdefault(g.dtype, ([], []))
                    by_dt[g.dtype][0].append(g)
                    by_dt[g.dtype][1].append(o)
                for gl, ol in by_dt.values():
                    K.pack(gl, a.grad, ol)
            self._mv_apply(a, 0, len(a.params), 1.0)
        self._mv_end_step()
        return loss

    def load_state_dict(self, state_dict):
        arenas = self._mv_build()
        # torch's loader casts every floating state tensor to its parameter's dtype
        # (bf16 for a bf16 model): take the exact fp32 values (master weights, Adam
        # moments) from the incoming dict instead of from the cast copies
        raw = {}
        for g_saved, g_live in zip(state_dict.get("param_groups", []), self.param_groups):
            for k, p in zip(g_saved["params"], g_live["params"]):
                if k in state_dict.get("state", {}):
                    raw[p] = state_dict["state"][k]
        super().load_state_dict(state_dict)
        # torch replaced our views with fresh tensors: copy them back into the arenas
        with torch.no_grad():
            for a in arenas:
                steps = []
                for i, p in enumerate(a.params):
                    st = raw.get(p) or self.state.get(p, {})
                    for n, flat in a.state.items():
                        if n in st and torch.is_tensor(st[n]):
                            a.slot(flat, i).copy_(st[n])
                    if a.low_precision:
                        if "master_param" in st:
                            a.slot(a.master, i).copy_(st["master_param"])
                        else:
                            a.slot(a.master, i).copy_(p.data)
                    if "step" in st:
                        steps.append(float(st["step"]))
                if steps:
                    a.step = int(max(steps))
                a.versions = [p._version for p in a.params]
        self._mv_expose_state()

    def zero_grad(self, set_to_none: bool = True):
        super().zero_grad(set_to_none=set_to_none)


class FusedSGD(FusedOptimizer):
    """SGD with momentum / dampening / nesterov / weight decay (torch.optim.SGD
    semantics, momentum buffer seeded with the first gradient)."""

    def __init__(self, params, lr=0.1, momentum=0.0, dampening=0.0, weight_decay=0.0,
                 nesterov=False, grad_dtype=None):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        self._state_names = ["momentum_buffer"] if momentum != 0 else []
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening,
                                      weight_decay=weight_decay, nesterov=nesterov), grad_dtype)

    def _mv_apply(self, a, i0, i1, gscale=1.0):
        g, w, st, model = self._mv_slices(a, i0, i1)
        hp = a.group
        K.sgd_step(g, w, st.get("momentum_buffer"), model, lr=hp["lr"], momentum=hp["momentum"],
                   dampening=hp["dampening"], weight_decay=hp["weight_decay"], gscale=gscale,
                   nesterov=hp["nesterov"], first=(a.step == 1), dyn=self._mv_dyn(a),
                   skip=self._mv_skip)


class FusedAdam(FusedOptimizer):
    """Adam / AdamW.  ``keras_eps=True`` uses Keras' epsilon placement
    (eps scaled by sqrt(1-beta2^t)), matching tf.optimizers.Adam."""

    _state_names = ["exp_avg", "exp_avg_sq"]

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 adamw=False, keras_eps=False, grad_dtype=None):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                      adamw=adamw, keras_eps=keras_eps), grad_dtype)

    def _mv_apply(self, a, i0, i1, gscale=1.0):
        g, w, st, model = self._mv_slices(a, i0, i1)
        hp = a.group
        b1, b2 = hp["betas"]
        K.adam_step(g, w, st["exp_avg"], st["exp_avg_sq"], model, lr=hp["lr"], beta1=b1, beta2=b2,
                    eps=hp["eps"], weight_decay=hp["weight_decay"], gscale=gscale, step=a.step,
                    adamw=hp["adamw"], keras_eps=hp["keras_eps"], dyn=self._mv_dyn(a),
                    skip=self._mv_skip)


class FusedAdamW(FusedAdam):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 grad_dtype=None):
        super().__init__(params, lr, betas, eps, weight_decay, adamw=True, grad_dtype=grad_dtype)


class FusedAdadelta(FusedOptimizer):
    """Adadelta (Zeiler 2012; torch / Keras semantics — Keras uses eps=1e-7)."""

    _state_names = ["square_avg", "acc_delta"]

    def __init__(self, params, lr=1.0, rho=0.9, eps=1e-6, weight_decay=0.0, grad_dtype=None):
        super().__init__(params, dict(lr=lr, rho=rho, eps=eps, weight_decay=weight_decay),
                         grad_dtype)

    def _mv_apply(self, a, i0, i1, gscale=1.0):
        g, w, st, model = self._mv_slices(a, i0, i1)
        hp = a.group
        K.adadelta_step(g, w, st["square_avg"], st["acc_delta"], model, lr=hp["lr"], rho=hp["rho"],
                        eps=hp["eps"], weight_decay=hp["weight_decay"], gscale=gscale,
                        dyn=self._mv_dyn(a), skip=self._mv_skip)


class FusedLARS(FusedOptimizer):
    """LARS (You, Gitman, Ginsburg 2017) with momentum.  Parameters with
    ``dim() <= 1`` (BN affine, biases) are excluded from adaptation and weight
    decay when ``exclude_1d=True`` (the common large-batch ResNet recipe)."""

    _state_names = ["momentum_buffer"]

    def __init__(self, params, lr=0.1, momentum=0.9, weight_decay=1e-4, eta=0.001, eps=0.0,
                 exclude_1d=True, grad_dtype=None):
        super().__init__(params, dict(lr=lr, momentum=momentum, weight_decay=weight_decay, eta=eta,
                                      eps=eps, exclude_1d=exclude_1d), grad_dtype)
        self._mv_flags: Dict[tuple, torch.Tensor] = {}

    def _mv_apply(self, a, i0, i1, gscale=1.0):
        g, w, st, model = self._mv_slices(a, i0, i1)
        hp = a.group
        key = (id(a), i0, i1)
        flags = self._mv_flags.get(key)
        if flags is None:
            fl = [1 if (hp["exclude_1d"] and a.params[i].dim() <= 1) else 0 for i in range(i0, i1)]
            flags = self._mv_flags[key] = torch.tensor(fl, dtype=torch.int32, device=a.device)
        K.lars_step(g, w, st["momentum_buffer"], model, a.table(i0, i1), flags, lr=hp["lr"],
                    momentum=hp["momentum"], weight_decay=hp["weight_decay"], eta=hp["eta"],
                    gscale=gscale, eps=hp["eps"], first=(a.step == 1), workspace=a.workspace,
                    dyn=self._mv_dyn(a), skip=self._mv_skip)
