"""Keras optimizers on mivod's fused flat-arena optimizers.

Keras semantics (keras 2.x / tf.keras): ``lr`` / ``learning_rate`` and
``momentum`` are backend Variables that callbacks mutate with
``K.set_value``; ``get_gradients(loss, params)`` is the hook point horovod's
Keras ``DistributedOptimizer`` overrides (/root/reference/tensorflow2_keras_mnist.py:60-65
explains why the reference must keep Keras on that path); ``get_config`` /
``from_config`` drive re-instantiation and ``load_model``.

The update itself is a mivod fused kernel (FusedAdadelta / FusedAdam with
Keras epsilon placement / FusedSGD): one launch per arena on the GPU, the
plain-PyTorch reference math on the CPU.
"""
from __future__ import annotations

from typing import List, Optional

import torch

from .backend import Variable, epsilon


class Optimizer:
    _hyper: tuple = ()

    def __init__(self, name: Optional[str] = None, **kwargs):
        lr = kwargs.pop("learning_rate", None)
        if lr is None:
            lr = kwargs.pop("lr", self._default_lr)
        else:
            kwargs.pop("lr", None)
        self.lr = Variable(lr, "lr")
        self.decay = float(kwargs.pop("decay", 0.0))
        self.clipnorm = kwargs.pop("clipnorm", None)
        self.clipvalue = kwargs.pop("clipvalue", None)
        self._name = name or type(self).__name__
        self.iterations = 0
        self._impl = None
        self._params: List[torch.nn.Parameter] = []

    _default_lr = 0.01

    @property
    def learning_rate(self):
        return self.lr

    # -- horovod hook point ------------------------------------------------
    def get_gradients(self, loss, params):
        grads = torch.autograd.grad(loss, params, allow_unused=True)
        grads = [torch.zeros_like(p) if g is None else g for g, p in zip(grads, params)]
        if self.clipnorm is not None:
            norm = torch.sqrt(sum((g.float() ** 2).sum() for g in grads))
            scale = torch.clamp(self.clipnorm / (norm + 1e-12), max=1.0)
            grads = [g * scale for g in grads]
        if self.clipvalue is not None:
            grads = [g.clamp(-self.clipvalue, self.clipvalue) for g in grads]
        return grads

    def _make_impl(self, params):
        raise NotImplementedError

    def _sync_hyper(self):
        lr = float(self.lr)
        if self.decay:
            lr = lr / (1.0 + self.decay * self.iterations)
        for g in self._impl.param_groups:
            g["lr"] = lr
            if hasattr(self, "momentum") and "momentum" in g:
                g["momentum"] = float(self.momentum)

    def apply_gradients(self, grads_and_vars):
        gv = list(grads_and_vars)
        params = [v for _, v in gv]
        if self._impl is None:
            self._params = params
            self._impl = self._make_impl(params)
        with torch.no_grad():
            for g, p in gv:
                p.grad = g
        self._sync_hyper()
        self._impl.step()
        for p in params:
            p.grad = None
        self.iterations += 1

    def minimize(self, loss, var_list):
        self.apply_gradients(zip(self.get_gradients(loss, var_list), var_list))

    # -- Keras config / weights --------------------------------------------
    def get_config(self) -> dict:
        cfg = {"name": self._name, "learning_rate": float(self.lr), "decay": self.decay}
        for h in self._hyper:
            v = getattr(self, h)
            cfg[h] = float(v) if isinstance(v, Variable) else v
        return cfg

    @classmethod
    def from_config(cls, config):
        return cls(**config)

    def variables(self) -> List[torch.Tensor]:
        out = []
        if self._impl is not None:
            for p in self._params:
                st = self._impl.state.get(p, {})
                out.extend(v for k, v in sorted(st.items()) if torch.is_tensor(v) and v.dim() > 0)
        return out

    weights = property(variables)

    def get_weights(self):
        return [self.iterations] + [v.detach().cpu().numpy() for v in self.variables()]

    def state_dict(self):
        return {"iterations": self.iterations, "lr": float(self.lr),
                "impl": self._impl.state_dict() if self._impl is not None else None}

    def load_state_dict(self, sd, params=None):
        self.iterations = int(sd.get("iterations", 0))
        if sd.get("impl") is not None:
            if self._impl is None:
                if params is None:
                    self._pending_state = sd["impl"]
                    return
                self._params = list(params)
                self._impl = self._make_impl(self._params)
            self._impl.load_state_dict(sd["impl"])

    def _maybe_load_pending(self):
        st = getattr(self, "_pending_state", None)
        if st is not None and self._impl is not None:
            self._impl.load_state_dict(st)
            self._pending_state = None


class SGD(Optimizer):
    _default_lr = 0.01
    _hyper = ("momentum", "nesterov")

    def __init__(self, lr=None, momentum=0.0, decay=0.0, nesterov=False, name=None, **kw):
        kw.setdefault("lr", lr if lr is not None else self._default_lr)
        super().__init__(name=name, decay=decay, **kw)
        self.momentum = Variable(momentum, "momentum")
        self.nesterov = bool(nesterov)

    def _make_impl(self, params):
        from ..optim import FusedSGD
        return FusedSGD(params, lr=float(self.lr), momentum=float(self.momentum) or 0.0,
                        nesterov=self.nesterov)

    def _sync_hyper(self):
        super()._sync_hyper()


class Adam(Optimizer):
    _default_lr = 0.001
    _hyper = ("beta_1", "beta_2", "epsilon", "amsgrad")

    def __init__(self, lr=None, beta_1=0.9, beta_2=0.999, epsilon=None, decay=0.0, amsgrad=False,
                 name=None, **kw):
        kw.setdefault("lr", lr if lr is not None else self._default_lr)
        super().__init__(name=name, decay=decay, **kw)
        self.beta_1, self.beta_2 = float(beta_1), float(beta_2)
        self.epsilon = float(epsilon if epsilon is not None else 1e-7)
        if amsgrad:
            raise NotImplementedError("amsgrad is not supported by mivod's fused Adam")
        self.amsgrad = False

    def _make_impl(self, params):
        from ..optim import FusedAdam
        return FusedAdam(params, lr=float(self.lr), betas=(self.beta_1, self.beta_2),
                         eps=self.epsilon, keras_eps=True)


class Adadelta(Optimizer):
    _default_lr = 1.0
    _hyper = ("rho", "epsilon")

    def __init__(self, lr=None, rho=0.95, epsilon=None, decay=0.0, name=None, **kw):
        kw.setdefault("lr", lr if lr is not None else self._default_lr)
        super().__init__(name=name, decay=decay, **kw)
        self.rho = float(rho)
        self.epsilon = float(epsilon if epsilon is not None else epsilon_default())

    def _make_impl(self, params):
        from ..optim import FusedAdadelta
        return FusedAdadelta(params, lr=float(self.lr), rho=self.rho, eps=self.epsilon)


def epsilon_default():
    return epsilon()


class RMSprop(Optimizer):
    _default_lr = 0.001
    _hyper = ("rho", "epsilon")

    def __init__(self, lr=None, rho=0.9, epsilon=None, decay=0.0, name=None, **kw):
        kw.setdefault("lr", lr if lr is not None else self._default_lr)
        super().__init__(name=name, decay=decay, **kw)
        self.rho = float(rho)
        self.epsilon = float(epsilon if epsilon is not None else 1e-7)

    def _make_impl(self, params):
        return torch.optim.RMSprop(params, lr=float(self.lr), alpha=self.rho, eps=self.epsilon)


OPTIMIZERS = {"SGD": SGD, "Adam": Adam, "Adadelta": Adadelta, "RMSprop": RMSprop}


def get(opt):
    if isinstance(opt, Optimizer):
        return opt
    if isinstance(opt, str):
        key = {k.lower(): k for k in OPTIMIZERS}.get(opt.lower())
        if key is None:
            raise ValueError(f"unknown optimizer {opt!r}")
        return OPTIMIZERS[key]()
    raise TypeError(f"not a Keras optimizer: {opt!r}")


def serialize(opt: Optimizer) -> dict:
    return {"class_name": type(opt).__name__, "config": opt.get_config()}


def deserialize(cfg: dict, custom_objects=None):
    custom_objects = custom_objects or {}
    name = cfg["class_name"]
    cls = custom_objects.get(name) or OPTIMIZERS.get(name)
    if cls is None:
        raise ValueError(f"unknown optimizer class {name!r}")
    return cls.from_config(cfg["config"])
