"""Keras ``backend`` subset used by the reference scripts and horovod's Keras
callbacks (``K.get_value`` / ``K.set_value`` on optimizer hyper-parameters,
``K.image_data_format``, ``K.epsilon``, ``K.set_learning_phase``)."""
from __future__ import annotations

import torch

_EPSILON = 1e-7
_learning_phase = None


class Variable:
    """A named scalar hyper-parameter (lr, momentum, ...) that callbacks mutate."""

    def __init__(self, value, name: str = ""):
        self.value = float(value)
        self.name = name

    def __float__(self):
        return float(self.value)

    def __repr__(self):
        return f"<Variable {self.name}={self.value}>"

    def numpy(self):
        return self.value


def get_value(x):
    if isinstance(x, Variable):
        return x.value
    if torch.is_tensor(x):
        return x.detach().cpu().numpy()
    return x


def set_value(x, value):
    if isinstance(x, Variable):
        x.value = float(value)
    elif torch.is_tensor(x):
        with torch.no_grad():
            x.copy_(torch.as_tensor(value, dtype=x.dtype))
    else:
        raise TypeError(f"cannot set_value on {type(x)}")


def variable(value, name=""):
    return Variable(value, name)


def constant(value, name=None):
    return torch.as_tensor(value)


def image_data_format() -> str:
    return "channels_last"


def epsilon() -> float:
    return _EPSILON


def set_epsilon(e: float):
    global _EPSILON
    _EPSILON = float(e)


def set_learning_phase(value):
    global _learning_phase
    _learning_phase = value


def learning_phase():
    return _learning_phase


def clear_session():
    pass


def floatx() -> str:
    return "float32"
