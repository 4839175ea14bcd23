"""Keras activation functions by name."""
from __future__ import annotations

import torch
import torch.nn.functional as F


def linear(x):
    return x


def relu(x):
    return F.relu(x)


def softmax(x):
    return torch.softmax(x, dim=-1)


def sigmoid(x):
    return torch.sigmoid(x)


def tanh(x):
    return torch.tanh(x)


def elu(x):
    return F.elu(x)


def gelu(x):
    return F.gelu(x)


_ACT = {"linear": linear, None: linear, "relu": relu, "softmax": softmax, "sigmoid": sigmoid,
        "tanh": tanh, "elu": elu, "gelu": gelu}


def get(a):
    if callable(a):
        return a
    if a not in _ACT:
        raise ValueError(f"unknown activation {a!r}")
    return _ACT[a]


def name_of(a):
    if a is None or isinstance(a, str):
        return a or "linear"
    for k, v in _ACT.items():
        if v is a and k:
            return k
    return getattr(a, "__name__", "custom")
