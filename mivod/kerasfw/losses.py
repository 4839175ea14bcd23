"""Keras losses (semantics of keras 2.x / tf.keras: probabilities clipped to
[eps, 1-eps] unless ``from_logits``).  When the model's last layer ends in a
softmax, ``Model`` feeds the pre-softmax logits to the ``*_from_logits`` form,
which is the numerically stable equivalent (identical away from the clip)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .backend import epsilon


def categorical_crossentropy(y_true, y_pred, from_logits=False):
    if from_logits:
        return -(y_true * F.log_softmax(y_pred, dim=-1)).sum(-1).mean()
    p = y_pred / y_pred.sum(-1, keepdim=True)
    p = p.clamp(epsilon(), 1 - epsilon())
    return -(y_true * torch.log(p)).sum(-1).mean()


def sparse_categorical_crossentropy(y_true, y_pred, from_logits=False):
    y = y_true.long().reshape(-1)
    if from_logits:
        return F.cross_entropy(y_pred, y)
    p = y_pred.clamp(epsilon(), 1 - epsilon())
    return F.nll_loss(torch.log(p), y)


def mean_squared_error(y_true, y_pred):
    return ((y_pred - y_true) ** 2).mean()


def binary_crossentropy(y_true, y_pred, from_logits=False):
    if from_logits:
        return F.binary_cross_entropy_with_logits(y_pred, y_true.to(y_pred.dtype))
    p = y_pred.clamp(epsilon(), 1 - epsilon())
    return F.binary_cross_entropy(p, y_true.to(p.dtype))


mse = MSE = mean_squared_error


class Loss:
    fn = None
    name = "loss"

    def __init__(self, from_logits=False, name=None, **kw):
        self.from_logits = from_logits
        if name:
            self.name = name

    def __call__(self, y_true, y_pred):
        return type(self).fn(y_true, y_pred, from_logits=self.from_logits)

    def get_config(self):
        return {"from_logits": self.from_logits}


class CategoricalCrossentropy(Loss):
    fn = staticmethod(categorical_crossentropy)
    name = "categorical_crossentropy"


class SparseCategoricalCrossentropy(Loss):
    fn = staticmethod(sparse_categorical_crossentropy)
    name = "sparse_categorical_crossentropy"


class BinaryCrossentropy(Loss):
    fn = staticmethod(binary_crossentropy)
    name = "binary_crossentropy"


class MeanSquaredError(Loss):
    name = "mean_squared_error"

    def __call__(self, y_true, y_pred):
        return mean_squared_error(y_true, y_pred)


_BY_NAME = {"categorical_crossentropy": categorical_crossentropy,
            "sparse_categorical_crossentropy": sparse_categorical_crossentropy,
            "mean_squared_error": mean_squared_error, "mse": mean_squared_error,
            "binary_crossentropy": binary_crossentropy}


def get(loss):
    if isinstance(loss, str):
        if loss not in _BY_NAME:
            raise ValueError(f"unknown loss {loss!r}")
        return _BY_NAME[loss]
    return loss


def kind(loss) -> str:
    """'categorical' | 'sparse' | 'binary' | 'regression' (for metrics / logits path)."""
    f = get(loss)
    if isinstance(f, Loss):
        f = type(f).fn if type(f).fn is not None else None
        if isinstance(loss, MeanSquaredError):
            return "regression"
    if f is categorical_crossentropy:
        return "categorical"
    if f is sparse_categorical_crossentropy:
        return "sparse"
    if f is binary_crossentropy:
        return "binary"
    return "regression"


def name_of(loss) -> str:
    if isinstance(loss, str):
        return loss
    if isinstance(loss, Loss):
        return type(loss).__name__
    return getattr(loss, "__name__", "loss")
