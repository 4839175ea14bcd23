"""Keras layers on PyTorch (channels_last / NHWC semantics, Keras weight layouts).

Covers what the reference models use — ``Conv2D``, ``MaxPooling2D``,
``Dropout``, ``Flatten``, ``Dense`` (/root/reference/mnist_keras.py:71-81,
/root/reference/tensorflow2_keras_mnist.py:43-52) — plus ``Activation``,
``BatchNormalization``, ``InputLayer``, ``AveragePooling2D``,
``GlobalAveragePooling2D``, ``Reshape``.

Activations are NHWC tensors.  Conv2D runs as a zero-copy ``permute`` to an
NCHW view with channels_last strides, so on the GPU MIOpen sees NHWC directly.
``get_weights()`` / ``set_weights()`` use Keras layouts (conv kernel HWIO, dense
kernel [in, out]) so checkpoints match Keras parameter counts and order
(ConvNet: 1,199,882 parameters).
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import activations as A

_UID = {}


def _uid(prefix: str) -> str:
    n = _UID.get(prefix, 0) + 1
    _UID[prefix] = n
    return prefix if n == 1 else f"{prefix}_{n - 1}"


def _pair(v) -> Tuple[int, int]:
    if isinstance(v, (list, tuple)):
        return int(v[0]), int(v[1])
    return int(v), int(v)


def _glorot_uniform_(t: torch.Tensor, fan_in: int, fan_out: int):
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    with torch.no_grad():
        t.uniform_(-lim, lim)


class Layer(nn.Module):
    """Base Keras-style layer: lazy ``build(input_shape)``, Keras weights API."""

    def __init__(self, name: Optional[str] = None, input_shape=None, trainable: bool = True,
                 **kwargs):
        super().__init__()
        self._name = name or _uid(self._default_name())
        self.built = False
        self.trainable = trainable
        self.input_shape_arg = tuple(input_shape) if input_shape is not None else None
        self._config_extra = {}

    @classmethod
    def _default_name(cls) -> str:
        n = cls.__name__
        out = []
        for i, ch in enumerate(n):
            if ch.isupper() and i and (not n[i - 1].isupper() or
                                       (i + 1 < len(n) and n[i + 1].islower())):
                out.append("_")
            out.append(ch.lower())
        return "".join(out)

    @property
    def name(self) -> str:
        return self._name

    def build(self, input_shape):
        self.built = True

    def compute_output_shape(self, input_shape):
        return input_shape

    def call(self, x, training=False):
        raise NotImplementedError

    def forward(self, x, training: Optional[bool] = None):
        if not self.built:
            self.build(tuple(x.shape[1:]))
            self.to(x.device)
        return self.call(x, self.training if training is None else training)

    # Keras weights API (layout conversion in subclasses)
    def _keras_weights(self) -> List[torch.Tensor]:
        return [p for p in self.parameters()]

    def get_weights(self) -> List[np.ndarray]:
        return [w.detach().float().cpu().numpy().copy() for w in self._keras_weights()]

    def set_weights(self, weights):
        raise NotImplementedError

    @property
    def weights(self):
        return self._keras_weights()

    def count_params(self) -> int:
        return sum(p.numel() for p in self.parameters())

    def get_config(self) -> dict:
        cfg = {"name": self.name, "trainable": self.trainable}
        if self.input_shape_arg is not None:
            cfg["input_shape"] = list(self.input_shape_arg)
        cfg.update(self._config_extra)
        return cfg

    @classmethod
    def from_config(cls, cfg):
        return cls(**cfg)


class InputLayer(Layer):
    def __init__(self, input_shape=None, name=None, **kw):
        super().__init__(name=name, input_shape=input_shape)

    def call(self, x, training=False):
        return x


class Conv2D(Layer):
    def __init__(self, filters, kernel_size, strides=(1, 1), padding="valid", activation=None,
                 use_bias=True, dilation_rate=(1, 1), data_format=None, name=None,
                 input_shape=None, kernel_initializer="glorot_uniform",
                 bias_initializer="zeros", **kw):
        super().__init__(name=name, input_shape=input_shape)
        if data_format not in (None, "channels_last"):
            raise ValueError("mivod.kerasfw layers are channels_last (NHWC)")
        self.filters = int(filters)
        self.kernel_size = _pair(kernel_size)
        self.strides = _pair(strides)
        self.padding = padding.lower()
        self.dilation = _pair(dilation_rate)
        self.activation = A.get(activation)
        self.activation_name = A.name_of(activation)
        self.use_bias = use_bias
        self._config_extra = dict(filters=self.filters, kernel_size=list(self.kernel_size),
                                  strides=list(self.strides), padding=self.padding,
                                  activation=self.activation_name, use_bias=use_bias,
                                  dilation_rate=list(self.dilation))
        if self.input_shape_arg is not None:
            self.build(self.input_shape_arg)

    def build(self, input_shape):
        cin = int(input_shape[-1])
        kh, kw = self.kernel_size
        self.weight = nn.Parameter(torch.empty(self.filters, cin, kh, kw))
        _glorot_uniform_(self.weight, kh * kw * cin, kh * kw * self.filters)
        self.weight.data = self.weight.data.contiguous(memory_format=torch.channels_last)
        self.bias = nn.Parameter(torch.zeros(self.filters)) if self.use_bias else None
        self.built = True

    def _pad(self, h, w):
        if self.padding == "valid":
            return (0, 0, 0, 0)
        kh, kw = self.kernel_size
        sh, sw = self.strides
        dh, dw = self.dilation
        eh, ew = (kh - 1) * dh + 1, (kw - 1) * dw + 1
        ph = max((math.ceil(h / sh) - 1) * sh + eh - h, 0)
        pw = max((math.ceil(w / sw) - 1) * sw + ew - w, 0)
        return (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2)

    def call(self, x, training=False):
        xc = x.permute(0, 3, 1, 2)            # NHWC -> NCHW view (channels_last strides)
        pad = self._pad(xc.shape[2], xc.shape[3])
        if any(pad):
            xc = F.pad(xc, pad)
        w = self.weight if self.weight.dtype == xc.dtype else self.weight.to(xc.dtype)
        b = self.bias
        if b is not None and b.dtype != xc.dtype:
            b = b.to(xc.dtype)
        y = F.conv2d(xc, w, b, self.strides, 0, self.dilation)
        return self.activation(y.permute(0, 2, 3, 1))

    def compute_output_shape(self, s):
        h, w, _ = s
        if self.padding == "same":
            return (math.ceil(h / self.strides[0]), math.ceil(w / self.strides[1]), self.filters)
        kh, kw = self.kernel_size
        dh, dw = self.dilation
        return ((h - (kh - 1) * dh - 1) // self.strides[0] + 1,
                (w - (kw - 1) * dw - 1) // self.strides[1] + 1, self.filters)

    def _keras_weights(self):
        ws = [self.weight]
        if self.bias is not None:
            ws.append(self.bias)
        return ws

    def get_weights(self):
        out = [self.weight.detach().float().permute(2, 3, 1, 0).cpu().numpy().copy()]   # HWIO
        if self.bias is not None:
            out.append(self.bias.detach().float().cpu().numpy().copy())
        return out

    def set_weights(self, weights):
        with torch.no_grad():
            k = torch.as_tensor(np.asarray(weights[0])).permute(3, 2, 0, 1)
            self.weight.copy_(k)
            if self.bias is not None:
                self.bias.copy_(torch.as_tensor(np.asarray(weights[1])))


class Dense(Layer):
    def __init__(self, units, activation=None, use_bias=True, name=None, input_shape=None,
                 input_dim=None, kernel_initializer="glorot_uniform", **kw):
        if input_dim is not None and input_shape is None:
            input_shape = (input_dim,)
        super().__init__(name=name, input_shape=input_shape)
        self.units = int(units)
        self.activation = A.get(activation)
        self.activation_name = A.name_of(activation)
        self.use_bias = use_bias
        self._config_extra = dict(units=self.units, activation=self.activation_name,
                                  use_bias=use_bias)
        if self.input_shape_arg is not None:
            self.build(self.input_shape_arg)

    def build(self, input_shape):
        fin = int(input_shape[-1])
        self.weight = nn.Parameter(torch.empty(self.units, fin))
        _glorot_uniform_(self.weight, fin, self.units)
        self.bias = nn.Parameter(torch.zeros(self.units)) if self.use_bias else None
        self.built = True

    def call(self, x, training=False):
        w = self.weight if self.weight.dtype == x.dtype else self.weight.to(x.dtype)
        b = self.bias
        if b is not None and b.dtype != x.dtype:
            b = b.to(x.dtype)
        return self.activation(F.linear(x, w, b))

    def compute_output_shape(self, s):
        return tuple(s[:-1]) + (self.units,)

    def _keras_weights(self):
        return [self.weight] + ([self.bias] if self.bias is not None else [])

    def get_weights(self):
        out = [self.weight.detach().float().t().cpu().numpy().copy()]   # [in, out]
        if self.bias is not None:
            out.append(self.bias.detach().float().cpu().numpy().copy())
        return out

    def set_weights(self, weights):
        with torch.no_grad():
            self.weight.copy_(torch.as_tensor(np.asarray(weights[0])).t())
            if self.bias is not None:
                self.bias.copy_(torch.as_tensor(np.asarray(weights[1])))


class _Pool2D(Layer):
    _fn = None

    def __init__(self, pool_size=(2, 2), strides=None, padding="valid", name=None,
                 input_shape=None, **kw):
        super().__init__(name=name, input_shape=input_shape)
        self.pool_size = _pair(pool_size)
        self.strides = _pair(strides) if strides is not None else self.pool_size
        self.padding = padding.lower()
        self._config_extra = dict(pool_size=list(self.pool_size), strides=list(self.strides),
                                  padding=self.padding)

    def call(self, x, training=False):
        xc = x.permute(0, 3, 1, 2)
        if self.padding == "same":
            h, w = xc.shape[2], xc.shape[3]
            ph = max((math.ceil(h / self.strides[0]) - 1) * self.strides[0] + self.pool_size[0] - h, 0)
            pw = max((math.ceil(w / self.strides[1]) - 1) * self.strides[1] + self.pool_size[1] - w, 0)
            fill = float("-inf") if type(self)._fn is F.max_pool2d else 0.0
            xc = F.pad(xc, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2), value=fill)
        y = type(self)._fn(xc, self.pool_size, self.strides)
        return y.permute(0, 2, 3, 1)

    def compute_output_shape(self, s):
        h, w, c = s
        if self.padding == "same":
            return (math.ceil(h / self.strides[0]), math.ceil(w / self.strides[1]), c)
        return ((h - self.pool_size[0]) // self.strides[0] + 1,
                (w - self.pool_size[1]) // self.strides[1] + 1, c)


class MaxPooling2D(_Pool2D):
    _fn = staticmethod(F.max_pool2d)


class AveragePooling2D(_Pool2D):
    _fn = staticmethod(F.avg_pool2d)


MaxPool2D = MaxPooling2D
AvgPool2D = AveragePooling2D


class GlobalAveragePooling2D(Layer):
    def call(self, x, training=False):
        return x.mean(dim=(1, 2))

    def compute_output_shape(self, s):
        return (s[-1],)


class Dropout(Layer):
    def __init__(self, rate, name=None, seed=None, **kw):
        super().__init__(name=name)
        self.rate = float(rate)
        self._config_extra = dict(rate=self.rate)

    def call(self, x, training=False):
        return F.dropout(x, self.rate, training=bool(training))


class Flatten(Layer):
    def call(self, x, training=False):
        return x.reshape(x.shape[0], -1)     # NHWC order, as Keras

    def compute_output_shape(self, s):
        return (int(np.prod(s)),)


class Reshape(Layer):
    def __init__(self, target_shape, name=None, **kw):
        super().__init__(name=name)
        self.target_shape = tuple(target_shape)
        self._config_extra = dict(target_shape=list(self.target_shape))

    def call(self, x, training=False):
        return x.reshape((x.shape[0],) + self.target_shape)

    def compute_output_shape(self, s):
        return self.target_shape


class Activation(Layer):
    def __init__(self, activation, name=None, **kw):
        super().__init__(name=name)
        self.activation = A.get(activation)
        self.activation_name = A.name_of(activation)
        self._config_extra = dict(activation=self.activation_name)

    def call(self, x, training=False):
        return self.activation(x)


class BatchNormalization(Layer):
    """Keras BN over the last (channel) axis; momentum in Keras convention."""

    def __init__(self, axis=-1, momentum=0.99, epsilon=1e-3, center=True, scale=True, name=None,
                 input_shape=None, **kw):
        super().__init__(name=name, input_shape=input_shape)
        if axis not in (-1, 3):
            raise ValueError("only channel-last BatchNormalization is supported")
        self.momentum = float(momentum)
        self.epsilon = float(epsilon)
        self.center, self.scale = center, scale
        self._config_extra = dict(momentum=self.momentum, epsilon=self.epsilon, center=center,
                                  scale=scale)
        if self.input_shape_arg is not None:
            self.build(self.input_shape_arg)

    def build(self, input_shape):
        c = int(input_shape[-1])
        self.gamma = nn.Parameter(torch.ones(c)) if self.scale else None
        self.beta = nn.Parameter(torch.zeros(c)) if self.center else None
        self.register_buffer("moving_mean", torch.zeros(c))
        self.register_buffer("moving_variance", torch.ones(c))
        self.built = True

    def call(self, x, training=False):
        from ..ops.bn import batch_norm_act
        xc = x.permute(0, 3, 1, 2)
        y = batch_norm_act(xc, self.gamma, self.beta, self.moving_mean, self.moving_variance,
                           bool(training), 1.0 - self.momentum, self.epsilon)
        return y.permute(0, 2, 3, 1)

    def _keras_weights(self):
        ws = [w for w in (self.gamma, self.beta) if w is not None]
        return ws + [self.moving_mean, self.moving_variance]

    def set_weights(self, weights):
        with torch.no_grad():
            for t, w in zip(self._keras_weights(), weights):
                t.copy_(torch.as_tensor(np.asarray(w)))


LAYERS = {c.__name__: c for c in (InputLayer, Conv2D, Dense, MaxPooling2D, AveragePooling2D,
                                  GlobalAveragePooling2D, Dropout, Flatten, Reshape, Activation,
                                  BatchNormalization)}
