"""Fused BatchNorm2d (+ residual add) (+ ReLU) for channels_last bf16 activations.

``BatchNorm2d`` is a drop-in subclass of ``torch.nn.BatchNorm2d`` (same
parameters, buffers and state_dict) whose ``forward(x, residual=None,
relu=False)`` computes ``act(bn(x) + residual)`` in one fused pass with the
hand-written gfx950 kernels of ``csrc/kernels/mv_bn.hip`` (fp32 statistics and
affine params, bf16 activations).  Any other input (CPU, fp32, NCHW, C % 8 != 0)
takes the plain PyTorch path with identical semantics.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import kernels as K


def _fusable(x: torch.Tensor, weight) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.size(1) % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last)
            and (weight is None or weight.dtype == torch.float32))


def _cl(t: torch.Tensor) -> torch.Tensor:
    if t.dtype != torch.bfloat16:
        t = t.to(torch.bfloat16)
    return t.contiguous(memory_format=torch.channels_last)


class _BNActTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, relu, residual):
        nat = K.native()
        y, vec = nat.bn_fwd_train(x, weight, bias, running_mean, running_var, momentum, eps, relu,
                                  residual)
        mode = 2 if (relu and residual is not None) else (1 if relu else 0)
        ctx.mode = mode
        ctx.has_res = residual is not None
        ctx.save_for_backward(x, y if mode == 2 else None, vec, weight)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, vec, weight = ctx.saved_tensors
        dy = _cl(dy)
        need_affine = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        dx, dg, db, dz = K.native().bn_bwd(ctx.mode, dy, x, y, vec, weight, need_affine)
        dres = None
        if ctx.has_res and ctx.needs_input_grad[8]:
            dres = dz if ctx.mode == 2 else dy
        return (dx if ctx.needs_input_grad[0] else None,
                dg if ctx.needs_input_grad[1] else None,
                db if ctx.needs_input_grad[2] else None,
                None, None, None, None, None, dres)


def batch_norm_act(x, weight, bias, running_mean, running_var, training, momentum, eps,
                   relu=False, residual=None):
    """Functional form: ``act(batch_norm(x) + residual)``."""
    if _fusable(x, weight) and (residual is None or (residual.dtype == torch.bfloat16 and
                                                     residual.shape == x.shape)):
        if residual is not None:
            residual = _cl(residual)
        if training:
            return _BNActTrain.apply(x, weight, bias, running_mean, running_var, float(momentum),
                                     float(eps), bool(relu), residual)
        if not (torch.is_grad_enabled() and (x.requires_grad or (weight is not None and
                                                                 weight.requires_grad))):
            inv = torch.rsqrt(running_var.float() + eps)
            scale = inv * (weight if weight is not None else 1.0)
            shift = (bias if bias is not None else 0.0) - running_mean.float() * scale
            return K.native().bn_apply(x, scale.contiguous(), shift.contiguous(), bool(relu),
                                       residual)
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    if residual is not None:
        y = y + residual
    if relu:
        y = F.relu(y)
    return y


class BatchNorm2d(nn.BatchNorm2d):
    """nn.BatchNorm2d with a fused ``forward(x, residual=None, relu=False)``."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self._mv_steps = 0   # host-side num_batches_tracked (saves a GPU add per call)

    def forward(self, x, residual=None, relu=False):
        self._check_input_dim(x)
        momentum = 0.0 if self.momentum is None else self.momentum
        if self.training and self.track_running_stats:
            self._mv_steps += 1
            if self.momentum is None:
                momentum = 1.0 / float(self._mv_steps + int(self.num_batches_tracked.item()))
        bn_training = self.training or (self.running_mean is None and self.running_var is None)
        rm = self.running_mean if (not self.training or self.track_running_stats) else None
        rv = self.running_var if (not self.training or self.track_running_stats) else None
        return batch_norm_act(x, self.weight, self.bias, rm, rv, bn_training, momentum, self.eps,
                              relu, residual)

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        if self._mv_steps and self.num_batches_tracked is not None:
            with torch.no_grad():
                self.num_batches_tracked.add_(self._mv_steps)
            self._mv_steps = 0
        super()._save_to_state_dict(destination, prefix, keep_vars)

    def _load_from_state_dict(self, *args, **kwargs):
        self._mv_steps = 0
        super()._load_from_state_dict(*args, **kwargs)
