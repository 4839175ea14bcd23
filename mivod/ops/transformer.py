"""Fused transformer elementwise ops (BERT workload, BASELINE.json config 5).

* ``bias_gelu(x, b)``                       -> ``gelu(x + b)``  (erf form)
* ``bias_dropout_add_ln(z, b, res, ln, p)`` -> ``LN(res + dropout(z + b))``

``x`` / ``z`` are GEMM outputs computed WITHOUT bias (``F.linear(a, W)``): the
bias add, activation, dropout, residual add and LayerNorm of a BERT sub-layer
become one HIP kernel forward and one backward, and the bias / LayerNorm
parameter gradients (column sums) come out of the same backward pass
(``csrc/kernels/mv_bert.hip``).  Dropout keep-masks are a counter hash of
(seed, row, col): nothing is stored for the backward.

GPU + bf16 uses the kernels; anything else falls back to the eager PyTorch
composition (also the numerics reference in ``tests/test_transformer_gpu.py``).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import kernels as K


def _fused_ok(t: torch.Tensor) -> bool:
    return (t.is_cuda and t.dtype == torch.bfloat16 and
            os.environ.get("MIVOD_FUSED_TRANSFORMER", "1") != "0")


def _bf16c(t):
    if t is None:
        return None
    return t.to(torch.bfloat16).contiguous()


def _seed(p: float) -> int:
    return int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) if p > 0 else 0


class _BiasGelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, b):
        ctx.b_dtype = b.dtype
        b = _bf16c(b)
        ctx.save_for_backward(x, b)
        return K.native().bias_gelu_fwd(x, b)

    @staticmethod
    def backward(ctx, dy):
        x, b = ctx.saved_tensors
        dx, db = K.native().bias_gelu_bwd(_bf16c(dy), x, b)
        return dx, db.to(ctx.b_dtype)


def bias_gelu(x: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    if _fused_ok(x) and x.shape[-1] % 8 == 0:
        return _BiasGelu.apply(x.contiguous(), b)
    return F.gelu(x + b)


class _BiasDropoutAddLN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, bias, res, gamma, beta, eps, p, seed, slot):
        N = K.native()
        y, v, mean, rstd = N.ln_fwd(z, _bf16c(bias), res, _bf16c(gamma), _bf16c(beta),
                                    float(eps), float(p), int(seed), True)
        ctx.save_for_backward(v, mean, rstd, _bf16c(gamma))
        ctx.slot = slot
        ctx.p, ctx.seed = float(p), int(seed)
        ctx.has_bias, ctx.has_res = bias is not None, res is not None
        ctx.dtypes = (gamma.dtype, beta.dtype, None if bias is None else bias.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        v, mean, rstd, gamma = ctx.saved_tensors
        # the residual use of y (tap) parked its gradient here: the kernel adds it on load
        dy2 = ctx.slot.take() if ctx.slot is not None else None
        dv, dz, dg, db, dbias = K.native().ln_bwd(_bf16c(dy), v, mean, rstd, gamma, ctx.p,
                                                  ctx.seed, ctx.has_bias, _bf16c(dy2))
        if dz is None:
            dz = dv                      # no dropout: d(z + b) == d(sum)
        gd, bd, bsd = ctx.dtypes
        return (dz, dbias.to(bsd) if ctx.has_bias else None, dv if ctx.has_res else None,
                dg.to(gd), db.to(bd), None, None, None, None)


def bias_dropout_add_ln(z: torch.Tensor, bias, residual, ln: torch.nn.LayerNorm,
                        p: float = 0.0, training: bool = True) -> torch.Tensor:
    """``ln(residual + dropout(z + bias))``; ``bias`` / ``residual`` may be None.

    The fused output carries a gradient slot: a second consumer that uses it as a
    residual should receive ``mivod.ops.bn.tap(y)``, so the LayerNorm backward adds
    that gradient while loading ``dy`` instead of autograd adding the two streams
    with a separate kernel (BERT: 48 bf16 adds of [tokens, 1024] per step)."""
    p = float(p) if training else 0.0
    H = z.shape[-1]
    if (_fused_ok(z) and H % 8 == 0 and H <= 4096 and ln.elementwise_affine and
            ln.normalized_shape == (H,)):
        res = None if residual is None else residual.to(torch.bfloat16).contiguous()
        from .bn import GradSlot
        slot = GradSlot() if torch.is_grad_enabled() else None
        y = _BiasDropoutAddLN.apply(z.contiguous(), bias, res, ln.weight, ln.bias, ln.eps,
                                    p, _seed(p), slot)
        if slot is not None:
            y._mv_slot = slot        # a later residual use goes through ops.bn.tap(y)
        return y
    t = z if bias is None else z + bias
    if p > 0:
        t = F.dropout(t, p, True)
    if residual is not None:
        t = residual + t
    return ln(t)


def dropout_keep_mask(M: int, H: int, p: float, seed: int, device=None) -> torch.Tensor:
    """The kernels' keep-mask for a [M, H] tensor (testing / debugging only)."""
    def mix32(x):
        x = x ^ (x >> 16)
        x = (x * 0x7FEB352D) & 0xFFFFFFFF
        x = x ^ (x >> 15)
        x = (x * 0x846CA68B) & 0xFFFFFFFF
        return x ^ (x >> 16)

    rows = torch.arange(M, dtype=torch.int64, device=device).view(M, 1)
    cols = torch.arange(H, dtype=torch.int64, device=device).view(1, H)
    h = mix32((seed + rows * 0x9E3779B1) & 0xFFFFFFFF)
    h = mix32((h + cols * 0x85EBCA6B) & 0xFFFFFFFF)
    thresh = min(int(p * 4294967296.0), 4294967295)
    return h >= thresh
