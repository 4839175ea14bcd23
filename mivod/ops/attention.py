"""Multi-head self-attention for the BERT workload.

``attention(qkv, mask_bias, p_drop)`` takes the fused QKV projection
``[b, s, 3, h, d]`` and returns the context ``[b, s, h*d]``.

* GPU, bf16, head dim 64 -> the hand-written MFMA kernels in
  ``csrc/kernels/mv_attn.hip`` (fused QK^T / online softmax / dropout / PV
  forward; FlashAttention-2-style backward with deterministic dQ partials).
* anything else -> ``attention_math`` (batched GEMMs + fp32 softmax), which is
  also the numerics reference for the kernels.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F

from . import kernels as K


def attention_math(qkv: torch.Tensor, mask_bias=None, p_drop: float = 0.0,
                   keep_mask=None) -> torch.Tensor:
    b, s, _, h, d = qkv.shape
    q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)          # [b, h, s, d]
    scores = torch.matmul(q, k.transpose(-1, -2)).float() * (1.0 / math.sqrt(d))
    if mask_bias is not None:
        scores = scores + mask_bias.float().reshape(b, 1, 1, s)
    p = torch.softmax(scores, dim=-1)
    if keep_mask is not None:
        p = p * keep_mask.to(p.dtype) / (1.0 - p_drop)
    elif p_drop > 0:
        p = F.dropout(p, p_drop, True)
    ctx = torch.matmul(p.to(v.dtype), v)                    # [b, h, s, d]
    return ctx.permute(0, 2, 1, 3).reshape(b, s, h * d)


class _FusedAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, mask, p_drop, seed):
        out, lse = K.native().attn_fwd(qkv, mask, float(p_drop), int(seed))
        ctx.save_for_backward(qkv, out, lse, mask)
        ctx.p_drop, ctx.seed = float(p_drop), int(seed)
        b, s, h, d = out.shape
        return out.view(b, s, h * d)

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse, mask = ctx.saved_tensors
        dout = dout.contiguous().view(out.shape)
        if dout.dtype != torch.bfloat16:
            dout = dout.to(torch.bfloat16)
        dqkv = K.native().attn_bwd(qkv, out, dout, lse, mask, ctx.p_drop, ctx.seed)
        return dqkv, None, None, None


def fused_available(qkv: torch.Tensor) -> bool:
    return (qkv.is_cuda and qkv.dtype == torch.bfloat16 and qkv.dim() == 5 and
            qkv.shape[-1] == 64 and os.environ.get("MIVOD_FUSED_ATTENTION", "1") != "0")


def mask_to_key_bias(mask_bias, b, s):
    """[b,1,1,s] additive bias (or None) -> contiguous fp32 [b, s]."""
    if mask_bias is None:
        return None
    return mask_bias.reshape(b, s).float().contiguous()


def attention(qkv: torch.Tensor, mask_bias=None, p_drop: float = 0.0, seed=None) -> torch.Tensor:
    if fused_available(qkv):
        b, s = qkv.shape[0], qkv.shape[1]
        if seed is None:
            seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) if p_drop > 0 else 0
        return _FusedAttention.apply(qkv.contiguous(), mask_to_key_bias(mask_bias, b, s),
                                     p_drop, seed)
    return attention_math(qkv, mask_bias, p_drop)
