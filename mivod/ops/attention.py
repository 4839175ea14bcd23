"""Multi-head self-attention for the BERT workload.

``attention(qkv, mask_bias, p_drop)`` takes the fused QKV projection
``[b, s, 3, h, d]`` and returns the context ``[b, s, h*d]``.  The reference
("math") path is batched GEMMs (hipBLASLt) + fp32 softmax; it is also the
numerics reference for the fused MFMA kernel path.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def attention_math(qkv: torch.Tensor, mask_bias=None, p_drop: float = 0.0) -> torch.Tensor:
    b, s, _, h, d = qkv.shape
    q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)          # [b, h, s, d]
    scores = torch.matmul(q, k.transpose(-1, -2)).float() * (1.0 / math.sqrt(d))
    if mask_bias is not None:
        scores = scores + mask_bias.float()
    p = torch.softmax(scores, dim=-1)
    if p_drop > 0:
        p = F.dropout(p, p_drop, True)
    ctx = torch.matmul(p.to(v.dtype), v)                    # [b, h, s, d]
    return ctx.permute(0, 2, 1, 3).reshape(b, s, h * d)


def attention(qkv: torch.Tensor, mask_bias=None, p_drop: float = 0.0) -> torch.Tensor:
    return attention_math(qkv, mask_bias, p_drop)
