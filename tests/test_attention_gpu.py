"""Fused MFMA attention (mv_attn.hip) vs the fp32 math reference: forward,
backward (dq, dk, dv), key-padding mask, dropout (same counter-hash mask),
odd sequence lengths."""
import math

import pytest
import torch

from mivod.ops import kernels as K
from mivod.ops.attention import _FusedAttention, attention_math

pytestmark = pytest.mark.gpu


def _ref(qkv, mask, p, keep):
    q = qkv.detach().float().requires_grad_()
    return q, attention_math(q, None if mask is None else mask.reshape(qkv.shape[0], 1, 1, -1),
                             p, keep)


@pytest.mark.parametrize("b,s,h", [(2, 128, 4), (1, 64, 2), (3, 200, 2), (1, 512, 2), (2, 17, 1)])
@pytest.mark.parametrize("use_mask", [False, True])
@pytest.mark.parametrize("p_drop", [0.0, 0.1])
def test_fused_attention_matches_reference(cuda, b, s, h, use_mask, p_drop):
    torch.manual_seed(0)
    qkv = (torch.randn(b, s, 3, h, 64, device=cuda) * 1.5).to(torch.bfloat16)
    mask = None
    if use_mask:
        mask = torch.zeros(b, s, device=cuda)
        mask[:, s - max(1, s // 5):] = -10000.0      # pad the tail keys
    seed = 1234
    keep = None
    if p_drop > 0:
        keep = K.native().attn_dropout_mask(b, h, s, p_drop, seed, qkv.device).bool()
        frac = 1.0 - keep.float().mean().item()
        assert abs(frac - p_drop) < 0.02, frac
    x = qkv.clone().requires_grad_()
    out = _FusedAttention.apply(x, mask, p_drop, seed)
    xr, ref = _ref(qkv, mask, p_drop, keep)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)
    g = torch.randn_like(ref)
    out.backward(g.to(torch.bfloat16))
    ref.backward(g)
    gx, gr = x.grad.float(), xr.grad
    scale = gr.abs().max().item()
    for i, nm in enumerate("qkv"):
        err = (gx[:, :, i] - gr[:, :, i]).abs().max().item()
        assert err <= 3e-2 * max(scale, 1e-3) + 2e-2, (nm, err, scale)


def test_fused_attention_deterministic(cuda):
    torch.manual_seed(1)
    qkv = torch.randn(2, 128, 3, 4, 64, device=cuda).to(torch.bfloat16)
    outs = []
    for _ in range(2):
        x = qkv.clone().requires_grad_()
        o = _FusedAttention.apply(x, None, 0.1, 77)
        o.float().sum().backward()
        outs.append((o.detach(), x.grad))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
