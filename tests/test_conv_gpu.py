"""mivod's implicit-GEMM 3x3 convolution (csrc/kernels/mv_conv.hip) against an fp32
PyTorch reference, plus its fused BN-statistics epilogue."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _nat():
    from mivod.ops import kernels as K
    return K.native()


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("n,c,h,w,k,s", [(2, 64, 9, 7, 64, 1), (3, 64, 16, 16, 128, 1),
                                         (2, 128, 12, 10, 128, 2), (1, 256, 7, 7, 256, 1),
                                         (2, 128, 15, 13, 64, 2), (4, 64, 56, 56, 64, 1),
                                         (2, 512, 7, 7, 512, 1)])
def test_conv3x3_matches_fp32(cuda, n, c, h, w, k, s):
    nat = _nat()
    g = torch.Generator(device=cuda).manual_seed(n * 1000 + c + h + k + s)
    x = _cl(torch.randn(n, c, h, w, device=cuda, generator=g).to(torch.bfloat16))
    wt = _cl((torch.randn(k, c, 3, 3, device=cuda, generator=g) / (9 * c) ** 0.5).to(torch.bfloat16))
    ref = F.conv2d(x.float(), wt.float(), None, s, 1)
    y = nat.conv3x3(x, wt, s)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2 * float(ref.abs().max()))
    # statistics epilogue: same output, per-channel sums of the bf16 output around shift
    M = ref.shape[0] * ref.shape[2] * ref.shape[3]
    P = nat.conv3x3_partials(M, k)
    part = torch.full((P, 2, k), float("nan"), device=cuda)
    shift = torch.randn(k, device=cuda, generator=g) * 0.1
    y2 = nat.conv3x3(x, wt, s, shift, part)
    assert torch.equal(y, y2)
    d = y.float().permute(0, 2, 3, 1).reshape(-1, k) - shift
    assert torch.isfinite(part).all()
    sm = part.sum(0)
    torch.testing.assert_close(sm[0], d.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(sm[1], (d * d).sum(0), rtol=1e-4, atol=1e-2)


def test_conv3x3_rejects_bad_shapes(cuda):
    nat = _nat()
    x = _cl(torch.zeros(1, 32, 8, 8, device=cuda, dtype=torch.bfloat16))
    w = _cl(torch.zeros(64, 32, 3, 3, device=cuda, dtype=torch.bfloat16))
    with pytest.raises(RuntimeError):
        nat.conv3x3(x, w, 1)
    x = _cl(torch.zeros(1, 64, 8, 8, device=cuda, dtype=torch.bfloat16))
    w = _cl(torch.zeros(64, 64, 3, 3, device=cuda, dtype=torch.bfloat16))
    with pytest.raises(RuntimeError):
        nat.conv3x3(x, w, 3)
