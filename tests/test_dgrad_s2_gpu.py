"""Stride-2 3x3 data gradient as output-parity-class gather GEMMs (csrc/kernels/
mv_gemm256.hip AMODE 4, mv_conv.hip conv3x3_kernel DG) against an fp32 PyTorch reference,
and through the ResNet conv path."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _nat():
    from mivod.ops import kernels as K
    return K.native()


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def _wt(w):
    return _cl(w.transpose(0, 1).flip(2, 3))


def _ref_dx(dy, w, h, wd):
    """fp32 input gradient of conv2d(x, w, stride 2, pad 1) for x [n, c, h, wd]."""
    n, c = dy.shape[0], w.shape[1]
    return torch.ops.aten.convolution_backward(
        dy.float(), torch.zeros(n, c, h, wd, device=dy.device), w.float(), None, [2, 2], [1, 1],
        [1, 1], False, [0, 0], 1, [True, False, False])[0]


# (n, c = dx channels, k = dy channels, h, w): ResNet-50 layer3/4 entries (scaled batch),
# small K, several N tiles, 2-pixel images (every class at the border), 224-row blocks
_SHAPES = [(2, 256, 256, 28, 28), (3, 512, 512, 14, 14), (3, 256, 64, 10, 6),
           (2, 512, 128, 4, 2), (32, 256, 256, 28, 28), (4, 768, 192, 2, 2), (1, 256, 320, 6, 14),
           # dx channels % 256 != 0: conv3x3_kernel's DG mode (128- and 64-wide column tiles)
           (2, 128, 128, 56, 56), (3, 128, 64, 10, 14), (2, 64, 128, 6, 8), (5, 192, 64, 2, 4)]


@pytest.mark.parametrize("n,c,k,h,w", _SHAPES)
def test_dgrad_s2_matches_fp32(cuda, n, c, k, h, w):
    nat = _nat()
    g = torch.Generator(device=cuda).manual_seed(n + c + 3 * k + h)
    ho, wo = h // 2, w // 2
    dy = _cl(torch.randn(n, k, ho, wo, device=cuda, generator=g).to(torch.bfloat16))
    wgt = (torch.randn(k, c, 3, 3, device=cuda, generator=g) / (9 * k) ** 0.5).to(torch.bfloat16)
    r = nat.conv3x3_s2_dgrad(dy, _wt(wgt), h, w)
    assert len(r) == 1
    dx = r[0]
    ref = _ref_dx(dy, wgt, h, w)
    assert dx.shape == ref.shape and dx.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(dx.float(), ref, rtol=1e-2, atol=1e-2 * float(ref.abs().max()))


def test_dgrad_s2_declines_uncovered_shapes(cuda):
    nat = _nat()
    dy = _cl(torch.zeros(1, 64, 4, 4, device=cuda, dtype=torch.bfloat16))
    w32 = torch.zeros(64, 32, 3, 3, device=cuda, dtype=torch.bfloat16)
    assert nat.conv3x3_s2_dgrad(dy, _wt(w32), 8, 8) == []       # dx channels % 64 != 0
    w256 = torch.zeros(64, 256, 3, 3, device=cuda, dtype=torch.bfloat16)
    assert nat.conv3x3_s2_dgrad(dy, _wt(w256), 7, 7) == []      # odd input size
    with pytest.raises(RuntimeError):
        nat.conv3x3_s2_dgrad(dy, _wt(w256), 12, 12)             # does not match dy


@pytest.mark.parametrize("c,h", [(256, 14), (512, 8), (128, 16)])
def test_conv_bn_s2_backward_matches_miopen(cuda, monkeypatch, c, h):
    """BN+ReLU -> stride-2 3x3 conv -> BN: the parity-class data gradient == MIOpen's
    backward-data (the whole chain's input, weight and BN-parameter gradients)."""
    from mivod.ops.bn import BatchNorm2d, conv_bn
    from mivod.ops.conv import Conv2d
    torch.manual_seed(0)
    bn0 = BatchNorm2d(c).to(cuda)
    conv = Conv2d(c, c, 3, stride=2, padding=1, bias=False).to(cuda).to(torch.bfloat16).to(
        memory_format=torch.channels_last)
    bn = BatchNorm2d(c).to(cuda)
    with torch.no_grad():
        for b in (bn0, bn):
            b.weight.uniform_(0.5, 1.5)
            b.bias.uniform_(-0.5, 0.5)
    z0 = _cl(torch.randn(4, c, h, h, device=cuda).to(torch.bfloat16))
    outs = []
    for on in ("1", "0"):
        monkeypatch.setenv("MIVOD_CONV3X3_DGRAD_S2", on)
        b0, c2, b2 = copy.deepcopy(bn0), copy.deepcopy(conv), copy.deepcopy(bn)
        z = z0.clone().requires_grad_()
        y = conv_bn(c2, b2, b0(z, relu=True), relu=True)
        y.float().square().mean().backward()
        outs.append((z.grad.float(), c2.weight.grad.float(), b0.weight.grad, b0.bias.grad))
    for a, b in zip(*outs):
        torch.testing.assert_close(a, b, rtol=5e-2, atol=5e-2 * float(b.abs().max()))


def test_resnet_uses_dgrad_s2(cuda, monkeypatch):
    """Every stride-2 conv2 takes the parity-class kernels in a ResNet backward."""
    from mivod.models.resnet import ResNet, to_mixed_bf16
    nat = _nat()
    calls = []
    real = nat.conv3x3_s2_dgrad

    def counted(*a):
        r = real(*a)
        calls.append((a[1].shape[0], len(r)))
        return r

    monkeypatch.setattr(nat, "conv3x3_s2_dgrad", counted)
    torch.manual_seed(0)
    m = to_mixed_bf16(ResNet((1, 1, 2, 1), num_classes=10)).to(cuda)
    x = _cl(torch.rand(4, 3, 64, 64, device=cuda).to(torch.bfloat16))
    F.cross_entropy(m(x).float(), torch.randint(0, 10, (4,), device=cuda)).backward()
    # layer2.0 (128 ch, 16x16 -> 8x8), layer3.0 (256 ch, 8x8 -> 4x4), layer4.0 (512 ch)
    assert sorted(calls) == [(128, 1), (256, 1), (512, 1)], calls
