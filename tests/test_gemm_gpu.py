"""mivod's MFMA NT GEMM (csrc/kernels/mv_gemm.hip) for NHWC 1x1 convolutions and
its fused BN-statistics epilogue, against fp32 PyTorch references; and the fused
conv1x1 -> BN path (ops.bn.conv_bn) against the unfused composition."""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _nat():
    from mivod.ops import kernels as K
    return K.native()


@pytest.mark.parametrize("K,N", [(64, 64), (64, 256), (128, 512), (256, 64), (256, 128),
                                 (512, 128), (512, 256), (1024, 512)])
@pytest.mark.parametrize("M", [1, 63, 64 * 7 + 5, 4096 + 17])
def test_gemm_nt_matches_fp32(cuda, M, K, N):
    nat = _nat()
    g = torch.Generator(device=cuda).manual_seed(M * 7 + K + N)
    a = torch.randn(M, K, device=cuda, generator=g).to(torch.bfloat16)
    b = (torch.randn(N, K, device=cuda, generator=g) / K ** 0.5).to(torch.bfloat16)
    c = torch.full((M, N), float("nan"), device=cuda).to(torch.bfloat16)
    shift = torch.randn(N, device=cuda, generator=g) * 0.1
    P = nat.gemm_partials(M, N, K)
    part = torch.full((P, 2, N), float("nan"), device=cuda)
    nat.gemm_nt(a, b, c, shift, part)
    ref = a.float() @ b.float().t()
    torch.testing.assert_close(c.float(), ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())
    # statistics of the bf16-ROUNDED output around shift, every partial row written
    d = c.float() - shift
    s = part.sum(0)
    assert torch.isfinite(part).all()
    torch.testing.assert_close(s[0], d.sum(0), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(s[1], (d * d).sum(0), rtol=1e-4, atol=1e-3)
    # plain variant writes the same C
    c2 = torch.empty_like(c)
    nat.gemm_nt(a, b, c2, None, None)
    assert torch.equal(c, c2)


def test_gemm_nt_rejects_bad_shapes(cuda):
    nat = _nat()
    a = torch.zeros(8, 96, device=cuda, dtype=torch.bfloat16)
    b = torch.zeros(64, 96, device=cuda, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        nat.gemm_nt(a, b, torch.zeros(8, 64, device=cuda, dtype=torch.bfloat16), None, None)


def test_conv_bn_fused_matches_unfused(cuda, monkeypatch):
    """conv1x1 -> BN(+residual)(+ReLU) with GEMM-epilogue statistics: same forward
    output, running statistics and gradients as the unfused path (to bf16 rounding)."""
    import copy

    from mivod.ops.bn import BatchNorm2d, conv_bn
    from mivod.ops.conv import Conv2d
    torch.manual_seed(0)
    for cin, cout, res in ((64, 256, True), (256, 64, False), (128, 512, True)):
        conv = Conv2d(cin, cout, 1, bias=False).to(cuda).to(torch.bfloat16).to(
            memory_format=torch.channels_last)
        bn = BatchNorm2d(cout).to(cuda)
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.5, 0.5)
            bn.running_mean.uniform_(-0.2, 0.2)
        x0 = torch.randn(4, cin, 14, 14, device=cuda).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        r0 = torch.randn(4, cout, 14, 14, device=cuda).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last) if res else None
        outs = []
        for fuse in ("1", "0"):
            monkeypatch.setenv("MIVOD_CONV_BN_FUSE", fuse)
            c2, b2 = copy.deepcopy(conv), copy.deepcopy(bn)
            x = x0.clone().requires_grad_()
            y = conv_bn(c2, b2, x, relu=True, residual=r0)
            y.float().square().mean().backward()
            outs.append((y.detach().float(), x.grad.float(), c2.weight.grad.float(),
                         b2.weight.grad, b2.running_mean.clone(), b2.running_var.clone()))
        (yf, dxf, dwf, dgf, rmf, rvf), (yu, dxu, dwu, dgu, rmu, rvu) = outs
        torch.testing.assert_close(rmf, rmu, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(rvf, rvu, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(yf, yu, rtol=2e-2, atol=2e-2)
        for a, b in ((dxf, dxu), (dwf, dwu), (dgf, dgu)):
            torch.testing.assert_close(a, b, rtol=5e-2, atol=5e-2 * float(b.abs().max()))
    os.environ.pop("MIVOD_CONV_BN_FUSE", None)


def test_resnet_uses_gemm_stats_path(cuda):
    """The bottleneck's qualifying 1x1 convs run through _Conv1x1Stats."""
    from mivod.models.resnet import ResNet, to_mixed_bf16
    m = to_mixed_bf16(ResNet((1, 1, 1, 1), num_classes=10)).to(cuda)
    x = torch.rand(2, 3, 64, 64, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    out = m(x)
    names, seen, stack = set(), set(), [out.grad_fn]
    while stack:
        f = stack.pop()
        if f is None or f in seen:
            continue
        seen.add(f)
        names.add(type(f).__name__)
        stack.extend(nf for nf, _ in f.next_functions)
    assert any("Conv1x1Stats" in n for n in names), names
