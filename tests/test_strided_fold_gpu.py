"""The strided-read kernels behind the projection-shortcut fold's backward (ops.bn.
_Conv1x1BNFold, stride-2 stage entries): x0[:, :, ::2, ::2] is read at the stride grid by
the Gram pass (wgrad1x1 with a gathered second dy stream), the dual-source data-gradient
GEMM (mv_gemm256 AMODE 2 with a gathered A2) and the column-sum statistics pass, instead
of being copied.  Each against the same op on the explicit strided copy / fp32 math."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _nat():
    from mivod.ops import kernels as K
    return K.native()


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("n,c0,k,h,w", [(2, 256, 512, 12, 10), (3, 128, 256, 7, 9),
                                        (1, 512, 1024, 14, 14)])
def test_wgrad1x1_gathered_dy2_matches_copy(cuda, n, c0, k, h, w):
    nat = _nat()
    g = torch.Generator(device=cuda).manual_seed(n + c0 + h)
    x0 = _cl(torch.randn(n, c0, h, w, device=cuda, generator=g).to(torch.bfloat16))
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    dz = _cl(torch.randn(n, k, ho, wo, device=cuda, generator=g).to(torch.bfloat16))
    x0s = _cl(x0[:, :, ::2, ::2])
    got = nat.wgrad1x1(x0, dz, 2, True, x0)
    ref = nat.wgrad1x1(x0, dz, 2, True, x0s)
    assert torch.equal(got, ref)
    a = torch.cat((dz, x0s), 1).float().permute(0, 2, 3, 1).reshape(-1, k + c0)
    b = x0s.float().permute(0, 2, 3, 1).reshape(-1, c0)
    torch.testing.assert_close(got.view(k + c0, c0), a.t() @ b, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("n,k1,c0,h,w", [(2, 512, 256, 12, 10), (3, 1024, 512, 14, 14),
                                         (1, 2048, 1024, 7, 7), (4, 256, 256, 5, 3)])
def test_gemm_dual_bias_strided_matches_fp32(cuda, n, k1, c0, h, w):
    nat = _nat()
    g = torch.Generator(device=cuda).manual_seed(k1 + c0 + h)
    x0 = _cl(torch.randn(n, c0, h, w, device=cuda, generator=g).to(torch.bfloat16))
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    m = n * ho * wo
    a1 = torch.randn(m, k1, device=cuda, generator=g).to(torch.bfloat16)
    b = (torch.randn(c0, k1 + c0, device=cuda, generator=g) / (k1 + c0) ** 0.5).to(torch.bfloat16)
    badd = torch.randn(c0, device=cuda, generator=g)
    d = torch.empty(m, c0, device=cuda, dtype=torch.bfloat16)
    assert nat.gemm_dual_bias_strided(a1, x0, 2, b, badd, d)
    x0s = x0[:, :, ::2, ::2].float().permute(0, 2, 3, 1).reshape(m, c0)
    ref = torch.cat((a1.float(), x0s), 1) @ b.float().t() + badd
    torch.testing.assert_close(d.float(), ref, rtol=1e-2, atol=1e-2 * float(ref.abs().max()))
    # the contiguous dual GEMM on the explicit copy gives the same bits
    d2 = torch.empty_like(d)
    nat.gemm_dual_bias(a1, _cl(x0[:, :, ::2, ::2]).permute(0, 2, 3, 1).reshape(m, c0), b, badd, d2)
    assert torch.equal(d, d2)


def test_gemm_dual_bias_strided_declines(cuda):
    nat = _nat()
    x0 = _cl(torch.zeros(1, 64, 4, 4, device=cuda, dtype=torch.bfloat16))
    a1 = torch.zeros(4, 256, device=cuda, dtype=torch.bfloat16)
    b = torch.zeros(64, 320, device=cuda, dtype=torch.bfloat16)
    d = torch.empty(4, 64, device=cuda, dtype=torch.bfloat16)
    assert not nat.gemm_dual_bias_strided(a1, x0, 2, b, torch.zeros(64, device=cuda), d)


@pytest.mark.parametrize("n,c,h,w,s", [(2, 256, 12, 10, 2), (3, 64, 7, 9, 2), (2, 512, 14, 14, 1),
                                       (5, 1024, 13, 14, 2)])
def test_bn_stats_strided_matches_copy(cuda, n, c, h, w, s):
    nat = _nat()
    g = torch.Generator(device=cuda).manual_seed(n + c + h + s)
    x = _cl(torch.randn(n, c, h, w, device=cuda, generator=g).to(torch.bfloat16))
    got = nat.bn_stats_strided(x, s)
    xs = _cl(x[:, :, ::s, ::s])
    ref = nat.bn_stats(xs, None, None, None, None, 0.0, 0.0)
    torch.testing.assert_close(got[0], ref[0], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(got[0], xs.float().mean((0, 2, 3)), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(got[1], ref[1], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("c,k,h", [(1024, 2048, 14), (256, 512, 9)])
def test_downsample_tap_stats_matches_conv(cuda, monkeypatch, c, k, h):
    """The strided shortcut conv on the 256 x 256 GEMM with its BN's statistics partials
    (ops.bn.downsample_tap(x, conv, shift)) == F.conv2d, partials == sums around shift; the
    weight gradient and the input gradient (parked in x's producer) match the MIOpen
    path's."""
    import copy

    from mivod.ops import bn as B
    from mivod.ops.conv import Conv2d
    torch.manual_seed(0)
    bn0 = B.BatchNorm2d(c).to(cuda)
    conv = Conv2d(c, k, 1, stride=2, bias=False).to(cuda).to(torch.bfloat16).to(
        memory_format=torch.channels_last)
    z0 = _cl(torch.randn(3, c, h, h, device=cuda).to(torch.bfloat16))
    shift = torch.randn(k, device=cuda) * 0.1
    grads = []
    for g256 in (True, False):
        monkeypatch.setattr(B, "_GEMM256", g256)
        b0, c2 = copy.deepcopy(bn0), copy.deepcopy(conv)
        zz = z0.clone().requires_grad_()
        x = b0(zz, relu=True)
        z, part = B.downsample_tap(x, c2, shift)
        ref = torch.nn.functional.conv2d(x.detach().float(), c2.weight.float(), None, 2)
        torch.testing.assert_close(z.float(), ref, rtol=1e-2, atol=1e-2 * float(ref.abs().max()))
        if g256:
            assert part is not None and torch.isfinite(part).all()
            d = z.float().permute(0, 2, 3, 1).reshape(-1, k) - shift
            sm = part.sum(0)
            torch.testing.assert_close(sm[0], d.sum(0), rtol=1e-3, atol=1e-1)
            torch.testing.assert_close(sm[1], (d * d).sum(0), rtol=1e-3, atol=1e-1)
        else:
            assert part is None
        z.float().square().mean().backward()
        grads.append((zz.grad.float(), c2.weight.grad.float()))
    for a, b in zip(*grads):
        torch.testing.assert_close(a, b, rtol=2e-2, atol=2e-2 * float(b.abs().max()))
