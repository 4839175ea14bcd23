"""BN + ReLU applied while the 64 -> 64 row-patch kernels stage their input (csrc/kernels/
mv_conv64.hip, ops.bn._BNReluConv64): the forward conv and the weight gradient on the BN
INPUT with the affine + ReLU done on load must equal the same kernels on the materialised
bf16 BN output bit for bit, and the fused ResNet layer1 path must match the unfused one."""
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


def _bn_relu(z, sc, bi):
    """The materialised BN + ReLU output: mv_bn.hip's apply kernel, bf16(relu(fma(z, sc, bi)))
    (fp32 fma — an unfused torch multiply-add rounds differently in the last bit)."""
    y = _nat().bn_apply(z, sc, bi, True, None)
    ref = torch.relu(z.float() * sc.view(1, -1, 1, 1) + bi.view(1, -1, 1, 1))
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2)
    return y


@pytest.mark.parametrize("n,h,w", [(3, 13, 9), (2, 56, 56), (4, 7, 40), (1, 1, 5)])
def test_conv64_input_bn_matches_materialised(cuda, n, h, w):
    nat = _nat()
    g = torch.Generator(device=cuda).manual_seed(n + h + w)
    z = _cl(torch.randn(n, 64, h, w, device=cuda, generator=g).to(torch.bfloat16))
    wt = _cl((torch.randn(64, 64, 3, 3, device=cuda, generator=g) / 24.0).to(torch.bfloat16))
    sc = torch.rand(64, device=cuda, generator=g) + 0.5
    bi = torch.randn(64, device=cuda, generator=g) * 0.5
    y = _bn_relu(z, sc, bi)
    m = n * h * w
    p_ref = torch.empty(nat.conv3x3_partials(m, 64), 2, 64, device=cuda)
    p_fus = torch.empty_like(p_ref)
    shift = torch.randn(64, device=cuda, generator=g) * 0.1
    ref = nat.conv3x3(y, wt, 1, shift, p_ref)
    got = nat.conv3x3(z, wt, 1, shift, p_fus, sc, bi)
    assert torch.equal(got, ref)
    assert torch.equal(p_fus, p_ref)
    torch.testing.assert_close(ref.float(), F.conv2d(y.float(), wt.float(), None, 1, 1),
                               rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("n,h,w", [(3, 13, 8), (2, 56, 56), (1, 3, 4)])
def test_wgrad64_input_bn_matches_materialised(cuda, n, h, w):
    nat = _nat()
    g = torch.Generator(device=cuda).manual_seed(7 * n + h + w)
    z = _cl(torch.randn(n, 64, h, w, device=cuda, generator=g).to(torch.bfloat16))
    dy = _cl(torch.randn(n, 64, h, w, device=cuda, generator=g).to(torch.bfloat16))
    sc = torch.rand(64, device=cuda, generator=g) + 0.5
    bi = torch.randn(64, device=cuda, generator=g) * 0.5
    y = _bn_relu(z, sc, bi)
    assert torch.equal(nat.wgrad3x3(z, dy, 1, sc, bi), nat.wgrad3x3(y, dy, 1))


def test_input_bn_rejected_off_the_row_patch_kernels(cuda):
    nat = _nat()
    z = _cl(torch.zeros(1, 128, 8, 8, device=cuda, dtype=torch.bfloat16))
    wt = _cl(torch.zeros(128, 128, 3, 3, device=cuda, dtype=torch.bfloat16))
    v = torch.ones(128, device=cuda)
    with pytest.raises(RuntimeError):
        nat.conv3x3(z, wt, 1, None, None, v, v)
    with pytest.raises(RuntimeError):
        nat.wgrad3x3(z, z, 1, v, v)


def test_resnet_layer1_bn_apply_fusion_matches_unfused(cuda, monkeypatch):
    """ResNet with BN1 applied inside layer1's conv2 kernels == the materialised path:
    output, every parameter gradient and the BN running statistics."""
    from mivod.models.resnet import ResNet, to_mixed_bf16
    from mivod.ops import kernels as K
    calls = []
    real = K.native().conv3x3

    def counted(*a, **k):
        calls.append(len(a) > 5 and a[5] is not None)
        return real(*a, **k)

    torch.manual_seed(0)
    base = to_mixed_bf16(ResNet((2, 1, 1, 1), num_classes=10)).to(cuda)
    x = _cl(torch.rand(4, 3, 64, 64, device=cuda).to(torch.bfloat16))
    tgt = torch.randint(0, 10, (4,), device=cuda)
    res = {}
    for on in ("1", "0"):
        monkeypatch.setenv("MIVOD_BN_APPLY_FUSE", on)
        monkeypatch.setattr(K.native(), "conv3x3", counted)
        calls.clear()
        m = copy.deepcopy(base)
        out = m(x)
        F.cross_entropy(out.float(), tgt).backward()
        res[on] = (out.float(), {k: p.grad.float() for k, p in m.named_parameters()},
                   {k: v.float() for k, v in m.state_dict().items() if "running" in k},
                   sum(calls))
    assert res["1"][3] == 2 and res["0"][3] == 0, (res["1"][3], res["0"][3])   # layer1.0 / .1
    torch.testing.assert_close(res["1"][0], res["0"][0], rtol=1e-2, atol=1e-2)
    for k, v in res["0"][1].items():
        torch.testing.assert_close(res["1"][1][k], v, rtol=2e-2, atol=2e-2 * float(v.abs().max()))
    for k, v in res["0"][2].items():
        torch.testing.assert_close(res["1"][2][k], v, rtol=1e-3, atol=1e-4)
