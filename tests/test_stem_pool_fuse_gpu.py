"""The ResNet stem's maxpool + BN+ReLU backward fused into the stem weight gradient
(mv_stem.hip MvStemPoolBwd, models.resnet._StemBNReluMaxPool): each row's dz is rebuilt
while the weight-gradient kernel stages it, with the math and summation order of the
materialising path (mv_pool.hip maxpool_bwd_k3s2_kernel<true> then stem_wgrad), so the
weight and BN-parameter gradients must equal that path's bit for bit; the model-level
step must match the unfused stem."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("n,with_dy2", [(2, False), (3, True)])
def test_stem_wgrad_pool_bn_matches_materialised(cuda, n, with_dy2):
    from mivod.ops import kernels as K
    nat = K.native()
    g = torch.Generator(device=cuda).manual_seed(n)
    x = _cl(torch.randn(n, 3, 224, 224, device=cuda, generator=g).to(torch.bfloat16))
    w4 = _cl((torch.randn(64, 4, 7, 7, device=cuda, generator=g) / 12).to(torch.bfloat16))
    w4[:, 3] = 0
    gamma = torch.rand(64, device=cuda, generator=g) + 0.5
    beta = torch.randn(64, device=cuda, generator=g) * 0.2
    rm, rv = torch.zeros(64, device=cuda), torch.ones(64, device=cuda)
    z, part = nat.stem_fwd(x, w4, rm)
    vec = nat.bn_finalize(part, gamma, beta, rm, rv, 0.1, 1e-5, z.numel() // 64)
    y, idx = nat.maxpool_fwd(z, vec[2], vec[3], True, 3, 2, 1)
    dy = _cl(torch.randn(y.shape, device=cuda, generator=g).to(torch.bfloat16))
    dy2 = _cl(torch.randn(y.shape, device=cuda, generator=g).to(torch.bfloat16)) if with_dy2 else None
    dz, dg_ref, db_ref = nat.maxpool_bn_bwd(dy, dy2, idx, y, z, vec, gamma)
    dw_ref = nat.stem_wgrad(x, dz)
    dw, dg, db = nat.stem_wgrad_pool_bn(x, dy, dy2, idx, y, z, vec, gamma)
    assert torch.equal(dg, dg_ref) and torch.equal(db, db_ref)
    assert torch.equal(dw, dw_ref)
    # and the weight gradient is the conv's: fp32 reference from the materialised dz
    ref = torch.ops.aten.convolution_backward(dz.float(), F.pad(x.float(), (0, 0, 0, 0, 0, 1)),
                                              w4.float(), None, [2, 2], [3, 3], [1, 1], False,
                                              [0, 0], 1, [False, True, False])[1]
    torch.testing.assert_close(dw.float(), ref, rtol=2e-2, atol=2e-2 * float(ref.abs().max()))


def test_resnet_stem_pool_fusion_matches_unfused(cuda, monkeypatch):
    from mivod.models.resnet import ResNet, to_mixed_bf16
    from mivod.ops import kernels as K
    calls = []
    real = K.native().stem_wgrad_pool_bn

    def counted(*a, **k):
        calls.append(1)
        return real(*a, **k)

    torch.manual_seed(0)
    base = to_mixed_bf16(ResNet((1, 1, 1, 1), num_classes=10)).to(cuda)
    x = _cl(torch.rand(2, 3, 224, 224, device=cuda).to(torch.bfloat16))
    tgt = torch.randint(0, 10, (2,), device=cuda)
    res = {}
    for on in ("1", "0"):
        monkeypatch.setenv("MIVOD_STEM_POOL_FUSE", on)
        monkeypatch.setattr(K.native(), "stem_wgrad_pool_bn", counted)
        calls.clear()
        m = copy.deepcopy(base)
        out = m(x)
        F.cross_entropy(out.float(), tgt).backward()
        res[on] = (out.float(), {k: p.grad.float() for k, p in m.named_parameters()},
                   {k: v.float() for k, v in m.state_dict().items() if "running" in k}, len(calls))
    assert res["1"][3] == 1 and res["0"][3] == 0
    # (not bitwise: library convs elsewhere in the model may pick nondeterministic solvers)
    torch.testing.assert_close(res["1"][0], res["0"][0], rtol=1e-3, atol=1e-3)
    for k, v in res["0"][1].items():
        torch.testing.assert_close(res["1"][1][k], v, rtol=1e-2, atol=1e-2 * float(v.abs().max()),
                                   msg=k)
    for k, v in res["0"][2].items():
        torch.testing.assert_close(res["1"][2][k], v, rtol=1e-3, atol=1e-4, msg=k)
