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
                                         (2, 512, 7, 7, 512, 1),
                                         # 64 -> 64 stride 1 = the row-patch kernel
                                         # (mv_conv64.hip): partial last row block, widest
                                         # row (62), 1-pixel rows, and W = 63 (falls back)
                                         (3, 64, 13, 9, 64, 1), (1, 64, 17, 62, 64, 1),
                                         (2, 64, 5, 1, 64, 1), (1, 64, 8, 63, 64, 1),
                                         (9, 64, 56, 56, 64, 1),
                                         # Cout % 256 == 0 = the 256 x 256 pipeline
                                         # (mv_gemm256.hip AMODE 3): stride 2, odd sizes,
                                         # small Cin, several N tiles, partial last M tile
                                         (3, 256, 14, 14, 256, 2), (2, 64, 9, 11, 256, 1),
                                         (5, 512, 7, 7, 512, 2), (9, 256, 14, 14, 512, 1),
                                         (3, 128, 13, 5, 768, 2),
                                         # N * Ho * Wo % 224 == 0: 224-row blocks
                                         (8, 256, 14, 14, 256, 1), (8, 256, 28, 28, 512, 2),
                                         (32, 512, 7, 7, 512, 1)])
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


@pytest.mark.parametrize("c,k,s", [(64, 64, 1), (128, 128, 2), (128, 128, 1), (256, 256, 1)])
def test_conv3x3_bn_matches_unfused(cuda, monkeypatch, c, k, s):
    """conv3x3 -> BN+ReLU through mivod's kernel (statistics in the epilogue, own or
    MIOpen data gradient) vs MIOpen + the separate BN statistics pass."""
    import copy

    from mivod.ops.bn import BatchNorm2d, conv_bn
    from mivod.ops.conv import Conv2d
    torch.manual_seed(0)
    conv = Conv2d(c, k, 3, stride=s, padding=1, bias=False).to(cuda).to(torch.bfloat16).to(
        memory_format=torch.channels_last)
    bn = BatchNorm2d(k).to(cuda)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-0.2, 0.2)
    x0 = _cl(torch.randn(4, c, 14, 14, device=cuda).to(torch.bfloat16))
    outs = []
    for on in ("1", "0"):
        monkeypatch.setenv("MIVOD_CONV3X3", on)
        c2, b2 = copy.deepcopy(conv), copy.deepcopy(bn)
        x = x0.clone().requires_grad_()
        y = conv_bn(c2, b2, x, relu=True)
        y.float().square().mean().backward()
        outs.append((y.detach().float(), x.grad.float(), c2.weight.grad.float(), b2.weight.grad,
                     b2.running_mean.clone(), b2.running_var.clone()))
    (yf, dxf, dwf, dgf, rmf, rvf), (yu, dxu, dwu, dgu, rmu, rvu) = outs
    torch.testing.assert_close(rmf, rmu, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rvf, rvu, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(yf, yu, rtol=2e-2, atol=2e-2)
    for a, b in ((dxf, dxu), (dwf, dwu), (dgf, dgu)):
        torch.testing.assert_close(a, b, rtol=5e-2, atol=5e-2 * float(b.abs().max()))


def test_resnet_bottleneck_uses_conv3x3(cuda):
    from mivod.models.resnet import ResNet, to_mixed_bf16
    m = to_mixed_bf16(ResNet((1, 1, 1, 1), num_classes=10)).to(cuda)
    x = _cl(torch.rand(2, 3, 64, 64, device=cuda).to(torch.bfloat16))
    out = m(x)
    names, seen, stack = set(), set(), [out.grad_fn]
    while stack:
        f = stack.pop()
        if f is None or f in seen:
            continue
        seen.add(f)
        names.add(type(f).__name__)
        stack.extend(nf for nf, _ in f.next_functions)
    assert any("Conv3x3" in n for n in names), names


@pytest.mark.parametrize("c,k,ks", [(64, 64, 3), (128, 128, 3), (64, 128, 3), (64, 256, 1),
                                    (128, 512, 1), (512, 2048, 1),
                                    # output channels % 256 == 0: mv_gemm256.hip AMODE 3 + EPI 4
                                    (256, 256, 3), (512, 512, 3), (256, 64, 3), (512, 128, 1)])
@pytest.mark.parametrize("n,h,w", [(3, 11, 9), (32, 7, 7)])    # M = 1568: 224-row blocks
def test_conv3x3_bn_bwd_matches_reference(cuda, c, k, ks, n, h, w):
    """dgrad (forward conv with the transposed filter; 3x3 or 1x1) + mode-1 BN backward
    reduce in the epilogue == conv2d + relu mask + (sum d, sum d (x - mean)) in fp32."""
    nat = _nat()
    g = torch.Generator(device=cuda).manual_seed(c + 7 * k + n)
    dy = _cl(torch.randn(n, k, h, w, device=cuda, generator=g).to(torch.bfloat16))
    wt = _cl((torch.randn(c, k, ks, ks, device=cuda, generator=g) / (ks * ks * k) ** 0.5).to(
        torch.bfloat16))
    xb = _cl(torch.randn(n, c, h, w, device=cuda, generator=g).to(torch.bfloat16))
    vec = torch.randn(4, c, device=cuda, generator=g)
    d, part = nat.conv3x3_bn_bwd(dy, wt, xb, vec)
    dg = F.conv2d(dy.float(), wt.float(), None, 1, ks // 2).to(torch.bfloat16).float()
    on = (xb.float() * vec[2].view(1, -1, 1, 1) + vec[3].view(1, -1, 1, 1)) > 0
    ref = torch.where(on, dg, torch.zeros_like(dg))
    torch.testing.assert_close(d.float(), ref, rtol=2e-2, atol=2e-2 * float(ref.abs().max()))
    rr = ref.permute(0, 2, 3, 1).reshape(-1, c)
    xr = xb.float().permute(0, 2, 3, 1).reshape(-1, c)
    sm = part.sum(0)
    torch.testing.assert_close(sm[0], rr.sum(0), rtol=2e-2, atol=0.5)
    torch.testing.assert_close(sm[1], (rr * (xr - vec[0])).sum(0), rtol=2e-2, atol=1.0)


def test_resnet_uses_conv3x3_bwd_fusion(cuda, monkeypatch):
    """conv2's data gradient carries BN1's backward reduce on every stride-1 conv2."""
    from mivod.models.resnet import ResNet, to_mixed_bf16
    nat = _nat()
    calls = []
    real = nat.conv3x3_bn_bwd

    def counted(*a):
        calls.append(a[1].shape[2])
        return real(*a)

    monkeypatch.setattr(nat, "conv3x3_bn_bwd", counted)
    monkeypatch.setenv("MIVOD_CONV3X3_DGRAD", "1")     # every width (default: <= 128)
    torch.manual_seed(0)
    m = to_mixed_bf16(ResNet((2, 2, 2, 1), num_classes=10)).to(cuda)
    x = _cl(torch.rand(4, 3, 64, 64, device=cuda).to(torch.bfloat16))
    F.cross_entropy(m(x).float(), torch.randint(0, 10, (4,), device=cuda)).backward()
    # 3x3: layer1.0, layer1.1, layer2.1, layer3.1 (x.0: stride 2)
    assert calls.count(3) == 4, calls


@pytest.mark.parametrize("n,c,k,h,w,s", [(2, 64, 64, 9, 7, 1), (3, 128, 128, 10, 10, 2),
                                         (2, 64, 128, 8, 8, 1), (1, 256, 64, 7, 7, 1),
                                         (2, 64, 64, 9, 8, 1), (1, 64, 64, 3, 4, 1),
                                         (3, 64, 64, 13, 28, 1), (2, 64, 64, 56, 56, 1),
                                         (5, 64, 64, 17, 52, 1),
                                         # C, K % 256 == 0: mv_gemm256.hip wgrad256_kernel<9>
                                         (2, 256, 256, 9, 7, 1), (3, 256, 512, 10, 10, 2),
                                         (2, 512, 256, 7, 7, 1), (9, 256, 256, 14, 14, 1),
                                         (4, 512, 512, 13, 13, 2)])
def test_wgrad3x3_matches_fp32(cuda, n, c, k, h, w, s):
    nat = _nat()
    g = torch.Generator(device=cuda).manual_seed(n + c + k + h + s)
    x = _cl(torch.randn(n, c, h, w, device=cuda, generator=g).to(torch.bfloat16))
    ho, wo = (h - 1) // s + 1, (w - 1) // s + 1
    dy = _cl(torch.randn(n, k, ho, wo, device=cuda, generator=g).to(torch.bfloat16))
    wref = torch.zeros(k, c, 3, 3, device=cuda, requires_grad=True)
    F.conv2d(x.float(), wref, None, s, 1).backward(dy.float())
    dw = nat.wgrad3x3(x, dy, s)
    assert dw.shape == (k, c, 3, 3) and dw.is_contiguous(memory_format=torch.channels_last)
    ref = wref.grad
    torch.testing.assert_close(dw.float(), ref, rtol=2e-2, atol=2e-2 * float(ref.abs().max()))


@pytest.mark.parametrize("n,c,k,h,w,s", [(2, 128, 256, 9, 7, 1), (3, 256, 128, 10, 10, 2),
                                         (2, 64, 256, 8, 9, 1), (2, 256, 64, 7, 7, 1),
                                         (3, 64, 64, 11, 5, 1), (2, 512, 1024, 7, 7, 2),
                                         (1, 64, 128, 3, 3, 2), (3, 512, 256, 9, 9, 1),
                                         (2, 256, 512, 13, 13, 1), (64, 256, 256, 28, 28, 1),
                                         (1, 256, 256, 1, 1, 1)])
def test_wgrad1x1_matches_fp32(cuda, n, c, k, h, w, s):
    """All four tile layouts (128x128, 128x64 / 64x128 with 2 m slices, 64x64 with 4),
    stride 1 and 2 (odd sizes), m tails that are not multiples of the stage rows."""
    nat = _nat()
    g = torch.Generator(device=cuda).manual_seed(n + c + k + h + s)
    x = _cl(torch.randn(n, c, h, w, device=cuda, generator=g).to(torch.bfloat16))
    ho, wo = (h - 1) // s + 1, (w - 1) // s + 1
    dy = _cl(torch.randn(n, k, ho, wo, device=cuda, generator=g).to(torch.bfloat16))
    wref = torch.zeros(k, c, 1, 1, device=cuda, requires_grad=True)
    F.conv2d(x.float(), wref, None, s).backward(dy.float())
    dw = nat.wgrad1x1(x, dy, s)
    assert dw.shape == (k, c, 1, 1)
    ref = wref.grad
    torch.testing.assert_close(dw.float(), ref, rtol=2e-2, atol=2e-2 * float(ref.abs().max()))
    assert torch.equal(nat.wgrad1x1(x, dy, s), dw)          # fixed-order reduce


def test_resnet_uses_wgrad1x1(cuda, monkeypatch):
    """The ResNet bottlenecks' >= 128-channel 1x1 weight gradients (conv1 / conv3 of the
    fused conv+BN path, plain stride-1 1x1 convs and the strided downsample shortcut) run
    on mivod's wgrad1x1 kernel."""
    from mivod.models.resnet import ResNet, to_mixed_bf16
    nat = _nat()
    calls = []
    real = nat.wgrad1x1

    def counted(x, dy, s=1, *rest):
        calls.append((x.shape[1], dy.shape[1], s, bool(rest and rest[0])))
        return real(x, dy, s, *rest)

    monkeypatch.setattr(nat, "wgrad1x1", counted)
    torch.manual_seed(0)
    m = to_mixed_bf16(ResNet((2, 2, 2, 1), num_classes=10)).to(cuda)
    x = _cl(torch.rand(4, 3, 64, 64, device=cuda).to(torch.bfloat16))
    F.cross_entropy(m(x).float(), torch.randint(0, 10, (4,), device=cuda)).backward()
    assert any(s == 2 for _, _, s, _ in calls), calls       # stage-entry shortcut
    # plain weight gradients from 128 channels (the folds' fp32-output products — dz^T x and
    # the Gram x^T x of ops.bn._Conv1x1BNFold — also take 64-channel operands)
    assert all(min(c, k) >= 128 for c, k, _, f in calls if not f), calls
    assert len(calls) >= 10, calls


@pytest.mark.parametrize("n,c,k,h,w,s", [(2, 512, 128, 9, 7, 1), (3, 1024, 256, 7, 7, 1),
                                         (2, 256, 512, 10, 10, 2), (1, 64, 64, 5, 6, 1)])
def test_conv1x1_kernel_matches_fp32(cuda, n, c, k, h, w, s):
    """The implicit-GEMM kernel with ks = 1 (pad 0) against an fp32 1x1 conv, + statistics."""
    nat = _nat()
    g = torch.Generator(device=cuda).manual_seed(n + c + k + s)
    x = _cl(torch.randn(n, c, h, w, device=cuda, generator=g).to(torch.bfloat16))
    wt = _cl((torch.randn(k, c, 1, 1, device=cuda, generator=g) / c ** 0.5).to(torch.bfloat16))
    ref = F.conv2d(x.float(), wt.float(), None, s)
    y = nat.conv1x1(x, wt, s)
    assert y.shape == ref.shape
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2 * float(ref.abs().max()))
    M = ref.shape[0] * ref.shape[2] * ref.shape[3]
    part = torch.full((nat.conv3x3_partials(M, k), 2, k), float("nan"), device=cuda)
    y2 = nat.conv1x1(x, wt, s, None, part)
    assert torch.equal(y, y2)
    d = y.float().permute(0, 2, 3, 1).reshape(-1, k)
    torch.testing.assert_close(part.sum(0)[0], d.sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("n,grid", [(1, 0), (3, 0), (3, 1), (3, 7), (5, 200), (8, 1000)])
def test_stem_kernel_matches_fp32(cuda, n, grid):
    """mv_stem.hip: 7x7/2/pad-3 stem conv (4-channel NHWC image) vs fp32 F.conv2d, and its
    BN-statistics partials vs the statistics of its own bf16 output — with the
    occupancy-sized grid (0) and forced persistent grids smaller and larger than the
    row-pair count (N*56), i.e. workgroups with many rows, one row, or none (round-2
    NaN regression: the result must not depend on the grid or the register allocation)."""
    nat = _nat()
    g = torch.Generator(device=cuda).manual_seed(n)
    x = torch.rand(n, 4, 224, 224, device=cuda, generator=g)
    x[:, 3] = 0
    x = _cl(x.to(torch.bfloat16))
    w = _cl((torch.randn(64, 4, 7, 7, device=cuda, generator=g) * 0.05).to(torch.bfloat16))
    shift = torch.randn(64, device=cuda, generator=g) * 0.1
    z, part = nat.stem_fwd(x, w, shift, grid)
    assert z.shape == (n, 64, 112, 112) and z.is_contiguous(memory_format=torch.channels_last)
    assert grid == 0 or part.shape[0] == grid
    assert bool(torch.isfinite(z).all()) and bool(torch.isfinite(part).all())
    ref = F.conv2d(x.float(), w.float(), None, 2, 3)
    torch.testing.assert_close(z.float(), ref, rtol=1e-2, atol=1e-2 * float(ref.abs().max()))
    d = (z.float() - shift[None, :, None, None]).permute(1, 0, 2, 3).reshape(64, -1)
    s = part.sum(0)
    torch.testing.assert_close(s[0], d.sum(1), rtol=1e-3, atol=1e-1)
    torch.testing.assert_close(s[1], (d * d).sum(1), rtol=1e-3, atol=1e-1)


def test_resnet_stem_kernel_path(cuda, monkeypatch):
    """ResNet at 224x224 takes the stem kernel (fused BN statistics); every parameter
    gradient is as close to the fp32 eager reference as the MIOpen stem path's, the stem
    BN's running statistics match, and the weight gradient of the stem kernel's backward
    equals F.conv2d's for the same upstream gradient."""
    import copy

    from mivod.models.resnet import ResNet, _StemConvStats, to_mixed_bf16
    nat = _nat()
    calls = []
    real = nat.stem_fwd

    def counted(*a):
        calls.append(a[0].shape)
        return real(*a)

    monkeypatch.setattr(nat, "stem_fwd", counted)
    torch.manual_seed(0)
    base = to_mixed_bf16(ResNet((1, 1, 1, 1), num_classes=10)).to(cuda)
    x = _cl(torch.rand(4, 3, 224, 224, device=cuda).to(torch.bfloat16))
    tgt = torch.randint(0, 10, (4,), device=cuda)

    def grads(m, inp):
        F.cross_entropy(m(inp).float(), tgt).backward()
        return ({k: p.grad.float() for k, p in m.named_parameters()},
                (m.bn1.running_mean.clone(), m.bn1.running_var.clone()))

    ref, _ = grads(copy.deepcopy(base).float(), x.float())
    out, st = {}, {}
    for on in ("1", "0"):
        monkeypatch.setenv("MIVOD_STEM_KERNEL", on)
        calls.clear()
        out[on], st[on] = grads(copy.deepcopy(base), x)
        assert (len(calls) == 1) == (on == "1"), calls
    for k, r in ref.items():
        n = float(r.norm()) + 1e-12
        e1 = float((out["1"][k] - r).norm()) / n
        e0 = float((out["0"][k] - r).norm()) / n
        assert e1 <= 1.25 * e0 + 5e-2, (k, e1, e0)
    for a, b in zip(st["1"], st["0"]):
        torch.testing.assert_close(a, b, rtol=1e-2, atol=1e-3)
    # backward of the kernel path == MIOpen's weight gradient through F.conv2d
    x4 = _cl(F.pad(x, (0, 0, 0, 0, 0, 1)))
    w4 = _cl((torch.randn(64, 4, 7, 7, device=cuda) * 0.05).to(torch.bfloat16)).requires_grad_()
    dz = _cl(torch.randn(4, 64, 112, 112, device=cuda).to(torch.bfloat16))
    z, _ = _StemConvStats.apply(x4, w4, None)
    z.backward(dz)
    g1 = w4.grad.float().clone()
    w4.grad = None
    F.conv2d(x4, w4, None, 2, 3).backward(dz)
    torch.testing.assert_close(g1, w4.grad.float(), rtol=2e-2, atol=2e-2 * float(g1.abs().max()))


@pytest.mark.parametrize("n,c,k,h,s", [(2, 64, 256, 9, 1), (2, 128, 512, 8, 1), (1, 256, 512, 10, 2),
                                       (1, 256, 1024, 7, 1), (40, 512, 2048, 7, 1)])
def test_wgrad1x1_dual_dy(cuda, n, c, k, h, s):
    """wgrad1x1 with a second dy stream: [dy | dy2]^T . x == the two products stacked."""
    nat = _nat()
    g = torch.Generator(device=cuda).manual_seed(n + c + k)
    x = _cl(torch.randn(n, c, h, h, device=cuda, generator=g).to(torch.bfloat16))
    ho = (h - 1) // s + 1
    dy = _cl(torch.randn(n, k, ho, ho, device=cuda, generator=g).to(torch.bfloat16))
    dy2 = _cl(torch.randn(n, c, ho, ho, device=cuda, generator=g).to(torch.bfloat16))
    both = nat.wgrad1x1(x, dy, s, True, dy2).view(k + c, c)
    a = nat.wgrad1x1(x, dy, s, True).view(k, c)
    b = nat.wgrad1x1(x, dy2, s, True).view(c, c)
    ref = torch.cat((a, b))
    torch.testing.assert_close(both, ref, rtol=1e-4, atol=1e-3 * float(ref.abs().max()))


@pytest.mark.parametrize("n", [1, 3])
def test_stem_wgrad_kernel_matches_miopen(cuda, n):
    """mv_stem.hip weight gradient vs MIOpen's (fp32-accumulated) for the same dz."""
    nat = _nat()
    g = torch.Generator(device=cuda).manual_seed(10 + n)
    x = torch.rand(n, 4, 224, 224, device=cuda, generator=g)
    x[:, 3] = 0
    x = _cl(x.to(torch.bfloat16))
    w = _cl((torch.randn(64, 4, 7, 7, device=cuda, generator=g) * 0.05).to(torch.bfloat16))
    dz = _cl(torch.randn(n, 64, 112, 112, device=cuda, generator=g).to(torch.bfloat16))
    dw = nat.stem_wgrad(x, dz)
    assert dw.shape == (64, 4, 7, 7) and dw.is_contiguous(memory_format=torch.channels_last)
    ref = torch.ops.aten.convolution_backward(dz.float(), x.float(), w.float(), None, [2, 2],
                                              [3, 3], [1, 1], False, [0, 0], 1,
                                              [False, True, False])[1]
    torch.testing.assert_close(dw.float(), ref, rtol=2e-2, atol=2e-2 * float(ref.abs().max()))


@pytest.mark.parametrize("n,h,w", [(2, 9, 8), (64, 56, 56), (3, 13, 28)])
def test_wgrad64_matches_general_kernel(cuda, n, h, w):
    """The 64 -> 64 row-patch weight gradient (mv_conv64.hip) vs the general wgrad3x3
    kernel on the same inputs (MIVOD_WGRAD64 is read once per process, so the general
    kernel is reached through a shape the row patch does not take: the same data with
    one zero column appended, W + 1 not a multiple of 4)."""
    nat = _nat()
    g = torch.Generator(device=cuda).manual_seed(n + h + w)
    x = torch.randn(n, 64, h, w, device=cuda, generator=g).to(torch.bfloat16)
    dy = torch.randn(n, 64, h, w, device=cuda, generator=g).to(torch.bfloat16)
    dw = nat.wgrad3x3(_cl(x), _cl(dy), 1)
    xp = F.pad(x, (0, 1)).contiguous()
    dyp = F.pad(dy, (0, 1)).contiguous()
    ref = nat.wgrad3x3(_cl(xp), _cl(dyp), 1)
    # the padded column only adds x[.., w] = 0 / dy[.., w] = 0 products
    assert torch.isfinite(dw.float()).all()
    torch.testing.assert_close(dw.float(), ref.float(), rtol=1e-2,
                               atol=1e-2 * float(ref.float().abs().max()))


@pytest.mark.parametrize("n", [1, 3])
def test_stem_kernels_read_rgb_directly(cuda, n):
    """The stem kernels on the raw 3-channel image == on its zero-padded 4-channel copy, bit
    for bit (forward output, statistics partials, weight gradient): no padded input copy."""
    nat = _nat()
    g = torch.Generator(device=cuda).manual_seed(50 + n)
    x3 = _cl(torch.rand(n, 3, 224, 224, device=cuda, generator=g).to(torch.bfloat16))
    x4 = _cl(F.pad(x3, (0, 0, 0, 0, 0, 1)))
    w = _cl((torch.randn(64, 4, 7, 7, device=cuda, generator=g) * 0.05).to(torch.bfloat16))
    shift = torch.randn(64, device=cuda, generator=g) * 0.1
    z3, p3 = nat.stem_fwd(x3, w, shift, 0)
    z4, p4 = nat.stem_fwd(x4, w, shift, 0)
    assert torch.equal(z3, z4) and torch.equal(p3, p4)
    dz = _cl(torch.randn(n, 64, 112, 112, device=cuda, generator=g).to(torch.bfloat16))
    assert torch.equal(nat.stem_wgrad(x3, dz), nat.stem_wgrad(x4, dz))


def test_transpose_filters_matches_torch(cuda):
    """The one-launch data-gradient filters == w.transpose(0, 1).flip(2, 3) for every
    filter (3x3 and 1x1, channel counts off the 64-tile grid), repeated calls reuse the
    cached outputs and follow the current weights."""
    nat = _nat()
    g = torch.Generator(device=cuda).manual_seed(3)
    shapes = [(64, 64, 3), (256, 128, 1), (100, 72, 3), (2048, 512, 1), (3, 5, 7), (512, 512, 3)]
    ws = [_cl(torch.randn(k, c, s, s, device=cuda, generator=g).to(torch.bfloat16))
          for k, c, s in shapes]
    for rnd in range(2):
        outs = nat.transpose_filters(ws)
        for w, o in zip(ws, outs):
            ref = _cl(w.transpose(0, 1).flip(2, 3))
            assert o.shape == ref.shape and o.is_contiguous(memory_format=torch.channels_last)
            assert torch.equal(o, ref)
        with torch.no_grad():
            for w in ws:
                w.mul_(-1.5)


def test_resnet_prepared_dgrad_filters_bitwise(cuda, monkeypatch):
    """Backward with the model-wide prepared filters == the per-conv transposes
    (MIVOD_DGRAD_FILTERS=0: the filters are bitwise equal, the gradients agree to MIOpen's
    run-to-run algorithm choice on the shapes it still runs), and the prepared map is
    closed after the forward."""
    import copy

    from mivod.models.resnet import ResNet, to_mixed_bf16
    from mivod.ops import conv as CV
    torch.manual_seed(0)
    base = to_mixed_bf16(ResNet((2, 1, 2, 1), num_classes=10)).to(cuda)
    x = _cl(torch.rand(4, 3, 64, 64, device=cuda).to(torch.bfloat16))
    tgt = torch.randint(0, 10, (4,), device=cuda)
    res = {}
    for on in ("1", "0"):
        monkeypatch.setenv("MIVOD_DGRAD_FILTERS", on)
        m = copy.deepcopy(base)
        out = m(x)
        assert not CV._DGRAD_FILTERS
        F.cross_entropy(out.float(), tgt).backward()
        res[on] = {k: p.grad for k, p in m.named_parameters()}
    for k, v in res["0"].items():
        torch.testing.assert_close(res["1"][k].float(), v.float(), rtol=1e-2,
                                   atol=1e-2 * float(v.float().abs().max()), msg=k)
