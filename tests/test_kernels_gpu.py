"""Numerics of the hand-written gfx950 kernels vs plain PyTorch fp32 references.

Each test runs the HIP kernel (mivod._mvk) on cuda:0 and compares against the
same op written in fp32 PyTorch on the same inputs.  Sizes include odd tails
(1, 63, 4097, 64K+1) and the 161-tensor ResNet-50 gradient layout.
"""
import math

import pytest
import torch

from mivod.ops import kernels as K

pytestmark = pytest.mark.gpu

DTYPES = [torch.float32, torch.bfloat16, torch.float16]
SIZES = [1, 63, 64, 4097, 65537]


def _resnet50_shapes():
    from mivod.models.resnet import resnet50
    return [tuple(p.shape) for p in resnet50().parameters()]


def test_native_loaded(cuda):
    assert K.available(), "HIP kernels must be built and loaded on the GPU box"
    import mivod._mvk  # noqa: F401


@pytest.mark.parametrize("tdt", DTYPES)
@pytest.mark.parametrize("fdt", DTYPES)
def test_pack_unpack_cast_scale(cuda, tdt, fdt):
    torch.manual_seed(0)
    ts = [torch.randn(n, device=cuda).to(tdt) for n in SIZES]
    offs, o = [], 0
    for t in ts:
        offs.append(o)
        o += (t.numel() + 63) // 64 * 64
    flat = torch.zeros(o, dtype=fdt, device=cuda)
    K.pack(ts, flat, offs, scale=0.5)
    for t, off in zip(ts, offs):
        ref = (t.float() * 0.5).to(fdt)
        torch.testing.assert_close(flat[off:off + t.numel()], ref, rtol=0, atol=0)
    outs = [torch.empty_like(t) for t in ts]
    K.unpack(outs, flat, offs, scale=2.0)
    for out, off in zip(outs, offs):
        ref = (flat[off:off + out.numel()].float() * 2.0).to(tdt)
        torch.testing.assert_close(out, ref, rtol=0, atol=0)


def test_pack_channels_last_and_many_tensors(cuda):
    shapes = _resnet50_shapes()
    assert len(shapes) == 161
    ts = []
    for s in shapes:
        t = torch.randn(s, device=cuda, dtype=torch.bfloat16)
        if len(s) == 4:
            t = t.contiguous(memory_format=torch.channels_last)
        ts.append(t)
    offs, o = [], 0
    for t in ts:
        offs.append(o)
        o += (t.numel() + 63) // 64 * 64
    flat = torch.zeros(o, dtype=torch.bfloat16, device=cuda)
    K.pack(ts, flat, offs)
    for t, off in zip(ts, offs):
        torch.testing.assert_close(flat[off:off + t.numel()], K._raw_flat(t), rtol=0, atol=0)


def test_nonfinite_flag(cuda):
    t = torch.ones(10000, device=cuda)
    t[7777] = float("inf")
    flat = torch.zeros(10048, dtype=torch.float16, device=cuda)
    nf = torch.zeros(1, dtype=torch.int32, device=cuda)
    K.pack([t], flat, [0], nonfinite=nf)
    assert nf.item() == 1
    nf.zero_()
    K.pack([torch.ones(100, device=cuda)], flat, [0], nonfinite=nf)
    assert nf.item() == 0


@pytest.mark.parametrize("sd,dd", [(torch.float32, torch.float16), (torch.float16, torch.float32),
                                   (torch.float32, torch.bfloat16), (torch.bfloat16, torch.float32)])
def test_flat_cast(cuda, sd, dd):
    x = torch.randn(100003, device=cuda).to(sd)
    y = torch.empty(100003, device=cuda, dtype=dd)
    K.flat_cast(x, y, 0.25)
    torch.testing.assert_close(y, (x.float() * 0.25).to(dd), rtol=0, atol=0)


def _mk(n, cuda, gdt, mdt):
    torch.manual_seed(1)
    g = torch.randn(n, device=cuda).to(gdt)
    w = torch.randn(n, device=cuda)
    model = torch.empty(n, device=cuda, dtype=mdt) if mdt is not None else None
    return g, w, model


@pytest.mark.parametrize("gdt", DTYPES)
@pytest.mark.parametrize("nesterov", [False, True])
def test_sgd(cuda, gdt, nesterov):
    n = 70001
    g, w, model = _mk(n, cuda, gdt, torch.bfloat16)
    mom = torch.randn(n, device=cuda)
    wr, mr = w.clone(), mom.clone()
    K.sgd_step(g, w, mom, model, lr=0.1, momentum=0.9, weight_decay=1e-4, gscale=0.125,
               nesterov=nesterov)
    d = g.float() * 0.125 + 1e-4 * wr
    mr = 0.9 * mr + d
    d = d + 0.9 * mr if nesterov else mr
    wr = wr - 0.1 * d
    torch.testing.assert_close(mom, mr, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(w, wr, rtol=1e-6, atol=1e-6)
    # the bf16 model copy is exactly the RNE rounding of the kernel's fp32 master
    torch.testing.assert_close(model, w.to(torch.bfloat16), rtol=0, atol=0)


@pytest.mark.parametrize("adamw", [False, True])
@pytest.mark.parametrize("keras_eps", [False, True])
def test_adam(cuda, adamw, keras_eps):
    n = 50001
    g, w, model = _mk(n, cuda, torch.bfloat16, None)
    m = torch.randn(n, device=cuda) * 0.1
    v = torch.rand(n, device=cuda) * 0.1
    wr, mr, vr = w.clone(), m.clone(), v.clone()
    K.adam_step(g, w, m, v, None, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-7, weight_decay=1e-2,
                gscale=0.5, step=7, adamw=adamw, keras_eps=keras_eps)
    gr = g.float() * 0.5
    if not adamw:
        gr = gr + 1e-2 * wr
    mr = 0.9 * mr + 0.1 * gr
    vr = 0.999 * vr + 0.001 * gr * gr
    bc1, bc2 = 1 - 0.9 ** 7, 1 - 0.999 ** 7
    if adamw:
        wr = wr * (1 - 1e-3 * 1e-2)
    if keras_eps:
        den = (vr.sqrt() + 1e-7) / math.sqrt(bc2)
    else:
        den = vr.sqrt() / math.sqrt(bc2) + 1e-7
    wr = wr - (1e-3 / bc1) * mr / den
    torch.testing.assert_close(m, mr, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(v, vr, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(w, wr, rtol=1e-5, atol=1e-6)


def test_adadelta(cuda):
    n = 33333
    g, w, model = _mk(n, cuda, torch.float32, torch.float16)
    sq = torch.rand(n, device=cuda)
    acc = torch.rand(n, device=cuda)
    wr, sr, ar = w.clone(), sq.clone(), acc.clone()
    K.adadelta_step(g, w, sq, acc, model, lr=1.0, rho=0.95, eps=1e-7, weight_decay=0.0)
    sr = 0.95 * sr + 0.05 * g * g
    delta = (ar + 1e-7).sqrt() / (sr + 1e-7).sqrt() * g
    ar = 0.95 * ar + 0.05 * delta * delta
    wr = wr - delta
    torch.testing.assert_close(sq, sr, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(acc, ar, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(w, wr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(model, wr.half(), rtol=1e-3, atol=1e-3)


def test_lars_vs_reference(cuda):
    sizes = [1, 300, 4096, 9000, 64]
    offs, o = [], 0
    for s in sizes:
        offs.append(o)
        o += (s + 63) // 64 * 64
    torch.manual_seed(3)
    g = torch.randn(o, device=cuda).to(torch.bfloat16)
    w = torch.randn(o, device=cuda)
    mom = torch.randn(o, device=cuda)
    table = K.make_chunk_table(sizes, cuda, offs)
    flags = torch.tensor([1, 0, 0, 0, 1], dtype=torch.int32, device=cuda)
    wc, mc = w.cpu().clone(), mom.cpu().clone()
    tc = K.make_chunk_table(sizes, "cpu", offs)
    K.lars_step(g, w, mom, None, table, flags, lr=0.5, momentum=0.9, weight_decay=1e-4,
                eta=0.001, gscale=0.25)
    K.lars_step(g.cpu(), wc, mc, None, tc, flags.cpu(), lr=0.5, momentum=0.9, weight_decay=1e-4,
                eta=0.001, gscale=0.25)
    for s, off in zip(sizes, offs):
        torch.testing.assert_close(w[off:off + s].cpu(), wc[off:off + s], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(mom[off:off + s].cpu(), mc[off:off + s], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("dt", DTYPES)
def test_adasum_dot3_combine(cuda, dt):
    sizes = [5, 4096, 12345, 1]
    offs, o = [], 0
    for s in sizes:
        offs.append(o)
        o += (s + 63) // 64 * 64
    torch.manual_seed(4)
    a = torch.randn(o, device=cuda).to(dt)
    b = torch.randn(o, device=cuda).to(dt)
    table = K.make_chunk_table(sizes, cuda, offs)
    dots = K.seg_dot3(a, b, table)
    for i, (s, off) in enumerate(zip(sizes, offs)):
        x, y = a[off:off + s].double(), b[off:off + s].double()
        ref = torch.tensor([(x * y).sum(), (x * x).sum(), (y * y).sum()], device=cuda)
        torch.testing.assert_close(dots[i].double(), ref, rtol=2e-5, atol=1e-4)
    # determinism: identical bits on a second run
    assert torch.equal(dots, K.seg_dot3(a, b, table))
    a_ref = a.clone()
    K.adasum_combine(a, b, table, dots)
    for i, (s, off) in enumerate(zip(sizes, offs)):
        dot, na, nb = dots[i].tolist()
        ca = 1 - dot / (2 * na) if na >= 1e-8 else 1.0
        cb = 1 - dot / (2 * nb) if nb >= 1e-8 else 1.0
        ref = (ca * a_ref[off:off + s].float() + cb * b[off:off + s].float()).to(dt)
        tol = 0 if dt == torch.float32 else 1e-2
        torch.testing.assert_close(a[off:off + s], ref, rtol=tol, atol=tol if tol else 1e-6)


def test_fused_optimizer_matches_torch_on_gpu(cuda):
    import copy

    from mivod.optim import FusedSGD
    torch.manual_seed(0)
    m1 = torch.nn.Sequential(torch.nn.Conv2d(3, 16, 3), torch.nn.ReLU(), torch.nn.Flatten(),
                             torch.nn.Linear(16 * 14 * 14, 10)).to(cuda)
    m1 = m1.to(memory_format=torch.channels_last)
    m2 = copy.deepcopy(m1)
    o1 = FusedSGD(m1.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    o2 = torch.optim.SGD(m2.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(8, 3, 16, 16, device=cuda).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=cuda)
    for _ in range(4):
        for m, o in ((m1, o1), (m2, o2)):
            o.zero_grad()
            torch.nn.functional.cross_entropy(m(x), y).backward()
            o.step()
    for p, q in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)
