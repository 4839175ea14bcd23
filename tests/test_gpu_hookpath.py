"""GPU: DistributedOptimizer hook path at world size 1 (fused and plain
optimizers) matches the base optimizer; ResNet-50 bf16 step runs through the
native kernels."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hvd():
    import mivod.torch as h
    h.init()
    yield h


def _net(dev):
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Conv2d(3, 16, 3), torch.nn.BatchNorm2d(16), torch.nn.ReLU(),
                            torch.nn.Flatten(), torch.nn.Linear(16 * 14 * 14, 10)).to(dev)
    return m.to(memory_format=torch.channels_last)


@pytest.mark.parametrize("fused", [True, False])
def test_size1_equals_base(hvd, cuda, fused):
    from mivod.optim import FusedSGD
    a = _net(cuda)
    b = copy.deepcopy(a)
    if fused:
        oa = FusedSGD(a.parameters(), lr=0.05, momentum=0.9)
    else:
        oa = torch.optim.SGD(a.parameters(), lr=0.05, momentum=0.9)
    oa = hvd.DistributedOptimizer(oa, named_parameters=a.named_parameters(), bucket_mb=0.01,
                                  first_bucket_mb=0.001)
    ob = torch.optim.SGD(b.parameters(), lr=0.05, momentum=0.9)
    x = torch.randn(8, 3, 16, 16, device=cuda).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=cuda)
    for _ in range(3):
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad()
            F.cross_entropy(m(x), y).backward()
            o.step()
    torch.cuda.synchronize()
    for p, q in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)


def test_resnet50_bf16_step(hvd, cuda):
    from mivod.models.resnet import resnet50, to_mixed_bf16
    from mivod.optim import FusedSGD
    model = to_mixed_bf16(resnet50(num_classes=100)).to(cuda)
    opt = hvd.DistributedOptimizer(FusedSGD(model.parameters(), lr=0.01, momentum=0.9),
                                   named_parameters=model.named_parameters())
    assert len(opt.bucket_plan()) >= 2
    x = torch.randn(8, 3, 64, 64, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 100, (8,), device=cuda)
    losses = []
    for _ in range(5):
        loss = F.cross_entropy(model(x).float(), y)
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(float(loss.detach()))
    assert all(map(lambda v: v == v, losses))
    assert losses[-1] < losses[0], losses


def test_named_allreduce_gpu(hvd, cuda):
    t = torch.randn(1000, device=cuda)
    out = hvd.allreduce(t, name="x")
    torch.testing.assert_close(out, t)
    hs = [hvd.allreduce_async(torch.full((100 + i,), float(i), device=cuda), name=f"t{i}")
          for i in range(5)]
    for i, h in enumerate(hs):
        torch.testing.assert_close(hvd.synchronize(h), torch.full((100 + i,), float(i), device=cuda))
