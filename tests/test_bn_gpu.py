"""Fused NHWC BatchNorm(+add)(+ReLU) kernels vs a plain PyTorch fp32 reference."""
import pytest
import torch
import torch.nn.functional as F

from mivod.ops import kernels as K
from mivod.ops.bn import BatchNorm2d, batch_norm_act

pytestmark = pytest.mark.gpu

SHAPES = [(4, 64, 8, 8), (2, 256, 7, 7), (3, 2048, 3, 3), (2, 96, 5, 5), (8, 512, 14, 14),
          (2, 64, 1, 1)]


def _ref(x, w, b, rm, rv, mom, eps, relu, res):
    xf = x.float()
    y = F.batch_norm(xf, rm, rv, w, b, True, mom, eps)
    if res is not None:
        y = y + res.float()
    if relu:
        y = F.relu(y)
    return y


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("relu,use_res", [(False, False), (True, False), (True, True),
                                          (False, True)])
def test_bn_fused_train(cuda, shape, relu, use_res):
    assert K.available()
    torch.manual_seed(0)
    N, C, H, W = shape
    x = (torch.randn(shape, device=cuda) * 2 + 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    res = (torch.randn(shape, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last) if use_res else None)
    w = (torch.rand(C, device=cuda) + 0.5).requires_grad_()
    b = (torch.randn(C, device=cuda) * 0.1).requires_grad_()
    rm = torch.randn(C, device=cuda) * 0.1
    rv = torch.rand(C, device=cuda) + 0.5
    rm2, rv2 = rm.clone(), rv.clone()
    xr = x.detach().float().requires_grad_()
    x1 = x.detach().clone().requires_grad_()
    r1 = res.detach().clone().requires_grad_() if use_res else None
    rr = res.detach().float().requires_grad_() if use_res else None
    w2 = w.detach().clone().requires_grad_()
    b2 = b.detach().clone().requires_grad_()

    y = batch_norm_act(x1, w, b, rm, rv, True, 0.1, 1e-5, relu, r1)
    yr = _ref(xr, w2, b2, rm2, rv2, 0.1, 1e-5, relu, rr)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(rm, rm2, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rv, rv2, rtol=1e-4, atol=1e-5)

    g = torch.randn(shape, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y.backward(g)
    # reference backward through the bf16-rounded output's mask (torch semantics
    # use the output for ReLU backward)
    yr.backward(g.float())
    torch.testing.assert_close(x1.grad.float(), xr.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(w.grad, w2.grad, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(b.grad, b2.grad, rtol=2e-2, atol=2e-2)
    if use_res:
        torch.testing.assert_close(r1.grad.float(), rr.grad, rtol=2e-2, atol=2e-2)


def test_bn_eval_and_module(cuda):
    torch.manual_seed(1)
    m = BatchNorm2d(128).to(cuda)
    ref = torch.nn.BatchNorm2d(128).to(cuda)
    ref.load_state_dict(m.state_dict())
    x = torch.randn(4, 128, 9, 9, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    for _ in range(3):
        m(x, relu=True)
        ref(x.float())
    torch.testing.assert_close(m.running_mean, ref.running_mean, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(m.running_var, ref.running_var, rtol=1e-4, atol=1e-5)
    sd = m.state_dict()
    assert int(sd["num_batches_tracked"]) == 3
    m.eval()
    ref.eval()
    with torch.no_grad():
        torch.testing.assert_close(m(x, relu=True).float(), F.relu(ref(x.float())), rtol=2e-2,
                                   atol=2e-2)


def test_bn_deterministic(cuda):
    torch.manual_seed(2)
    x = torch.randn(16, 256, 14, 14, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = torch.ones(256, device=cuda)
    b = torch.zeros(256, device=cuda)
    outs = []
    for _ in range(2):
        rm, rv = torch.zeros(256, device=cuda), torch.ones(256, device=cuda)
        outs.append((batch_norm_act(x, w, b, rm, rv, True, 0.1, 1e-5, True, None), rm, rv))
    for a, c in zip(outs[0], outs[1]):
        assert torch.equal(a, c)
