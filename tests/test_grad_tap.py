"""The gradient side channel behind mivod.ops.bn.tap: the producer of a tensor
that is used twice reads the shortcut's gradient itself.  Pins the autograd
property it relies on (a None gradient still satisfies the dependency edge, so
the producer's backward runs after the tap's) on CPU."""
import torch

from mivod.ops.bn import GradSlot, tap


class _Producer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, slot):
        ctx.slot = slot
        return x * 2

    @staticmethod
    def backward(ctx, g):
        g2 = ctx.slot.take()
        if g2 is not None:
            g = g + g2
        return g * 2, None


def _producer(x):
    slot = GradSlot()
    y = _Producer.apply(x, slot)
    y._mv_slot = slot
    return y


def test_tap_matches_plain_autograd():
    torch.manual_seed(0)
    x = torch.randn(5, 7, requires_grad=True)
    w1, w2 = torch.randn(7, 7), torch.randn(7, 7)
    # chained residual blocks: y = f(y) + y  with the shortcut tapped
    y = _producer(x)
    for _ in range(3):
        z = torch.tanh(y @ w1) @ w2
        y = _producer(z + tap(y))
    y.sum().backward()
    got = x.grad.clone()

    x.grad = None
    y = x * 2
    for _ in range(3):
        z = torch.tanh(y @ w1) @ w2
        y = (z + y) * 2
    y.sum().backward()
    torch.testing.assert_close(got, x.grad)


def test_tap_without_slot_is_identity():
    x = torch.randn(3, requires_grad=True)
    assert tap(x) is x
    with torch.no_grad():
        y = _producer(x)
        assert tap(y) is y
