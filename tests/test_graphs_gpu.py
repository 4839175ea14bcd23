"""HIP-graph captured training step (mivod.torch.make_graphed_step) == eager steps.

Two identical models train side by side on the same static batch: one eagerly,
one through a captured graph (eager warmup, then replays).  The learning rate
changes between replays (the fused kernels must read it from device memory,
not from the launch arguments baked at capture time).  Parameters, optimizer
state and BN running statistics must match the eager run."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _small_resnet():
    # zero_init_residual: a random-init ResNet without it is chaotic at this tiny
    # size — bf16 rounding flips from the running-mean shift of the fused BN
    # statistics (scripts/debug/grad_repro.py) grow into 50% weight-grad
    # differences between two otherwise identical eager runs.
    from mivod.models.resnet import ResNet, to_mixed_bf16
    torch.manual_seed(0)
    return to_mixed_bf16(ResNet((1, 1, 1, 1), num_classes=10, zero_init_residual=True))


@pytest.mark.parametrize("kind", ["sgd", "adam", "lars"])
def test_graphed_step_matches_eager(cuda, kind):
    import mivod.torch as hvd
    from mivod.optim import FusedAdam, FusedLARS, FusedSGD

    hvd.init()
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    base = _small_resnet().to(cuda)
    models = [copy.deepcopy(base), copy.deepcopy(base)]

    def make(m):
        if kind == "sgd":
            o = FusedSGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
        elif kind == "adam":
            o = FusedAdam(m.parameters(), lr=1e-3)
        else:
            o = FusedLARS(m.parameters(), lr=0.5, momentum=0.9, weight_decay=1e-4)
        return hvd.DistributedOptimizer(o, named_parameters=m.named_parameters())

    opts = [make(m) for m in models]
    g = torch.Generator(device=cuda).manual_seed(7)
    x = torch.rand(8, 3, 64, 64, device=cuda, generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=cuda, generator=g)

    def stepper(m, o):
        def step():
            loss = F.cross_entropy(m(x).float(), y)
            loss.backward()
            o.step()
            o.zero_grad(set_to_none=True)
            return loss.detach()
        return step

    eager = stepper(models[0], opts[0])
    for _ in range(2):           # the graphed side runs 2 eager warmup steps
        eager()
    graphed = hvd.make_graphed_step(stepper(models[1], opts[1]), opts[1], model=models[1],
                                    warmup=2)
    lrs = [None, None, 0.5, 0.5, 0.25]
    for lr in lrs:
        if lr is not None:
            for o in opts:
                for grp in o.param_groups:
                    grp["lr"] = grp["lr"] * lr
        le = eager()
        lg = graphed()
        torch.cuda.synchronize()
        torch.testing.assert_close(lg, le, rtol=1e-2, atol=1e-2)
    assert graphed.replays == len(lrs)
    torch.cuda.synchronize()
    for (n, p), q in zip(models[0].named_parameters(), models[1].parameters()):
        torch.testing.assert_close(q.float(), p.float(), rtol=2e-2, atol=2e-2, msg=n)
    sa, sb = models[0].state_dict(), models[1].state_dict()
    for k in sa:
        if sa[k].is_floating_point():
            torch.testing.assert_close(sb[k].float(), sa[k].float(), rtol=2e-2, atol=2e-2, msg=k)
        else:
            assert torch.equal(sa[k], sb[k]), k
    torch.backends.cudnn.deterministic = False
    assert opts[1]._mvd_steps == opts[0]._mvd_steps
    hvd.shutdown()


def test_graphed_step_rejects_plain_optimizer(cuda):
    import mivod.torch as hvd
    hvd.init()
    m = torch.nn.Linear(4, 4).to(cuda)
    opt = hvd.DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.1),
                                   named_parameters=m.named_parameters())
    with pytest.raises(TypeError):
        hvd.make_graphed_step(lambda: None, opt)
    hvd.shutdown()


@pytest.mark.parametrize("kind", ["sgd", "adam", "adadelta"])
def test_dyn_hyperparameters_override_launch_args(cuda, kind):
    """With a dyn block the kernels take lr / first / bias corrections from device
    memory (what a graph replay refreshes), not from the scalar arguments."""
    from mivod.ops import kernels as K
    torch.manual_seed(3)
    n = 1000
    g = torch.randn(n, device=cuda)
    w0 = torch.randn(n, device=cuda)
    s0 = torch.rand(n, device=cuda)
    s1 = torch.rand(n, device=cuda)
    dyn = torch.tensor([0.3, 0.0, 1 - 0.9 ** 5, 1 - 0.999 ** 5], device=cuda)

    def run(lr, dyn_t, first, step):
        w, a, b = w0.clone(), s0.clone(), s1.clone()
        if kind == "sgd":
            K.sgd_step(g, w, a, None, lr=lr, momentum=0.9, first=first, dyn=dyn_t)
        elif kind == "adam":
            K.adam_step(g, w, a, b, None, lr=lr, step=step, dyn=dyn_t)
        else:
            K.adadelta_step(g, w, a, b, None, lr=lr, dyn=dyn_t)
        return w

    got = run(99.0, dyn, True, 1)          # bogus scalars: the dyn block must win
    want = run(0.3, None, False, 5)
    torch.testing.assert_close(got, want, rtol=1e-6, atol=1e-6)
