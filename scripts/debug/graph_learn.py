"""Does a graph replay apply the optimizer update?  Prints dyn blocks and param deltas."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import mivod.torch as hvd  # noqa: E402
from mivod.models.resnet import ResNet, to_mixed_bf16  # noqa: E402
from mivod.optim import FusedSGD  # noqa: E402

hvd.init()
dev = hvd.device()
if os.environ.get("DET") == "1":
    torch.backends.cudnn.deterministic = True
torch.manual_seed(0)
m = to_mixed_bf16(ResNet((1, 1, 1, 1), num_classes=10, zero_init_residual=True)).to(dev)
opt = hvd.DistributedOptimizer(FusedSGD(m.parameters(), lr=0.05, momentum=0.9),
                               named_parameters=m.named_parameters())
x = torch.rand(8, 3, 64, 64, device=dev).to(torch.bfloat16).contiguous(
    memory_format=torch.channels_last)
y = torch.randint(0, 10, (8,), device=dev)


def step():
    loss = F.cross_entropy(m(x).float(), y)
    loss.backward()
    opt.step()
    opt.zero_grad(set_to_none=True)
    return loss.detach()


MODE = os.environ.get("MODE", "graph")
if MODE == "eager_inline":
    opt._mvd_inline = True
    gs = step
else:
    if MODE == "graph_fork":
        opt._mvd_size_saved = opt._mvd_size
        import mivod.torch.graphs as G
        G.GraphedStep._force_fork = True
    gs = hvd.make_graphed_step(step, opt, model=m, warmup=2)
print("MODE", MODE, flush=True)
for i in range(4):
    w0 = m.fc.weight.detach().float().clone()
    mst = opt._mv_arenas[0].master.clone()
    loss = gs()
    torch.cuda.synchronize()
    dyn = [a.dyn.tolist() if a.dyn is not None else None for a in opt._mv_arenas]
    print(f"replay {i}: loss {loss.item():.4f} |dW_fc| {(m.fc.weight.float() - w0).abs().max().item():.3e} "
          f"|d master0| {(opt._mv_arenas[0].master - mst).abs().max().item():.3e} "
          f"dyn {dyn} grad0 |g| "
          f"{opt._mv_arenas[0].grad.float().abs().max().item():.3e}", flush=True)
    names = {id(p): n for n, p in m.named_parameters()}
    for ai, a in enumerate(opt._mv_arenas):
        bad = [names[id(p)] for k, p in enumerate(a.params)
               if not torch.isfinite(a.slot(a.grad, k)).all()]
        if bad:
            print(f"   arena {ai} ({a.dtype}) non-finite grads: {bad}", flush=True)
for i in range(3):
    w0 = m.fc.weight.detach().float().clone()
    loss = step()
    torch.cuda.synchronize()
    print(f"eager {i}: loss {loss.item():.4f} |dW_fc| {(m.fc.weight.float() - w0).abs().max().item():.3e}",
          flush=True)
