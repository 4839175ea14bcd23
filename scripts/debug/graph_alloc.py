"""Graph replays with / without eager allocations between them (memory-ownership check)."""
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


if os.environ.get("FORK") == "1":
    import mivod.torch.graphs as G
    G.GraphedStep._force_fork = True
gs = hvd.make_graphed_step(step, opt, model=m, warmup=2)
losses = []
junk = []
for i in range(6):
    losses.append(gs().clone() if os.environ.get("ALLOC") == "1" else gs())
    if os.environ.get("ALLOC") == "1":
        junk.append(torch.full((4 << 20,), float("nan"), device=dev))   # 16 MB of NaN
    else:
        losses[-1] = float(losses[-1].item()) if False else losses[-1]
    torch.cuda.synchronize()
    print(i, float(losses[-1]), flush=True)
ok = all(torch.isfinite(p).all() for p in m.parameters())
print("ALLOC", os.environ.get("ALLOC"), "DET", os.environ.get("DET"), "params finite:", bool(ok),
      flush=True)
