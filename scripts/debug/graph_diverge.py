"""Which parameters diverge between an eager step and a HIP-graph replay?"""
import copy
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
torch.manual_seed(0)
base = to_mixed_bf16(ResNet((1, 1, 1, 1), num_classes=10)).to(dev)
models = [copy.deepcopy(base), copy.deepcopy(base)]
opts = [hvd.DistributedOptimizer(FusedSGD(m.parameters(), lr=0.05, momentum=0.9),
                                 named_parameters=m.named_parameters()) for m in models]
g = torch.Generator(device=dev).manual_seed(7)
x = torch.rand(8, 3, 64, 64, device=dev, generator=g).to(torch.bfloat16).contiguous(
    memory_format=torch.channels_last)
y = torch.randint(0, 10, (8,), device=dev, generator=g)


def stepper(m, o):
    def step():
        loss = F.cross_entropy(m(x).float(), y)
        loss.backward()
        o.step()
        o.zero_grad(set_to_none=True)
        return loss.detach()
    return step


def report(tag):
    torch.cuda.synchronize()
    bad = []
    for (n, p), q in zip(models[0].named_parameters(), models[1].parameters()):
        d = (p.float() - q.float()).abs().max().item()
        if d > 1e-3:
            bad.append((n, d))
    print(tag, "diverged params:", len(bad), bad[:12], flush=True)


eager = stepper(models[0], opts[0])
gs = hvd.make_graphed_step(stepper(models[1], opts[1]), opts[1], model=models[1], warmup=2)
for _ in range(2):
    eager()
report("after warmup")
le = eager()
lg = gs()
torch.cuda.synchronize()
print("loss eager", le.item(), "graph", lg.item(), flush=True)
report("after 1 replay")
# mode 2: replay a graph whose step has NO optimizer (fwd+bwd only) and compare grads
m3 = copy.deepcopy(base)
for p in m3.parameters():
    p.grad = None


def fb():
    loss = F.cross_entropy(m3(x).float(), y)
    loss.backward()
    return loss.detach()


side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for _ in range(2):
        for p in m3.parameters():
            p.grad = None
        fb()
torch.cuda.current_stream().wait_stream(side)
ref = {n: p.grad.float().clone() for n, p in m3.named_parameters()}
for p in m3.parameters():
    p.grad = None
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    fb()
for p in m3.parameters():
    p.grad.zero_()
gr.replay()
torch.cuda.synchronize()
bad = []
for n, p in m3.named_parameters():
    d = (p.grad.float() - ref[n]).abs().max().item()
    s = ref[n].abs().max().item()
    if d > 1e-2 * max(s, 1e-6):
        bad.append((n, d, s))
print("fwd+bwd graph: params with wrong grads:", len(bad), bad[:20], flush=True)
