"""Reproducibility of one ResNet fwd+bwd: default stream twice, side stream, HIP graph.
Usage: python grad_repro.py  (env MIVOD_FUSED_BN / MIVOD_CONV_DGRAD_FWD to isolate)."""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mivod.models.resnet import ResNet, to_mixed_bf16  # noqa: E402

dev = torch.device("cuda", 0)
if os.environ.get("DET") == "1":
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
torch.manual_seed(0)
DEPTH = tuple(int(v) for v in os.environ.get("DEPTH", "1,1,1,1").split(","))
IMG = int(os.environ.get("IMG", "64"))
base = to_mixed_bf16(ResNet(DEPTH, num_classes=10)).to(dev)
g = torch.Generator(device=dev).manual_seed(7)
x = torch.rand(8, 3, IMG, IMG, device=dev, generator=g).to(torch.bfloat16).contiguous(
    memory_format=torch.channels_last)
y = torch.randint(0, 10, (8,), device=dev, generator=g)


def fb(m):
    for p in m.parameters():
        p.grad = None
    if os.environ.get("RESET") == "1":     # identical running stats (the BN shift) every run
        with torch.no_grad():
            for mod in m.modules():
                if isinstance(mod, torch.nn.BatchNorm2d):
                    mod.running_mean.zero_()
                    mod.running_var.fill_(1.0)
    loss = F.cross_entropy(m(x).float(), y)
    loss.backward()
    return loss.detach()


def grads(m):
    return {n: p.grad.float().clone() for n, p in m.named_parameters()}


def cmp(tag, a, b):
    worst = max(((a[k] - b[k]).abs().max().item() / max(a[k].abs().max().item(), 1e-12), k)
                for k in a)
    c1 = (a["conv1.weight"] - b["conv1.weight"]).abs().max().item()
    print(f"{tag}: worst rel diff {worst[0]:.3e} ({worst[1]}); conv1 abs diff {c1:.3e}", flush=True)


m = copy.deepcopy(base)
fb(m)
A1 = grads(m)
fb(m)
A2 = grads(m)
cmp("default stream, run1 vs run2", A1, A2)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    fb(m)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
B = grads(m)
cmp("default vs side stream", A1, B)
with torch.cuda.stream(s):
    fb(m)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
cmp("default vs side stream (2nd)", A1, grads(m))
for p in m.parameters():
    p.grad = None
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    loss = F.cross_entropy(m(x).float(), y)
    loss.backward()
gr.replay()
torch.cuda.synchronize()
cmp("default vs graph replay", A1, grads(m))
gr.replay()
torch.cuda.synchronize()
cmp("default vs graph replay (2nd)", A1, grads(m))
