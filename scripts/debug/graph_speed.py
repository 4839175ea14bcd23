"""Eager vs HIP-graph replay speed of a ResNet-50 fwd+bwd (no optimizer, one stream)."""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402,F401  (MIOpen find-db env setup)
from mivod.models.resnet import resnet50, to_mixed_bf16  # noqa: E402

dev = torch.device("cuda", 0)
bs = int(os.environ.get("BS", 512))
m = to_mixed_bf16(resnet50()).to(dev)
x = torch.rand(bs, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(
    memory_format=torch.channels_last)
y = torch.randint(0, 1000, (bs,), device=dev)


def fb():
    for p in m.parameters():
        p.grad = None
    loss = F.cross_entropy(m(x).float(), y)
    loss.backward()


def timeit(fn, n=10):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        fb()
torch.cuda.current_stream().wait_stream(s)
print("eager fwd+bwd ms", round(timeit(fb), 2), flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    fb()
print("graph fwd+bwd ms", round(timeit(g.replay), 2), flush=True)
print("eager fwd+bwd ms (again)", round(timeit(fb), 2), flush=True)
os.environ["MIVOD_FUSED_BN"] = "0"
with torch.cuda.stream(s):
    for _ in range(2):
        fb()
torch.cuda.current_stream().wait_stream(s)
print("eager fwd+bwd ms, MIOpen BN", round(timeit(fb), 2), flush=True)
g2 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g2):
    fb()
print("graph fwd+bwd ms, MIOpen BN", round(timeit(g2.replay), 2), flush=True)
