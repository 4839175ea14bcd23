"""Gradient error vs an fp32 eager reference: recompute on / off (two runs each)."""
import copy
import sys
import torch
import torch.nn.functional as F
sys.path.insert(0, ".")
from mivod.models.resnet import ResNet, to_mixed_bf16
from mivod.ops import bn as B

cuda = torch.device("cuda")
torch.manual_seed(0)
base = to_mixed_bf16(ResNet((2, 2, 2, 1), num_classes=10)).to(cuda)
x = torch.rand(16, 3, 64, 64, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
tgt = torch.randint(0, 10, (16,), device=cuda)


def grads(m, inp):
    F.cross_entropy(m(inp).float(), tgt).backward()
    return {k: p.grad.float() for k, p in m.named_parameters()}


ref = grads(copy.deepcopy(base).float(), x.float())
res = {}
for name, rc in (("off", False), ("on", True), ("off2", False), ("on2", True)):
    B._RECOMPUTE = rc
    g = grads(copy.deepcopy(base), x)
    res[name] = {k: float((g[k] - r).norm()) / (float(r.norm()) + 1e-12) for k, r in ref.items()}
import statistics
for name, e in res.items():
    print(name, "median rel err", round(statistics.median(e.values()), 4), "max", round(max(e.values()), 4))
worst = sorted(ref, key=lambda k: res["on"][k] - 1.25 * res["off"][k], reverse=True)[:8]
for k in worst:
    print(k, {n: round(res[n][k], 4) for n in res})
