"""Diagnostic: ResNet gradients with the conv1-dgrad/BN-backward fusion on and off,
each against an fp32 eager reference of the same weights (relative L2 error)."""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mivod.models.resnet import ResNet, to_mixed_bf16  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
layers = tuple(int(v) for v in os.environ.get("LAYERS", "2,2,2,1").split(","))
bs, hw = int(os.environ.get("BS", 4)), int(os.environ.get("HW", 64))
base = to_mixed_bf16(ResNet(layers, num_classes=10)).to(dev)
x = torch.rand(bs, 3, hw, hw, device=dev).to(torch.bfloat16).contiguous(
    memory_format=torch.channels_last)
tgt = torch.randint(0, 10, (bs,), device=dev)


def grads(model, inp):
    F.cross_entropy(model(inp).float(), tgt).backward()
    return {k: p.grad.float().clone() for k, p in model.named_parameters()}


ref = copy.deepcopy(base).float()
g_ref = grads(ref, x.float())
res = {}
for fuse in ("1", "0"):
    os.environ["MIVOD_CONV_BN_BWD_FUSE"] = fuse
    res[fuse] = grads(copy.deepcopy(base), x)
worst = []
for k in g_ref:
    r = g_ref[k]
    n = r.norm().item() + 1e-12
    ef = (res["1"][k] - r).norm().item() / n
    eu = (res["0"][k] - r).norm().item() / n
    efu = (res["1"][k] - res["0"][k]).norm().item() / n
    worst.append((ef / max(eu, 1e-6), k, ef, eu, efu))
worst.sort(reverse=True)
for q, k, ef, eu, efu in worst[:15]:
    print(f"{k:40s} fused-vs-fp32 {ef:.3e} unfused-vs-fp32 {eu:.3e} fused-vs-unfused {efu:.3e}")
print("max ratio", worst[0][0])
