"""Per-parameter gradient error of the fused ResNet path vs the plain path."""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mivod.models.resnet import ResNet, to_mixed_bf16  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
base = to_mixed_bf16(ResNet((2, 2, 2, 2), num_classes=10, zero_init_residual=True)).to(dev)
g = torch.Generator(device=dev).manual_seed(1)
x = torch.rand(16, 3, 64, 64, device=dev, generator=g).to(torch.bfloat16).contiguous(
    memory_format=torch.channels_last)
y = torch.randint(0, 10, (16,), device=dev, generator=g)


def run(env):
    for k, v in env.items():
        os.environ[k] = v
    m = copy.deepcopy(base)
    loss = F.cross_entropy(m(x).float(), y)
    loss.backward()
    return float(loss.detach()), {n: p.grad.float().clone() for n, p in m.named_parameters()}


def run32():
    for k, v in off.items():
        os.environ[k] = v
    m = copy.deepcopy(base).float()
    loss = F.cross_entropy(m(x.float()), y)
    loss.backward()
    return float(loss.detach()), {n: p.grad.float().clone() for n, p in m.named_parameters()}


off = {"MIVOD_FUSED_BN": "0", "MIVOD_CONV_DGRAD_FWD": "0", "MIVOD_BN_TAP": "0",
       "MIVOD_DOWNSAMPLE_TAP": "0", "MIVOD_STEM_CHANNELS": "3"}
lp, gp = run32()   # fp32 reference
print("reference: fp32 plain path", flush=True)
for name, env in (("bf16 plain", off),
                  ("fused all", {"MIVOD_FUSED_BN": "1", "MIVOD_CONV_DGRAD_FWD": "1", "MIVOD_BN_TAP": "1",
                                 "MIVOD_DOWNSAMPLE_TAP": "1", "MIVOD_STEM_CHANNELS": "4"}),
                  ("fused, no downsample tap", {"MIVOD_DOWNSAMPLE_TAP": "0"}),
                  ("fused, stem 3ch", {"MIVOD_DOWNSAMPLE_TAP": "1", "MIVOD_STEM_CHANNELS": "3"}),
                  ("fused BN only", {"MIVOD_CONV_DGRAD_FWD": "0", "MIVOD_BN_TAP": "0",
                                     "MIVOD_DOWNSAMPLE_TAP": "0", "MIVOD_STEM_CHANNELS": "3"})):
    lf, gf = run(env)
    errs = sorted(((float((gf[n] - gp[n]).norm() / max(gp[n].norm(), 1e-6)), n) for n in gp),
                  reverse=True)
    print(f"{name}: loss {lf:.5f} vs {lp:.5f}; worst {[(round(e, 3), n) for e, n in errs[:5]]}",
          flush=True)
