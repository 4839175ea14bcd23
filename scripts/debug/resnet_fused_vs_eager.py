"""ResNet-50 forward, bf16 fused (mivod) and bf16 eager, each vs an fp32 eager
reference of the same weights: per-block relative error."""
import copy
import os
import torch
from mivod.models.resnet import resnet50, to_mixed_bf16

dev = torch.device("cuda")
torch.manual_seed(3)
base = resnet50(num_classes=10).to(dev)
B, R = int(os.environ.get("B", 4)), int(os.environ.get("R", 64))
x = torch.randn(B, 3, R, R, device=dev).contiguous(memory_format=torch.channels_last)


def run(model, inp, fused):
    os.environ["MIVOD_FUSED_BN"] = fused
    rec = {}
    hs = [m.register_forward_hook(lambda m, i, o, n=n: rec.__setitem__(n, o.detach().float()))
          for n, m in model.named_modules() if n.count(".") == 1 or n == "fc"]
    with torch.no_grad():
        model.train()
        rec["logits"] = model(inp).detach().float()
    for h in hs:
        h.remove()
    return rec


ref = run(copy.deepcopy(base).to(memory_format=torch.channels_last), x, "0")
bf = to_mixed_bf16(copy.deepcopy(base))
xb = x.to(torch.bfloat16)
fused = run(bf, xb, "1")
eager = run(bf, xb, "0")
for n in ref:
    r = ref[n]
    ef = (fused[n] - r).norm().item() / (r.norm().item() + 1e-9)
    ee = (eager[n] - r).norm().item() / (r.norm().item() + 1e-9)
    print(f"{n:12s} fused-vs-fp32 {ef:.4f}   eager-vs-fp32 {ee:.4f}")
