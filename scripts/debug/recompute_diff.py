"""Per-parameter gradient differences: recompute on/off and off/off (nondeterminism floor)."""
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
x = torch.rand(8, 3, 64, 64, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
tgt = torch.randint(0, 10, (8,), device=cuda)


def run(rc):
    B._RECOMPUTE = rc
    m = copy.deepcopy(base)
    lg = m(x)
    F.cross_entropy(lg.float(), tgt).backward()
    return lg.float(), {k: p.grad.float() for k, p in m.named_parameters()}


run(False)
outs = [("off", run(False)), ("off2", run(False)), ("on", run(True)), ("on2", run(True))]
ref = outs[0][1]
for name, o in outs[1:]:
    print(name, "logits maxdiff", float((o[0] - ref[0]).abs().max()))
    bad = []
    for k, r in ref[1].items():
        e = float((o[1][k] - r).norm()) / (float(r.norm()) + 1e-12)
        if e > 1e-3:
            bad.append((k, round(e, 4)))
    print(name, "params with rel err > 1e-3:", len(bad), bad[:12])
