"""Python call sites that make real copies (.contiguous / .to / clone) of >1 MB tensors in a
ResNet-50 training step (instrumented Tensor methods)."""
import collections
import sys
import traceback
import torch
import torch.nn.functional as F
sys.path.insert(0, ".")
from mivod.models.resnet import resnet50, to_mixed_bf16
from mivod.optim import FusedSGD
import mivod.torch as hvd

hvd.init()
dev = hvd.device()
m = to_mixed_bf16(resnet50()).to(dev)
opt = hvd.DistributedOptimizer(FusedSGD(m.parameters(), lr=0.1, momentum=0.9), named_parameters=m.named_parameters())
x = torch.rand(64, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (64,), device=dev)
hits = collections.Counter()
orig_contig = torch.Tensor.contiguous


def contig(self, *a, **k):
    mf = k.get("memory_format", a[0] if a else torch.contiguous_format)
    if self.numel() * self.element_size() > (1 << 20) and not self.is_contiguous(memory_format=mf):
        fr = [f for f in traceback.extract_stack()[:-1] if "repo" in f.filename][-3:]
        hits["contiguous " + " <- ".join(f"{f.filename.split('/')[-1]}:{f.lineno}" for f in fr)] += 1
    return orig_contig(self, *a, **k)


def step():
    opt.zero_grad(set_to_none=True)
    F.cross_entropy(m(x).float(), y).backward()
    opt.step()


for _ in range(2):
    step()
torch.Tensor.contiguous = contig
step()
torch.cuda.synchronize()
for k, v in hits.most_common(30):
    print(v, k)
