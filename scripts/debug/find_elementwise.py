"""Where do the stray at::native elementwise kernels of the ResNet-50 step come from?
torch.profiler over 2 bench-shaped steps (bs 256 to keep it quick — same op graph),
grouped by the Python stack of the launching op."""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402,F401  (MIOpen db staging)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import mivod.torch as hvd  # noqa: E402
from mivod.models.resnet import resnet50, to_mixed_bf16  # noqa: E402
from mivod.optim import FusedSGD  # noqa: E402

hvd.init()
dev = hvd.device()
bs = int(os.environ.get("BS", 256))
model = to_mixed_bf16(resnet50()).to(dev)
opt = hvd.DistributedOptimizer(FusedSGD(model.parameters(), lr=0.1, momentum=0.9),
                               named_parameters=model.named_parameters())
x = torch.rand(bs, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(
    memory_format=torch.channels_last)
y = torch.randint(0, 1000, (bs,), device=dev)


def step():
    loss = F.cross_entropy(model(x).float(), y)
    loss.backward()
    opt.step()
    opt.zero_grad(set_to_none=True)


for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
             record_shapes=True) as prof:
    step()
    torch.cuda.synchronize()
rows = collections.Counter()
for ev in prof.events():
    if ev.device_type.name != "CPU" or not ev.name.startswith("aten::"):
        continue
    kern = [k for k in ev.kernels if "elementwise" in k.name or "vectorized" in k.name
            or "reduce_kernel" in k.name or "fill" in k.name.lower()]
    if not kern:
        continue
    stack = [s for s in (ev.stack or []) if "mivod" in s or "bench" in s or "resnet" in s][:3]
    rows[(ev.name, str(ev.input_shapes)[:80], " <- ".join(stack))] += len(kern)
for (name, shp, st), n in rows.most_common(60):
    print(f"{n:3d}  {name:28s} {shp:80s} {st}")
hvd.shutdown()
