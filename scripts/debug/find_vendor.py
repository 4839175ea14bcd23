"""Which launches of the ResNet-50 step are NOT mivod kernels (CK / MIOpen / hipBLASLt /
at::native), and which op + Python frame issues each?  torch.profiler over one
bench-shaped step (BS env, default 2048), grouped by (aten op, shapes, mivod frame),
summed device time."""
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

torch.backends.cudnn.benchmark = True
hvd.init()
dev = hvd.device()
bs = int(os.environ.get("BS", 2048))
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
rows = collections.defaultdict(lambda: [0, 0.0, ""])
for ev in prof.events():
    if ev.device_type.name != "CPU" or not ev.name.startswith("aten::"):
        continue
    kern = [k for k in ev.kernels if not (k.name.startswith("_ZN2mv") or k.name.startswith("mv::")
                                          or "mv::" in k.name[:40])]
    if not kern:
        continue
    stack = [s for s in (ev.stack or []) if "mivod" in s or "bench" in s][:2]
    key = (ev.name, str(ev.input_shapes)[:110], " <- ".join(stack))
    rows[key][0] += len(kern)
    rows[key][1] += sum(k.duration for k in kern) / 1e3
    rows[key][2] = kern[0].name[:60]
tot = sum(v[1] for v in rows.values())
print(f"non-mivod device time: {tot:.2f} ms/step")
for (name, shp, st), (n, ms, kn) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:45]:
    print(f"{ms:7.3f} ms {n:3d}x  {name:24s} {shp}\n      {kn}\n      {st}")
hvd.shutdown()
