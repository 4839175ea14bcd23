"""Which PyTorch ops launch the non-mivod kernels of a ResNet-50 training step.

    python scripts/debug/find_stray_kernels.py [--batch 256]

Runs a few bench-shaped steps (model, fused SGD via DistributedOptimizer) under
torch.profiler with shapes recorded and prints, for every device kernel whose name
matches --pattern (default: PyTorch elementwise / copy / fill / flip kernels and
MIOpen's tensor ops), the CPU op chain that launched it and the op's input shapes.
"""
import argparse
import collections
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--pattern", default=r"elementwise|flip|copyBuffer|fillBuffer|SubTensorOp|"
                                         r"Cijk|igemm|grouped_conv|reduce_kernel")
    a = ap.parse_args()
    import torch
    import torch.nn.functional as F
    import mivod.torch as hvd
    from mivod.models.resnet import resnet50, to_mixed_bf16
    from mivod.optim import FusedSGD

    hvd.init()
    dev = hvd.device()
    torch.manual_seed(0)
    model = to_mixed_bf16(resnet50()).to(dev)
    opt = hvd.DistributedOptimizer(FusedSGD(model.parameters(), lr=0.1, momentum=0.9,
                                            weight_decay=5e-5),
                                   named_parameters=model.named_parameters())
    x = torch.rand(a.batch, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (a.batch,), device=dev)

    def step():
        loss = F.cross_entropy(model(x).float(), y)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    pat = re.compile(a.pattern)
    agg = collections.Counter()
    dur = collections.defaultdict(float)
    for ev in prof.events():
        for k in getattr(ev, "kernels", []) or []:
            if not pat.search(k.name):
                continue
            chain = []
            p = ev
            while p is not None and len(chain) < 6:
                chain.append(p.name)
                p = p.cpu_parent
            key = (k.name[:70], " <- ".join(chain), str(ev.input_shapes)[:160])
            agg[key] += 1
            dur[key] += k.duration
    for key, n in sorted(agg.items(), key=lambda kv: -dur[kv[0]]):
        print(f"{dur[key]:9.1f} us  x{n}  {key[0]}\n      {key[1]}\n      shapes {key[2]}")
    hvd.shutdown()


if __name__ == "__main__":
    main()
