"""One-shot driver for PMC passes: the hot 256x256-pipeline kernels of a ResNet-50 bs2048
step, a few launches each (layer3 conv3 1x1 forward with statistics, layer3 3x3 forward,
layer3 3x3 weight gradient, layer3 1x1 weight gradient)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mivod.ops import kernels as K  # noqa: E402

nat = K.native()
dev = torch.device("cuda")
cl = torch.channels_last
M = 2048 * 14 * 14
a = torch.randn(M, 256, device=dev).to(torch.bfloat16)
b = torch.randn(1024, 256, device=dev).to(torch.bfloat16) / 16
c = torch.empty(M, 1024, device=dev, dtype=torch.bfloat16)
part = torch.empty(nat.gemm_partials(M, 1024, 256), 2, 1024, device=dev)
shift = torch.zeros(1024, device=dev)
x = torch.randn(2048, 256, 14, 14, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
w = (torch.randn(256, 256, 3, 3, device=dev) / 48).to(torch.bfloat16).contiguous(memory_format=cl)
p3 = torch.empty(nat.conv3x3_partials(M, 256), 2, 256, device=dev)
dy = torch.randn(2048, 256, 14, 14, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
x4 = torch.randn(2048, 1024, 14, 14, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
for _ in range(3):
    nat.gemm_nt(a, b, c, shift, part)                 # gemm256_kernel<1, 0, *>
    nat.conv3x3(x, w, 1, shift[:256].contiguous(), p3)  # gemm256_kernel<1, 3, *>
    nat.wgrad3x3(x, dy, 1)                            # wgrad256_kernel<9>
    nat.wgrad1x1(x4, dy, 1)                           # wgrad256_kernel<1> (C 1024, K 256)
torch.cuda.synchronize()
print("done")
