"""One-shot driver for PMC passes: the ResNet-50 bs2048 stem maxpool forward (BN + ReLU
prologue) on [2048, 64, 112, 112]."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mivod.ops import kernels as K  # noqa: E402

nat = K.native()
dev = torch.device("cuda")
x = torch.randn(2048, 64, 112, 112, device=dev).to(torch.bfloat16).contiguous(
    memory_format=torch.channels_last)
sc = torch.rand(64, device=dev) + 0.5
bi = torch.randn(64, device=dev) * 0.1
for _ in range(3):
    nat.maxpool_fwd(x, sc, bi, True, 3, 2, 1)
torch.cuda.synchronize()
print("done")
