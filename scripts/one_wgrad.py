"""Run mivod's wgrad3x3 on one ResNet-50 shape a few times (for rocprofv3 --pmc)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mivod.ops import kernels as K  # noqa: E402

nat = K.native()
h, c, k = (int(v) for v in os.environ.get("SHAPE", "14,256,256").split(","))
bs = int(os.environ.get("BS", 2048))
x = torch.randn(bs, c, h, h, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
dy = torch.randn(bs, k, h, h, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
for _ in range(5):
    dw = nat.wgrad3x3(x, dy, 1)
torch.cuda.synchronize()
print("done", dw.shape)
