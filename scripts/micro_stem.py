"""Microbenchmark: ResNet-50 stem conv (7x7/2, 64 out, NHWC bf16) fwd + wgrad with
the image padded to Cin = 3 / 4 / 8 channels (zero channels leave the output
unchanged) — MIOpen's kernels for Cin=3 run at ~170 TFLOP/s on gfx950."""
import os
import time

import torch
import torch.nn.functional as F

os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
torch.backends.cudnn.benchmark = True
dev = torch.device("cuda")
N = int(os.environ.get("BS", 512))


def bench(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


for cin in (3, 4, 8):
    x = torch.rand(N, cin, 224, 224, device=dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(64, cin, 7, 7, device=dev) * 0.05).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_()
    gy = torch.randn(N, 64, 112, 112, device=dev, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)

    def fwd():
        return F.conv2d(x, w, stride=2, padding=3)

    def fwdbwd():
        y = F.conv2d(x, w, stride=2, padding=3)
        y.backward(gy)

    a = bench(fwd)
    b = bench(fwdbwd)
    print(f"cin={cin}: fwd {a:8.1f} us  fwd+wgrad {b:8.1f} us", flush=True)
