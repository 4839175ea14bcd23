"""Microbenchmark: ResNet-50 1x1 convs (bs256, NHWC bf16) — MIOpen conv2d vs a
GEMM formulation via torch.matmul (hipBLASLt), fwd and bwd (dX, dW)."""
import os
import time

import torch
import torch.nn.functional as F

os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
torch.backends.cudnn.benchmark = True
dev = torch.device("cuda")
N = int(os.environ.get("BS", 256))
shapes = [(56, 64, 256), (56, 256, 64), (56, 256, 128), (28, 128, 512), (28, 512, 128),
          (14, 256, 1024), (14, 1024, 256), (7, 512, 2048), (7, 2048, 512)]


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


tot = [0.0, 0.0]
for hw, cin, cout in shapes:
    x = torch.randn(N, cin, hw, hw, device=dev, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_()
    w = (torch.randn(cout, cin, 1, 1, device=dev, dtype=torch.bfloat16) * 0.05).contiguous(
        memory_format=torch.channels_last).requires_grad_()
    gy = torch.randn(N, cout, hw, hw, device=dev, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)

    def conv():
        y = F.conv2d(x, w)
        y.backward(gy)

    M = N * hw * hw
    x2 = x.detach().permute(0, 2, 3, 1).reshape(M, cin).requires_grad_()
    w2 = w.detach().reshape(cout, cin).requires_grad_()
    gy2 = gy.permute(0, 2, 3, 1).reshape(M, cout)

    def mm():
        y = torch.matmul(x2, w2.t())
        y.backward(gy2)

    a, b = bench(conv), bench(mm)
    tot[0] += a
    tot[1] += b
    byt = (M * cin + M * cout) * 2 * 3   # fwd x,y + bwd (gy,x ->dw ; gy,w->dx) approx
    print(f"hw={hw:3d} {cin:5d}->{cout:5d}  miopen {a:8.1f} us  matmul {b:8.1f} us  "
          f"(~{byt / a / 1e6:.2f} / {byt / b / 1e6:.2f} TB/s eff)", flush=True)
print(f"total fwd+bwd: miopen {tot[0]:.0f} us, matmul {tot[1]:.0f} us")
