"""ResNet-50 stride-1 1x1 convs at bs1024 (NHWC bf16): the three GEMMs of mivod's
conv path (fwd, dgrad-as-forward-conv, wgrad via MIOpen) vs the same GEMMs on the
NHWC [M, C] views through torch.matmul (hipBLASLt).  Prints us per op."""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402,F401  (MIOpen find-db env)

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda")
N = int(os.environ.get("BS", 1024))
# (hw, cin, cout, count in ResNet-50)
SHAPES = [(56, 64, 64, 1), (56, 256, 64, 2), (56, 64, 256, 4), (28, 256, 128, 1), (28, 512, 128, 3),
          (28, 128, 512, 4), (14, 512, 256, 1), (14, 1024, 256, 5), (14, 256, 1024, 6),
          (7, 1024, 512, 1), (7, 2048, 512, 2), (7, 512, 2048, 3)]


def bench_us(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


tot = {"conv": 0.0, "mm": 0.0}
for hw, cin, cout, cnt in SHAPES:
    M = N * hw * hw
    x = torch.randn(N, cin, hw, hw, device=dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, 1, 1, device=dev) * 0.05).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dy = torch.randn(N, cout, hw, hw, device=dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    wt = w.transpose(0, 1).contiguous(memory_format=torch.channels_last)
    x2 = x.permute(0, 2, 3, 1).reshape(M, cin)
    dy2 = dy.permute(0, 2, 3, 1).reshape(M, cout)
    w2 = w.reshape(cout, cin)
    c = [bench_us(lambda: F.conv2d(x, w)),
         bench_us(lambda: F.conv2d(dy, wt)),
         bench_us(lambda: torch.ops.aten.convolution_backward(
             dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False]))]
    m = [bench_us(lambda: torch.matmul(x2, w2.t())),
         bench_us(lambda: torch.matmul(dy2, w2)),
         bench_us(lambda: torch.matmul(dy2.t(), x2))]
    tot["conv"] += sum(c) * cnt
    tot["mm"] += sum(m) * cnt
    print(f"hw={hw:2d} {cin:4d}->{cout:4d} x{cnt}: conv fwd/dgrad/wgrad "
          f"{c[0]:7.1f} {c[1]:7.1f} {c[2]:7.1f} us | matmul {m[0]:7.1f} {m[1]:7.1f} {m[2]:7.1f} us",
          flush=True)
    del x, w, dy, wt, x2, dy2
print(f"weighted total per step: conv {tot['conv'] / 1e3:.2f} ms, matmul {tot['mm'] / 1e3:.2f} ms")
