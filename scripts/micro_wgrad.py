"""Microbenchmark: MIOpen weight-gradient kernels of ResNet-50 bs2048 convs —
time per conv, achieved bytes/s (x + dy read once) and FLOP/s, vs. roofline."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402,F401  (stages the shipped MIOpen find-db / kernel cache like the bench)
torch.backends.cudnn.benchmark = True
dev = torch.device("cuda")
BS = int(os.environ.get("BS", 2048))
# (H_in, cin, cout, k, stride, count per step)
ONLY3 = os.environ.get("ONLY3x3", "0") == "1"
SH = [(56, 256, 64, 1, 1, 2), (56, 64, 64, 1, 1, 1), (56, 64, 64, 3, 1, 3), (56, 64, 256, 1, 1, 4),
      (56, 256, 128, 1, 1, 1), (56, 128, 128, 3, 2, 1), (28, 128, 128, 3, 1, 3),
      (28, 128, 512, 1, 1, 4), (56, 256, 512, 1, 2, 1), (28, 512, 128, 1, 1, 3),
      (28, 512, 256, 1, 1, 1), (28, 256, 256, 3, 2, 1), (14, 256, 256, 3, 1, 5),
      (14, 256, 1024, 1, 1, 6), (28, 512, 1024, 1, 2, 1), (14, 1024, 256, 1, 1, 5),
      (14, 1024, 512, 1, 1, 1), (14, 512, 512, 3, 2, 1), (7, 512, 512, 3, 1, 2),
      (7, 512, 2048, 1, 1, 3), (14, 1024, 2048, 1, 2, 1), (7, 2048, 512, 1, 1, 2)]


def bench(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1000.0


tot, tot_roof = 0.0, 0.0
for h, cin, cout, k, s, cnt in SH:
    if ONLY3 and k != 3:
        continue
    x = torch.randn(BS, cin, h, h, device=dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, k, k, device=dev) / (cin * k * k) ** 0.5).to(
        torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ho = (h + 2 * (k // 2) - k) // s + 1
    dy = torch.randn(BS, cout, ho, ho, device=dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    fn = lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [k // 2] * 2, [1, 1],
                                                     False, [0, 0], 1, [False, True, False])
    t = bench(fn)
    byts = (x.numel() + dy.numel()) * 2
    fl = 2 * dy.numel() * cin * k * k
    roof = max(byts / 6.0e12, fl / 1.6e15) * 1e6
    tot += t * cnt
    tot_roof += roof * cnt
    print(f"wgrad H{h:3d} {cin:4d}->{cout:4d} k{k} s{s} x{cnt}: {t:8.1f} us  {byts / t / 1e6:5.2f} TB/s "
          f"{fl / t / 1e9:7.1f} TF/s  roofline {roof:7.1f} us ({roof / t * 100:4.0f}%)", flush=True)
    del x, dy, w
    torch.cuda.empty_cache()
print(f"wgrad per step: {tot / 1e3:.2f} ms, roofline {tot_roof / 1e3:.2f} ms")
