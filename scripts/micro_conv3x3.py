"""Microbenchmark: ResNet-50 bs2048 3x3 convs — MIOpen/CK (F.conv2d) vs mivod's
implicit-GEMM kernel (csrc/kernels/mv_conv.hip), plain and with fused BN stats."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402,F401  (stages the shipped MIOpen find-db / kernel cache like the bench)
torch.backends.cudnn.benchmark = True
from mivod.ops import kernels as K  # noqa: E402

nat = K.native()
dev = torch.device("cuda")
BS = int(os.environ.get("BS", 2048))
# (H_in, C, K, stride, launches per step (fwd + stride-1 dgrad-as-forward))
SH = [(56, 64, 64, 1, 6), (56, 128, 128, 2, 1), (28, 128, 128, 1, 6), (28, 256, 256, 2, 1),
      (14, 256, 256, 1, 10), (14, 512, 512, 2, 1), (7, 512, 512, 1, 4)]


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


tot = [0.0, 0.0, 0.0]
for h, c, k, s, cnt in SH:
    x = (torch.randn(BS, c, h, h, device=dev) * 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(k, c, 3, 3, device=dev) / (9 * c) ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    ho = (h - 1) // s + 1
    M = BS * ho * ho
    P = nat.conv3x3_partials(M, k)
    part = torch.empty(P, 2, k, device=dev)
    shift = torch.zeros(k, device=dev)
    t_ref = bench(lambda: F.conv2d(x, w, None, s, 1))
    t_mv = bench(lambda: nat.conv3x3(x, w, s))
    t_st = bench(lambda: nat.conv3x3(x, w, s, shift, part))
    ref = F.conv2d(x, w, None, s, 1)
    y = nat.conv3x3(x, w, s)
    err = ((y.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
    fl = 2 * M * k * 9 * c
    tot[0] += t_ref * cnt
    tot[1] += t_mv * cnt
    tot[2] += t_st * cnt
    print(f"H{h:3d} {c:4d}->{k:4d} s{s} x{cnt}: conv2d {t_ref:8.1f} us ({fl / t_ref / 1e6:6.1f} TF/s) | "
          f"mivod {t_mv:8.1f} us ({fl / t_mv / 1e6:6.1f} TF/s) | +stats {t_st:8.1f} us | "
          f"P={P} rel err {err:.1e}", flush=True)
    del x, y, ref
    torch.cuda.empty_cache()
print(f"per step: conv2d {tot[0] / 1e3:.2f} ms, mivod {tot[1] / 1e3:.2f} ms, +stats {tot[2] / 1e3:.2f} ms")

# ---- weight gradient: MIOpen (aten.convolution_backward, weight only) vs mivod wgrad3x3
tw = [0.0, 0.0]
for h, c, k, s, cnt in SH:
    x = (torch.randn(BS, c, h, h, device=dev) * 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(k, c, 3, 3, device=dev) / (9 * c) ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    ho = (h - 1) // s + 1
    dy = torch.randn(BS, k, ho, ho, device=dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    t_ref = bench(lambda: torch.ops.aten.convolution_backward(
        dy, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]))
    t_mv = bench(lambda: nat.wgrad3x3(x, dy, s))
    ref = torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [1, 1], [1, 1], False,
                                              [0, 0], 1, [False, True, False])[1]
    got = nat.wgrad3x3(x, dy, s)
    err = ((got.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
    fl = 2 * BS * ho * ho * k * 9 * c
    n_w = cnt // 2 if s == 1 else cnt     # SH counts fwd + dgrad launches for stride 1
    tw[0] += t_ref * n_w
    tw[1] += t_mv * n_w
    print(f"wgrad H{h:3d} {c:4d}->{k:4d} s{s}: miopen {t_ref:8.1f} us ({fl / t_ref / 1e6:6.1f} TF/s) | "
          f"mivod {t_mv:8.1f} us ({fl / t_mv / 1e6:6.1f} TF/s) | rel err {err:.1e}", flush=True)
    del x, dy
    torch.cuda.empty_cache()
print(f"wgrad per step: miopen {tw[0] / 1e3:.2f} ms, mivod {tw[1] / 1e3:.2f} ms")
