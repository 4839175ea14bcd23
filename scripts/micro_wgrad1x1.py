"""Microbenchmark: ResNet-50 bs2048 1x1 weight gradients, MIOpen (aten.convolution_backward,
weight only) vs mivod's wgrad1x1 kernel (csrc/kernels/mv_conv.hip), with an fp32 check."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402,F401  (stages the shipped MIOpen find-db like the bench)
from mivod.ops import kernels as K  # noqa: E402

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda")
nat = K.native()
BS = int(os.environ.get("BS", 2048))
# (H_in, cin, cout, stride, count per step)
SH = [(56, 64, 64, 1, 1), (56, 64, 256, 1, 4), (56, 256, 64, 1, 2), (56, 256, 128, 1, 1),
      (28, 128, 512, 1, 4), (56, 256, 512, 2, 1), (28, 512, 128, 1, 3), (28, 512, 256, 1, 1),
      (14, 256, 1024, 1, 6), (28, 512, 1024, 2, 1), (14, 1024, 256, 1, 5), (14, 1024, 512, 1, 1),
      (7, 512, 2048, 1, 3), (14, 1024, 2048, 2, 1), (7, 2048, 512, 1, 2)]


def bench_us(fn, iters=10):
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


tot = [0.0, 0.0]
for h, cin, cout, s, cnt in SH:
    x = torch.randn(BS, cin, h, h, device=dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, 1, 1, device=dev) / cin ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    ho = (h - 1) // s + 1
    dy = torch.randn(BS, cout, ho, ho, device=dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    ref_fn = lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [0, 0], [1, 1],
                                                         False, [0, 0], 1, [False, True, False])
    t_ref = bench_us(ref_fn)
    t_mv = bench_us(lambda: nat.wgrad1x1(x, dy, s))
    if os.environ.get("SWEEP"):
        res = []
        for b in os.environ["SWEEP"].split(","):
            os.environ["MIVOD_WGRAD1_BLOCKS"] = b
            res.append(f"{b}:{bench_us(lambda: nat.wgrad1x1(x, dy, s)):.1f}")
        os.environ.pop("MIVOD_WGRAD1_BLOCKS")
        print("   blocks sweep (us): " + " ".join(res), flush=True)
    ref = ref_fn()[1].float()
    got = nat.wgrad1x1(x, dy, s).float()
    err = float((got - ref).abs().max() / ref.abs().max())
    fl = 2 * dy.numel() * cin
    tot[0] += t_ref * cnt
    tot[1] += t_mv * cnt
    print(f"wgrad1x1 H{h:3d} {cin:4d}->{cout:4d} s{s} x{cnt}: miopen {t_ref:8.1f} us "
          f"({fl / t_ref / 1e6:6.1f} TF/s) | mivod {t_mv:8.1f} us ({fl / t_mv / 1e6:6.1f} TF/s) | "
          f"rel err {err:.1e}", flush=True)
    del x, dy, w
    torch.cuda.empty_cache()
print(f"wgrad1x1 per step: miopen {tot[0] / 1e3:.2f} ms, mivod {tot[1] / 1e3:.2f} ms")
