"""Stride-2 3x3 data gradient, ResNet-50 bs2048 shapes: MIOpen's backward-data solver vs
mivod's parity-class gather GEMMs (mv_gemm256.hip AMODE 4), plain and with the producing
BN+ReLU's backward reduce fused.

    python scripts/micro_dgrad_s2.py [--batch 2048]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def bench(fn, reps=10):
    import torch
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    a = ap.parse_args()
    import torch
    from mivod.ops import kernels as K
    nat = K.native()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda")
    cl = torch.channels_last
    for c, h in ((128, 56), (256, 28), (512, 14)):
        n = a.batch
        dy = torch.randn(n, c, h // 2, h // 2, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        w = (torch.randn(c, c, 3, 3, device=dev) / (9 * c) ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
        x = torch.randn(n, c, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        wt = w.transpose(0, 1).flip(2, 3).contiguous(memory_format=cl)
        vec = torch.randn(4, c, device=dev)
        flop = 2.0 * n * (h // 2) ** 2 * c * c * 9

        def miopen():
            torch.ops.aten.convolution_backward(dy, x, w, None, [2, 2], [1, 1], [1, 1], False,
                                                [0, 0], 1, [True, False, False])
        t0 = bench(miopen)
        line = f"H {h:3d} {c:4d} ch s2 dgrad: miopen {t0:8.1f} us ({flop / t0 / 1e6:6.1f} TF/s)"
        if nat.conv3x3_s2_dgrad(dy, wt, h, h):
            t1 = bench(lambda: nat.conv3x3_s2_dgrad(dy, wt, h, h))
            t2 = bench(lambda: nat.conv3x3_s2_dgrad(dy, wt, h, h, x, vec))
            ref = torch.ops.aten.convolution_backward(dy, x, w, None, [2, 2], [1, 1], [1, 1],
                                                      False, [0, 0], 1, [True, False, False])[0]
            got = nat.conv3x3_s2_dgrad(dy, wt, h, h)[0]
            err = float((got.float() - ref.float()).abs().max() / ref.float().abs().max())
            line += (f" | mivod {t1:8.1f} us ({flop / t1 / 1e6:6.1f} TF/s) | +BN reduce "
                     f"{t2:8.1f} us | rel err {err:.1e}")
        else:
            line += " | mivod: not covered"
        print(line, flush=True)


if __name__ == "__main__":
    main()
