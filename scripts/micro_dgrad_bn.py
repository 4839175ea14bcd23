"""Microbenchmark: conv2's stride-1 data gradient + BN1 (BN+ReLU) backward, ResNet-50 bs2048:
MIOpen forward-solver dgrad + mode-1 BN backward (reduce, finalize, dx) vs mivod's conv3x3
dgrad with the BN reduce in its epilogue + finalize/dx from the partials."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402,F401
from mivod.ops import kernels as K  # noqa: E402

nat = K.native()
dev = torch.device("cuda")
BS = int(os.environ.get("BS", 2048))


def tm(fn, iters=10):
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


for h, c in ((56, 64), (28, 128), (14, 256), (7, 512)):
    cl = torch.channels_last
    dy = torch.randn(BS, c, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(c, c, 3, 3, device=dev) / (9 * c) ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
    wt = w.transpose(0, 1).flip(2, 3).contiguous(memory_format=cl)
    xb = torch.randn(BS, c, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    gm = torch.ones(c, device=dev)
    _, vec = nat.bn_fwd_train(xb, gm, torch.zeros(c, device=dev), torch.zeros(c, device=dev),
                              torch.ones(c, device=dev), 0.1, 1e-5, True, None)
    t_mi = tm(lambda: F.conv2d(dy, wt, None, 1, 1))
    t_mv = tm(lambda: nat.conv3x3(dy, wt, 1))
    g = F.conv2d(dy, wt, None, 1, 1)
    t_bn = tm(lambda: nat.bn_bwd(1, g, xb, None, vec, gm, True, None, 1))
    t_ep = tm(lambda: nat.conv3x3_bn_bwd(dy, wt, xb, vec))
    d, part = nat.conv3x3_bn_bwd(dy, wt, xb, vec)
    t_fin = tm(lambda: nat.bn_bwd_from_partials(d, xb, vec, gm, True, part))
    print(f"H{h:3d} C{c:4d}: MIOpen dgrad {t_mi:7.1f} + bn_bwd {t_bn:7.1f} = {t_mi + t_bn:7.1f} us | "
          f"mivod dgrad {t_mv:7.1f} | fused dgrad+reduce {t_ep:7.1f} + finalize/dx {t_fin:7.1f} = "
          f"{t_ep + t_fin:7.1f} us", flush=True)
    del dy, xb, g, d
    torch.cuda.empty_cache()

# ---- bottleneck conv3 (1x1, 4c -> c data gradient) + BN2 (BN+ReLU) backward: the unfused
# path (mivod streaming GEMM for 4c = 256, MIOpen's forward solver otherwise) vs the
# implicit-GEMM kernel with ks = 1 and the reduce epilogue
for h, c in ((56, 64), (28, 128), (14, 256), (7, 512)):
    cl = torch.channels_last
    dy = torch.randn(BS, 4 * c, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(4 * c, c, 1, 1, device=dev) / c ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
    wt = w.transpose(0, 1).contiguous(memory_format=cl)
    xb = torch.randn(BS, c, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    gm = torch.ones(c, device=dev)
    _, vec = nat.bn_fwd_train(xb, gm, torch.zeros(c, device=dev), torch.zeros(c, device=dev),
                              torch.ones(c, device=dev), 0.1, 1e-5, True, None)
    t_mi = tm(lambda: F.conv2d(dy, wt))
    g = F.conv2d(dy, wt)
    t_bn = tm(lambda: nat.bn_bwd(1, g, xb, None, vec, gm, True, None, 1))
    t_ep = tm(lambda: nat.conv3x3_bn_bwd(dy, wt, xb, vec))
    d, part = nat.conv3x3_bn_bwd(dy, wt, xb, vec)
    t_fin = tm(lambda: nat.bn_bwd_from_partials(d, xb, vec, gm, True, part))
    print(f"1x1 H{h:3d} {4 * c:4d}->{c:4d}: MIOpen dgrad {t_mi:7.1f} + bn_bwd {t_bn:7.1f} = "
          f"{t_mi + t_bn:7.1f} us | fused dgrad+reduce {t_ep:7.1f} + finalize/dx {t_fin:7.1f} = "
          f"{t_ep + t_fin:7.1f} us", flush=True)
    del dy, xb, g, d
    torch.cuda.empty_cache()
