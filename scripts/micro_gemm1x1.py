"""Microbenchmark: ResNet-50 bs2048 1x1 conv forwards — MIOpen/CK (F.conv2d) vs
mivod's MFMA NT GEMM (mv_gemm.hip), plain and with the fused BN-statistics
epilogue, plus the separate BN statistics pass the epilogue replaces.
Checks the GEMM against F.conv2d and the fused statistics against torch."""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402,F401  (stages the shipped MIOpen find-db / kernel cache like the bench)
torch.backends.cudnn.benchmark = True
from mivod.ops import kernels as K  # noqa: E402

nat = K.native()
dev = torch.device("cuda")
BS = int(os.environ.get("BS", 2048))
# (H, Cin, Cout, launches per ResNet-50 step)
SH = [(56, 64, 64, 1), (56, 256, 64, 2), (56, 64, 256, 4), (56, 256, 128, 1), (28, 512, 128, 3),
      (28, 128, 512, 4), (28, 512, 256, 1), (14, 1024, 256, 5), (14, 256, 1024, 6),
      (14, 1024, 512, 1), (7, 2048, 512, 2), (7, 512, 2048, 3)]


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


tot = [0.0] * 4
for hw, cin, cout, cnt in SH:
    M = BS * hw * hw
    x = (torch.randn(BS, cin, hw, hw, device=dev) * 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, 1, 1, device=dev) / cin ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    a2 = x.permute(0, 2, 3, 1).reshape(M, cin)
    w2 = w.reshape(cout, cin)
    y = torch.empty(M, cout, device=dev, dtype=torch.bfloat16)
    P = nat.gemm_partials(M, cout, cin)
    part = torch.empty(P, 2, cout, device=dev)
    shift = torch.zeros(cout, device=dev)
    t_conv = bench(lambda: F.conv2d(x, w))
    t_gemm = bench(lambda: nat.gemm_nt(a2, w2, y, None, None))
    t_gst = bench(lambda: nat.gemm_nt(a2, w2, y, shift, part))
    ref = F.conv2d(x, w).permute(0, 2, 3, 1).reshape(M, cout)
    rm = torch.zeros(cout, device=dev)
    rv = torch.ones(cout, device=dev)
    yv = y.view(BS, hw, hw, cout).permute(0, 3, 1, 2)
    t_stats = bench(lambda: nat.bn_stats(yv, None, None, rm, rv, 0.0, 1e-5))
    nat.gemm_nt(a2, w2, y, shift, part)
    torch.cuda.synchronize()
    err = (y.float() - ref.float()).abs().max().item() / ref.float().abs().max().item()
    s = part.sum(0)
    yf = y.float()
    es = ((s[0] - yf.sum(0)).abs().max() / yf.abs().sum(0).max()).item()
    tot[0] += t_conv * cnt
    tot[1] += t_gemm * cnt
    tot[2] += t_gst * cnt
    tot[3] += t_stats * cnt
    gb = (M * cin + M * cout) * 2 / 1e9
    print(f"M={M:8d} K={cin:4d} N={cout:4d} x{cnt}: conv2d {t_conv:8.1f} us | gemm {t_gemm:8.1f} us "
          f"({gb / t_gemm * 1e6 / 1e3:5.2f} TB/s, {2 * M * cin * cout / t_gemm / 1e6:6.1f} TF) | "
          f"gemm+stats {t_gst:8.1f} us | stats pass {t_stats:7.1f} us | rel err {err:.1e} "
          f"stats err {es:.1e}", flush=True)
    del x, y, a2, ref, yf
    torch.cuda.empty_cache()
print(f"per step: conv2d {tot[0] / 1e3:.2f} ms, gemm {tot[1] / 1e3:.2f} ms, gemm+stats "
      f"{tot[2] / 1e3:.2f} ms, stats passes {tot[3] / 1e3:.2f} ms -> fused saving "
      f"{(tot[0] + tot[3] - tot[2]) / 1e3:.2f} ms")

# ---- backward: conv1 data gradient + the previous block's BN(+add+ReLU) backward
# (dgrad K = conv1's Cout, N = its Cin); unfused = MIOpen forward-conv dgrad + the
# 3-kernel mode-3 BN backward; fused = gemm_nt_bn_bwd + finalize/dx from partials
BW = [(56, 64, 256, 2), (28, 128, 512, 3), (14, 256, 1024, 5)]
tb = [0.0, 0.0]
for hw, k, n, cnt in BW:
    M = BS * hw * hw
    dy = (torch.randn(BS, k, hw, hw, device=dev)).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    wt = (torch.randn(n, k, 1, 1, device=dev) / k ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    xb = torch.randn(BS, n, hw, hw, device=dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    res = torch.randn_like(xb)
    dy2 = torch.randn_like(xb)
    gm = torch.ones(n, device=dev)
    bt = torch.zeros(n, device=dev)
    _, vec, mask = nat.bn_fwd_train_mask(xb, gm, bt, torch.zeros(n, device=dev),
                                         torch.ones(n, device=dev), 0.1, 1e-5, res)
    a2 = dy.permute(0, 2, 3, 1).reshape(M, k)
    w2 = wt.reshape(n, k)
    dz = torch.empty_like(xb)
    dz2 = dz.permute(0, 2, 3, 1).reshape(M, n)
    x2 = xb.permute(0, 2, 3, 1).reshape(M, n)

    def unfused():
        g = F.conv2d(dy, wt)
        nat.bn_bwd(3, g, xb, mask, vec, gm, True, dy2, 1)

    def fused():
        p = nat.gemm_nt_bn_bwd(a2, w2, dz2, dy2, mask, x2, vec)
        nat.bn_bwd_from_partials(dz, xb, vec, gm, True, p)

    def fused_gemm(bn=0):
        nat.gemm_nt_bn_bwd(a2, w2, dz2, dy2, mask, x2, vec, bn)

    tu = bench(unfused)
    tf = bench(fused)
    tg = bench(fused_gemm)
    sweep = " ".join(f"bn{b}={bench(lambda: fused_gemm(b)):.0f}" for b in (64, 128, 256)
                     if nat.gemm_bwd_partials(M, n, k, b) > 0)
    tc = bench(lambda: F.conv2d(dy, wt))
    tb[0] += tu * cnt
    tb[1] += tf * cnt
    gb = (M * k + 4 * M * n) * 2 / 1e9
    print(f"bwd M={M:8d} K={k:4d} N={n:4d} x{cnt}: dgrad conv {tc:8.1f} us, dgrad+bn_bwd "
          f"{tu:8.1f} us | fused gemm {tg:8.1f} us ({gb / tg * 1e6 / 1e3:5.2f} TB/s), "
          f"fused total {tf:8.1f} us [{sweep}]", flush=True)
    del dy, xb, res, dy2, dz, mask
    torch.cuda.empty_cache()
print(f"bwd per step: unfused {tb[0] / 1e3:.2f} ms, fused {tb[1] / 1e3:.2f} ms -> saving "
      f"{(tb[0] - tb[1]) / 1e3:.2f} ms")

# ---- forward on the implicit-GEMM conv kernel (ks = 1) for the large-K 1x1 shapes
print("-- conv kernel (ks=1) forward")
for hw, cin, cout, cnt in SH:
    if cin < 512:
        continue
    x = (torch.randn(BS, cin, hw, hw, device=dev) * 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, 1, 1, device=dev) / cin ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    M = BS * hw * hw
    part = torch.empty(nat.conv3x3_partials(M, cout), 2, cout, device=dev)
    t_conv = bench(lambda: F.conv2d(x, w))
    t_mv = bench(lambda: nat.conv1x1(x, w, 1))
    t_st = bench(lambda: nat.conv1x1(x, w, 1, None, part))
    fl = 2 * M * cin * cout
    print(f"1x1 M={M:8d} K={cin:4d} N={cout:4d} x{cnt}: conv2d {t_conv:7.1f} us ({fl / t_conv / 1e6:6.1f} TF/s) | "
          f"mivod {t_mv:7.1f} us ({fl / t_mv / 1e6:6.1f} TF/s) | +stats {t_st:7.1f} us", flush=True)
    del x
    torch.cuda.empty_cache()
