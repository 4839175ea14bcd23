"""Microbenchmark: the 256x256 glds-pipelined NT GEMM (mv_gemm256.hip) on the
compute-bound ResNet-50 bs2048 1x1-conv shapes vs CK (F.conv2d), hipBLASLt (torch.mm)
and gemm_nt's routing (MIVOD_GEMM256=0 selects the older 128-tile kernel), random data."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402,F401  (MIOpen db staging)
from mivod.ops import kernels as K  # noqa: E402

torch.backends.cudnn.benchmark = True
nat = K.native()
dev = torch.device("cuda")
BS = int(os.environ.get("BS", 2048))
# (H, Cin, Cout, launches per step)
SH = [(28, 512, 256, 1), (14, 1024, 256, 6), (14, 256, 1024, 6), (14, 1024, 512, 1),
      (7, 2048, 512, 3), (7, 512, 2048, 3), (14, 1024, 2048, 1), (28, 512, 1024, 1)]


def timed(fn, iters=20):
    for _ in range(3):
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
    x = (torch.rand(BS, cin, hw, hw, device=dev) * 2 - 1).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = ((torch.rand(cout, cin, 1, 1, device=dev) * 2 - 1) / cin ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    a2 = x.permute(0, 2, 3, 1).reshape(M, cin)
    w2 = w.reshape(cout, cin)
    y = torch.empty(M, cout, device=dev, dtype=torch.bfloat16)
    y2 = torch.empty_like(y)
    t_ck = timed(lambda: F.conv2d(x, w))
    t_bl = timed(lambda: torch.mm(a2, w2.t()))
    t_nt = timed(lambda: nat.gemm_nt(a2, w2, y, None, None))
    t_256 = timed(lambda: nat.gemm256_nt(a2, w2, y2))
    ref = torch.mm(a2[:65536].float(), w2.float().t())
    e256 = ((y2[:65536].float() - ref).abs().max() / ref.abs().max()).item()
    ent = ((y[:65536].float() - ref).abs().max() / ref.abs().max()).item()
    tail = ((y2[-300:].float() - torch.mm(a2[-300:].float(), w2.float().t())).abs().max()).item()
    fl = 2 * M * cin * cout
    for i, t in enumerate((t_ck, t_bl, t_nt, t_256)):
        tot[i] += t * cnt
    print(f"M={M:8d} K={cin:4d} N={cout:4d} x{cnt}: CK {t_ck:7.1f} us ({fl / t_ck / 1e6:6.1f} TF) | "
          f"hipBLASLt {t_bl:7.1f} ({fl / t_bl / 1e6:6.1f}) | gemm_nt {t_nt:7.1f} ({fl / t_nt / 1e6:6.1f}) | "
          f"gemm256 {t_256:7.1f} ({fl / t_256 / 1e6:6.1f}) | err nt {ent:.1e} 256 {e256:.1e} tail {tail:.2e}",
          flush=True)
    del x, y, y2, a2, ref
    torch.cuda.empty_cache()
print(f"per step: CK {tot[0] / 1e3:.2f} ms, hipBLASLt {tot[1] / 1e3:.2f}, gemm_nt {tot[2] / 1e3:.2f}, "
      f"gemm256 {tot[3] / 1e3:.2f}")
for n in (4096, 8192):
    a = (torch.rand(n, n, device=dev) * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(n, n, device=dev) * 2 - 1).to(torch.bfloat16)
    c = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
    t1 = timed(lambda: nat.gemm256_nt(a, b, c))
    t2 = timed(lambda: torch.mm(a, b.t()))
    print(f"{n}^3: gemm256 {2 * n ** 3 / t1 / 1e6:6.1f} TF, hipBLASLt {2 * n ** 3 / t2 / 1e6:6.1f} TF")
