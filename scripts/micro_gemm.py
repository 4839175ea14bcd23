"""Microbenchmark: BERT-Large linear layers (tokens = 8192) — forward (x W^T),
dgrad (dy W) and wgrad (dy^T x) through torch (hipBLASLt by default), with the
achieved TFLOP/s.  BLAS=rocblas switches torch's preferred library; run under
PYTORCH_TUNABLEOP_ENABLED=1 to let TunableOp pick among rocBLAS/hipBLASLt
solutions."""
import os
import time

import torch

dev = torch.device("cuda")
if os.environ.get("BLAS"):
    torch.backends.cuda.preferred_blas_library(os.environ["BLAS"])
T = int(os.environ.get("TOKENS", 8192))
H = 1024
layers = [("qkv", H, 3 * H), ("dense", H, H), ("inter", H, 4 * H), ("output", 4 * H, H)]


def bench(fn, iters=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


tot_us, tot_fl = 0.0, 0.0
for name, k, n in layers:
    x = torch.randn(T, k, device=dev, dtype=torch.bfloat16)
    w = torch.randn(n, k, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(T, n, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * T * k * n
    for kind, fn in (("fwd", lambda: torch.nn.functional.linear(x, w)),
                     ("dgrad", lambda: torch.matmul(dy, w)),
                     ("wgrad", lambda: torch.matmul(dy.t(), x))):
        us = bench(fn)
        tot_us += us
        tot_fl += fl
        print(f"{name:7s} {kind:6s} M={T} N={n} K={k}: {us:8.1f} us  {fl / us / 1e6:7.1f} TFLOP/s",
              flush=True)
print(f"TOTAL per layer {tot_us:.1f} us  {tot_fl / tot_us / 1e6:.1f} TFLOP/s; "
      f"x24 layers = {tot_us * 24 / 1e3:.2f} ms", flush=True)
