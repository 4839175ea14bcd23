"""Probe RCCL PreMulSum / ncclAvg on a 1-rank communicator: which elements of an
odd-length buffer come back unscaled (round-3 finding: the last of 4097)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from mivod.parallel.transport import RcclTransport

dev = torch.device("cuda", 0)
tr = RcclTransport.create(0, 1, dev)
for dt in (torch.float32, torch.bfloat16, torch.float16):
    for n in (1, 7, 8, 9, 63, 64, 65, 1000, 4095, 4096, 4097, 65537, 1 << 20 | 3):
        x = (torch.arange(n, device=dev) % 13 + 1).to(dt)
        ref = x.float() * 0.5
        y = x.clone()
        tr.allreduce_(y, "sum", prescale=0.5)
        torch.cuda.synchronize()
        bad = (y.float() - ref).abs() > 1e-3 * ref.abs().clamp_min(1)
        idx = bad.nonzero().flatten().tolist()
        print(f"premul {str(dt):15s} n={n:8d} wrong={len(idx)} first={idx[:6]}", flush=True)
tr.close()
