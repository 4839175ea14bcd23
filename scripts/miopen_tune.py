"""Exhaustively tune MIOpen's conv solvers for every ResNet-50 conv problem at the
bench batch size, so the shipped perf-db (.miopen/db/*.udb.txt) carries tuned
kernel configurations instead of MIOpen's heuristic defaults.

Run on the GPU box with a fresh user-db dir, e.g.
    MIOPEN_USER_DB_PATH=gpurun_out/mio_tune/db MIOPEN_CUSTOM_CACHE_DIR=gpurun_out/mio_tune/cache \
    MIOPEN_FIND_MODE=NORMAL MIOPEN_FIND_ENFORCE=SEARCH python scripts/miopen_tune.py
Problems are tuned one at a time (fwd, bwd-data, bwd-weights via one fwd+bwd),
the 3x3 convs first (they run at ~600 TFLOP/s with default configs), and no new
problem is started after --budget seconds.  A heartbeat line every 30 s keeps
the run visibly alive while MIOpen searches.
"""
import argparse
import os
import sys
import threading
import time

for _d in ("FWD", "BWD", "WRW"):
    os.environ.setdefault(f"MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_{_d}", "0")

import torch
import torch.nn.functional as F


def problems(batch):
    """(cin, cout, k, stride, hw_in) for every distinct conv in ResNet-50."""
    out = [(3, 64, 7, 2, 224)]
    inplanes = 64
    hw = 56
    for planes, blocks, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
        for b in range(blocks):
            s = stride if b == 0 else 1
            out.append((inplanes, planes, 1, 1, hw))
            out.append((planes, planes, 3, s, hw))
            hw_o = hw // s
            out.append((planes, planes * 4, 1, 1, hw_o))
            if b == 0:
                out.append((inplanes, planes * 4, 1, s, hw))
            inplanes = planes * 4
            hw = hw_o
    seen, uniq = set(), []
    for p in out:
        if p not in seen:
            seen.add(p)
            uniq.append(p)
    # 3x3 first, then the stem, then the 1x1s
    return sorted(uniq, key=lambda p: (0 if p[2] == 3 else 1 if p[2] == 7 else 2))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--budget", type=float, default=900.0)
    ap.add_argument("--only", default="", help="comma list of kernel sizes to tune, e.g. 3,7")
    args = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda")
    t0 = time.time()
    state = {"cur": "init"}
    stop = threading.Event()

    def beat():
        while not stop.wait(30):
            print(f"[tune] {time.time() - t0:7.0f}s still on {state['cur']}", flush=True)

    threading.Thread(target=beat, daemon=True).start()
    only = {int(k) for k in args.only.split(",") if k}
    for cin, cout, k, s, hw in problems(args.batch):
        if only and k not in only:
            continue
        if time.time() - t0 > args.budget:
            print(f"[tune] budget reached; skipping {cin}->{cout} k{k} s{s} hw{hw}", flush=True)
            continue
        state["cur"] = f"{cin}->{cout} k{k} s{s} hw{hw}"
        x = torch.randn(args.batch, cin, hw, hw, device=dev, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last).requires_grad_(k != 7)
        w = (torch.randn(cout, cin, k, k, device=dev) * 0.05).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last).requires_grad_()
        ts = time.time()
        y = F.conv2d(x, w, stride=s, padding=k // 2)
        y.backward(torch.randn_like(y))
        torch.cuda.synchronize()
        print(f"[tune] {state['cur']}: {time.time() - ts:.1f}s (total {time.time() - t0:.0f}s)",
              flush=True)
        del x, w, y
    stop.set()
    print("[tune] done", flush=True)


if __name__ == "__main__":
    sys.exit(main())
