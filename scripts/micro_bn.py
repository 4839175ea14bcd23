"""Microbenchmark of the fused NHWC BatchNorm kernels (mv_bn.hip) on ResNet-50 bs512
shapes.  Run under ``rocprofv3 --kernel-trace`` and summarise with
``--parse <kernel_trace.csv>``: shapes are separated by idle gaps, and each
kernel's achieved HBM bandwidth is computed from the bytes it must move."""
import argparse
import collections
import csv
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(6422528, 64), (1605632, 64), (1605632, 256), (401408, 128), (401408, 512),
          (100352, 256), (100352, 1024), (25088, 512), (25088, 2048)]
# bytes per element each kernel must move (bf16 = 2 B)
BYTES = {"stats_kernel": 2, "apply_kernelILb1ELb0": 4, "apply_kernelILb1ELb1": 6,
         "apply_kernelILb0ELb0": 4, "bwd_reduce_kernelILi1": 4, "bwd_reduce_kernelILi2": 10,
         "bwd_reduce_kernelILi0": 4, "bwd_reduce_kernelILi3": 8.125,
         "bwd_dx_kernelILi1": 6, "bwd_dx_kernelILi0": 6}


def run(reps):
    import torch
    from mivod.ops import kernels as K
    nat = K.native()
    dev = torch.device("cuda")
    for M, C in SHAPES:
        def t(*s):
            return torch.randn(*s, device=dev)
        x = t(M, C).to(torch.bfloat16).view(1, M, 1, C).permute(0, 3, 1, 2)   # NHWC [1,C,M,1]
        res = t(M, C).to(torch.bfloat16).view(1, M, 1, C).permute(0, 3, 1, 2)
        dy = t(M, C).to(torch.bfloat16).view(1, M, 1, C).permute(0, 3, 1, 2)
        dy2 = t(M, C).to(torch.bfloat16).view(1, M, 1, C).permute(0, 3, 1, 2)
        g, b = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        for _ in range(reps):
            y1, vec = nat.bn_fwd_train(x, g, b, rm, rv, 0.1, 1e-5, True, None)
            y2, vec2 = nat.bn_fwd_train(x, g, b, rm, rv, 0.1, 1e-5, True, res)
            nat.bn_bwd(1, dy, x, None, vec, g, True, None, 1)
            nat.bn_bwd(2, dy, x, y2, vec2, g, True, dy2, 1)
            y3, vec3, mk = nat.bn_fwd_train_mask(x, g, b, rm, rv, 0.1, 1e-5, res)
            nat.bn_bwd(3, dy, x, mk, vec3, g, True, dy2, 1)
        torch.cuda.synchronize()
        time.sleep(0.05)
        del x, res, dy, dy2, y1, y2


def parse(path):
    rows = list(csv.DictReader(open(path)))
    rows = [r for r in rows if "mv2bn" in r["Kernel_Name"] or "mv::bn" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    groups, cur, last = [], [], None
    for r in rows:
        s = int(r["Start_Timestamp"])
        if last is not None and s - last > 20e6:   # 20 ms gap = next shape
            groups.append(cur)
            cur = []
        cur.append(r)
        last = int(r["End_Timestamp"])
    groups.append(cur)
    print("| M | C | kernel | us | GB moved | TB/s |\n|---:|---:|---|---:|---:|---:|")
    for (M, C), grp in zip(SHAPES, groups):
        agg = collections.defaultdict(list)
        for r in grp:
            agg[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for name, ds in agg.items():
            key = next((k for k in BYTES if k in name), None)
            if key is None:
                continue
            ds = sorted(ds)[len(ds) // 4:]      # drop the warm-up quarter
            us = sum(ds) / len(ds) / 1e3
            gb = M * C * BYTES[key] / 1e9
            print(f"| {M} | {C} | {key} | {us:.1f} | {gb:.3f} | {gb / us * 1e3:.2f} |")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--parse", default="")
    ap.add_argument("--reps", type=int, default=8)
    a = ap.parse_args()
    if a.parse:
        parse(a.parse)
    else:
        run(a.reps)
