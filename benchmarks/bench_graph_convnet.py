#!/usr/bin/env python3
"""Eager vs HIP-graph training step on the reference's MNIST ConvNet (launch-bound).

The reference model (/root/reference/mnist_keras.py:71-81): Conv(32,3x3,relu) ->
Conv(64,3x3,relu) -> MaxPool 2x2 -> Dropout .25 -> Flatten -> Dense 128 relu ->
Dropout .5 -> Dense 10, batch 128, Adadelta (lr 1.0 x size).  Written here in
plain torch.nn on the GPU (bf16 activations, fp32 master weights in mivod's
FusedAdadelta via DistributedOptimizer).  A step is ~20 tiny kernels, so eager
execution is bound by launch latency and Python; make_graphed_step replays the
whole step as one graph.  Prints one JSON line with both timings.

    python benchmarks/bench_graph_convnet.py --steps 200
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args()
    import torch
    import torch.nn as nn
    import torch.nn.functional as F

    import mivod.torch as hvd
    from mivod.optim import FusedAdadelta

    hvd.init()
    dev = hvd.device()

    def build():
        torch.manual_seed(0)
        return nn.Sequential(nn.Conv2d(1, 32, 3), nn.ReLU(), nn.Conv2d(32, 64, 3), nn.ReLU(),
                             nn.MaxPool2d(2), nn.Dropout(0.25), nn.Flatten(),
                             nn.Linear(9216, 128), nn.ReLU(), nn.Dropout(0.5),
                             nn.Linear(128, 10)).to(dev).to(torch.bfloat16)

    x = torch.rand(a.batch, 1, 28, 28, device=dev).to(torch.bfloat16)
    y = torch.randint(0, 10, (a.batch,), device=dev)
    res = {}
    for mode in ("eager", "graph"):
        m = build()
        opt = hvd.DistributedOptimizer(FusedAdadelta(m.parameters(), lr=1.0 * hvd.size()),
                                       named_parameters=m.named_parameters())

        def step():
            loss = F.cross_entropy(m(x).float(), y)
            loss.backward()
            opt.step()
            opt.zero_grad(set_to_none=True)
            return loss.detach()

        if mode == "graph":
            step = hvd.make_graphed_step(step, opt, warmup=a.warmup)
        else:
            for _ in range(a.warmup):
                step()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.steps):
            loss = step()
        torch.cuda.synchronize()
        res[mode] = (time.perf_counter() - t) / a.steps * 1e3
        res[mode + "_loss"] = float(loss)
    if hvd.rank() == 0:
        print(json.dumps({"model": "reference MNIST ConvNet (1,199,882 params)", "batch": a.batch,
                          "eager_ms_per_step": round(res["eager"], 4),
                          "graph_ms_per_step": round(res["graph"], 4),
                          "speedup": round(res["eager"] / res["graph"], 2),
                          "final_loss": {"eager": res["eager_loss"], "graph": res["graph_loss"]}}))
    hvd.shutdown()


if __name__ == "__main__":
    main()
