#!/usr/bin/env python3
"""Config 5 of BASELINE.json: BERT-Large bf16 pre-training (MLM + NSP, seq 128)
with fp16 gradient compression + Adasum through mivod.torch.DistributedOptimizer.

    python benchmarks/bench_bert.py --steps 20 --warmup 5
    python benchmarks/bench_bert.py --gpus 8          # spawns its own 8 ranks
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        benchmarks/bench_bert.py --gpus 8
Prints one JSON line (sequences/sec for the whole job) with a ``comm`` record.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# GEMM selection: PyTorch TunableOp replays a table of the fastest hipBLASLt / rocBLAS
# solution per BERT-Large GEMM shape, tuned once on MI355X and shipped in .tunableop/
# (scripts/gpu_bert_sweep.sh / gpu_bert_bs512.sh regenerate them), one per per-GPU batch.
# TunableOp reads the table under a device-ordinal-suffixed name, so the shipped table is
# staged into a private directory under both the plain and every ordinal-suffixed name.


def _stage_tunableop(batch: int, seq: int) -> None:
    src = os.path.join(ROOT, ".tunableop", f"bert_large_bs{batch}_seq{seq}.csv")
    if not os.path.exists(src) or "PYTORCH_TUNABLEOP_ENABLED" in os.environ:
        return
    import shutil

    import torch
    from mivod.utils.privdir import private_tmp
    d = private_tmp("tunableop")            # 0700, owner-checked
    base = os.path.join(d, f"bert_large_bs{batch}_seq{seq}")
    ndev = max(1, torch.cuda.device_count())
    for name in [base + ".csv"] + [f"{base}{i}.csv" for i in range(ndev)]:
        part = f"{name}.{os.getpid()}.part"
        shutil.copyfile(src, part)
        os.replace(part, name)      # atomic: the ranks of one node share the directory
    os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "1"
    os.environ.setdefault("PYTORCH_TUNABLEOP_TUNING", "0")
    os.environ.setdefault("PYTORCH_TUNABLEOP_FILENAME", base + ".csv")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    # 512 sequences per GPU (64k tokens): bs64 2020 -> bs128 2393 -> bs256 2672 seq/s
    # (1x MI355X, untuned GEMMs); bs256 2733 vs bs512 2962 untuned / 3048 tuned (one box)
    ap.add_argument("--batch", type=int, default=512, help="per-GPU sequences")
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--model", default="large", choices=["large", "base", "tiny"])
    ap.add_argument("--compression", default="fp16", choices=["none", "fp16", "bf16"])
    ap.add_argument("--op", default="adasum", choices=["adasum", "average"])
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--gpus", type=int, default=1)
    args = ap.parse_args()
    if args.gpus > 1 and not any(k in os.environ for k in ("WORLD_SIZE", "HOROVOD_RANK")):
        sys.path.insert(0, ROOT)
        import importlib.util
        spec = importlib.util.spec_from_file_location("mivod_bench", os.path.join(ROOT, "bench.py"))
        mb = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mb)
        sys.exit(mb.self_launch(sys.argv[1:], args.gpus, script=os.path.abspath(__file__)))
    if args.model == "large":
        _stage_tunableop(args.batch, args.seq)

    import torch

    from mivod.utils import benchutil as BU
    BU.multi_rank_defaults()        # multi-rank: a stuck collective ends the job with a diagnosis

    import mivod.torch as hvd
    from mivod.models.bert import BertConfig, BertForPreTraining, synthetic_batch
    from mivod.optim import FusedAdam
    from mivod.common import basics
    from mivod.parallel import collectives as C

    hvd.init()
    rank, size, dev = hvd.rank(), hvd.size(), hvd.device()
    cfg = getattr(BertConfig, args.model)()
    torch.manual_seed(7)
    model = BertForPreTraining(cfg).to(dev).to(torch.bfloat16)
    opt = FusedAdam(model.parameters(), lr=args.lr, weight_decay=0.01, adamw=True)
    op = hvd.Adasum if args.op == "adasum" else hvd.Average
    opt = hvd.DistributedOptimizer(opt, named_parameters=model.named_parameters(),
                                   compression=hvd.Compression.by_name(args.compression), op=op)
    hvd.broadcast_parameters(model.state_dict(), 0)
    hvd.broadcast_optimizer_state(opt, 0)
    g = torch.Generator(device=dev)
    g.manual_seed(100 + rank)
    batch = synthetic_batch(cfg, args.batch, args.seq, dev, generator=g)

    comm_stream = hvd.comm_stream()
    timing = []

    def step(timed=False):
        loss = model(*batch)
        loss.backward()
        if timed:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        opt.step()
        if timed:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(comm_stream)
            timing.append((e0, e1))
        opt.zero_grad(set_to_none=True)
        return loss

    t0 = time.perf_counter()
    for i in range(args.warmup):
        loss = step()
        if rank == 0 and i == 0:
            torch.cuda.synchronize()
            print(f"[bert] first step {time.perf_counter() - t0:.1f}s", file=sys.stderr,
                  flush=True)
    torch.cuda.synchronize()
    timed_comm = getattr(opt, "_mvd_comm", False)
    if timed_comm:
        opt.time_comm(True)          # timing events around every bucket collective
    stats0 = C.gpu_stats()
    C.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step(timed=True)
    torch.cuda.synchronize()
    C.barrier()
    el = C.max_over_ranks(time.perf_counter() - t0)
    stats1 = C.gpu_stats()
    plan = opt.bucket_plan()
    exposed = [max(0.0, a.elapsed_time(b)) for a, b in timing]
    comm = {"buckets": len(plan), "grad_bytes_per_step": sum(nb for _, nb, _ in plan),
            "collectives_per_step": round((stats1.get("calls", 0) - stats0.get("calls", 0))
                                          / max(args.steps, 1), 2),
            "exposed_comm_ms": round(sum(exposed) / len(exposed), 3) if exposed else None,
            "guard": opt.guard_stats(),
            **BU.comm_timing_record(opt.comm_timings() if timed_comm else [], args.steps, size),
            "rccl": BU.rccl_info()}
    if rank == 0:
        print(json.dumps({
            "metric": "sequences/sec (whole node), BERT-Large bf16 pre-training, fp16 compression + Adasum",
            "value": round(args.batch * size * args.steps / el, 2), "unit": "sequences/sec",
            "n_gpus": size, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1000, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (random token ids, 15% masked positions; random-init weights)",
            "loss": round(float(loss.detach()), 4),
            "config": {"model": f"BERT-{args.model}", "global_batch": args.batch * size,
                       "seq_len": args.seq, "parallelism": f"dp{size}",
                       "compression": args.compression, "op": args.op,
                       "optimizer": "mivod FusedAdamW",
                       "transport": basics.state().backend if size > 1 else "local"},
            "comm": comm}), flush=True)
    hvd.shutdown()


if __name__ == "__main__":
    main()
