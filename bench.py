#!/usr/bin/env python3
"""mivod headline benchmark: ResNet-50 bf16 synthetic-ImageNet training throughput.

BASELINE.json metric: images/sec for the whole node (+ scaling efficiency,
computed by the driver from the per-N values) at 1/2/4/8 MI355X.  Each rank
trains a full ResNet-50 step — forward, backward, gradient allreduce (RCCL over
xGMI through mivod's static bucket schedule on the comm stream) and the fused
SGD-momentum update — on a fixed per-GPU batch (weak scaling).

    python bench.py --gpus 1 --steps 30 --warmup 10
    python bench.py --gpus 8                      # spawns its own 8 ranks
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 8

``--gpus N`` without a launcher environment (no WORLD_SIZE / HOROVOD_RANK):
bench.py starts N rank processes itself through mivod's launcher
(``mivod.run.launcher.launch``, the horovodrun path) BEFORE touching the GPU,
one per GPU, and exits with their status.  Fewer than N visible GPUs is an
error unless ``MIVOD_BENCH_SHARE_GPUS=1`` (test rehearsal: ranks share GPUs
over ``MIVOD_TRANSPORT=gloo-gpu``, since RCCL refuses two ranks on one GPU).

Data: synthetic, generated on the GPU once (uniform images, random labels);
weights: random init.  Rank 0 prints ONE JSON line, with a ``comm`` record:
gradient buckets, bytes per step, collectives per step, the exposed
communication time (comm-stream work still running after backward's last
kernel was enqueued, per step), the MEASURED allreduce time per step with
per-bucket algorithm / bus bandwidth (timing events around every bucket
collective on the comm stream), and what RCCL itself sees (run-time and header
version, ncclCommCount, CTA range).  Multi-rank runs default the RCCL watchdog
and stall-shutdown timeouts (mivod.utils.benchutil) so a hang exits non-zero
with the stuck collective's name.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
# MIOpen's naive direct-conv fallbacks are never competitive on gfx950, and their
# kernels are not kept in the kernel cache, which invalidates every find-db record
# that lists them: Find then re-runs on each fresh process (~115 s at bs512,
# benchmarking 50-150 ms naive kernels).  Keep them out of the search.
for _d in ("FWD", "BWD", "WRW"):
    os.environ.setdefault(f"MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_{_d}", "0")
# Ship MIOpen's find-db + compiled-kernel cache with the repo (.miopen/): a fresh
# MI355X box otherwise spends ~3 minutes JIT-compiling ResNet-50's conv kernels.
_MIO = os.path.join(os.path.dirname(os.path.abspath(__file__)), ".miopen")
if os.path.isdir(_MIO) and "MIOPEN_USER_DB_PATH" not in os.environ:
    import shutil
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from mivod.utils.privdir import private_tmp
    _tmp = private_tmp("miopen")            # 0700, owner-checked (not a shared /tmp path)
    for sub, var in (("db", "MIOPEN_USER_DB_PATH"), ("cache", "MIOPEN_CUSTOM_CACHE_DIR")):
        dst = os.path.join(_tmp, sub)
        os.makedirs(dst, mode=0o700, exist_ok=True)
        src = os.path.join(_MIO, sub)
        if os.path.isdir(src):
            for f in os.listdir(src):
                if not os.path.exists(os.path.join(dst, f)):
                    # copy + atomic rename: the ranks of one node share this dir
                    part = os.path.join(dst, f".{f}.{os.getpid()}.part")
                    shutil.copy2(os.path.join(src, f), part)
                    os.replace(part, os.path.join(dst, f))
        os.environ.setdefault(var, dst)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

BASELINE_METRIC = "images/sec (whole node) + scaling efficiency, ResNet-50 bf16 at 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    # 2048 images per GPU (peak HBM use is printed on stderr; one MI355X holds
    # 288 GB).  bs512 -> 1024: +4.6% img/s, 1024 -> 1536 -> 2048: +1.4% / +2.9% (fewer,
    # longer kernels per image; the find-db in .miopen covers 512/768/1024/1536/2048).
    # 8 x 2048 = 16k global batch is LARS territory (You et al., arXiv 1708.03888):
    # --optimizer lars measures the same img/s; 8 x 1024 = Goyal et al.'s 8k SGD recipe.
    ap.add_argument("--batch", type=int, default=int(os.environ.get("MIVOD_BENCH_BATCH", 2048)),
                    help="per-GPU batch")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--optimizer", default="sgd", choices=["sgd", "lars", "torch-sgd"])
    ap.add_argument("--compression", default="none", choices=["none", "fp16", "bf16"])
    ap.add_argument("--no-channels-last", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--graph", action="store_true",
                    help="capture the whole step (fwd+bwd+allreduce+fused update) in a HIP graph "
                         "after the warmup steps and replay it (mivod.torch.make_graphed_step)")
    return ap.parse_args()


def _transport(size: int) -> str:
    from mivod.common import basics
    st = basics.state()
    if size == 1 and st.gpu is None:
        return "local"
    return st.backend


def self_launch(argv, nproc: int, script: str = None) -> int:
    """Start ``nproc`` ranks of this script (one per GPU) and wait for them.
    Runs before any GPU call in this process (device_count() does not
    initialise the GPU), so no process that touched the GPU is ever replaced."""
    import torch
    from mivod.run.launcher import assign_slots, launch
    ndev = torch.cuda.device_count()
    extra = {}
    if ndev < nproc:
        if os.environ.get("MIVOD_BENCH_SHARE_GPUS", "0") != "1":
            print(f"bench.py: --gpus {nproc} but only {ndev} GPU(s) are visible "
                  "(set MIVOD_BENCH_SHARE_GPUS=1 to rehearse with shared GPUs)", file=sys.stderr)
            return 2
        extra["MIVOD_TRANSPORT"] = os.environ.get("MIVOD_TRANSPORT", "gloo-gpu")
    slots = assign_slots([("localhost", nproc)], nproc)
    cmd = [sys.executable, script or os.path.abspath(__file__)] + list(argv)
    return launch(slots, cmd, extra, tag_output=False)


def make_record(args, size: int, ips: float, ms: float, transport: str, comm: dict) -> dict:
    """The ONE JSON line rank 0 prints (driver contract + BASELINE.json metric)."""
    return {
        "metric": BASELINE_METRIC,
        "value": round(ips, 2),
        "unit": "images/sec",
        "n_gpus": size,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (on-device uniform images, random labels; random-init weights)",
        "config": {
            "model": "ResNet-50",
            "global_batch": args.batch * size,
            "per_gpu_batch": args.batch,
            "seq_len": None,
            "image": args.image,
            "parallelism": f"dp{size}",
            "optimizer": f"mivod Fused{args.optimizer.upper()} via DistributedOptimizer",
            "compression": args.compression,
            "transport": transport,
            "hip_graph": bool(args.graph),
        },
        "comm": comm,
    }


def _launched() -> bool:
    return any(k in os.environ for k in ("WORLD_SIZE", "HOROVOD_RANK", "OMPI_COMM_WORLD_RANK"))


def main():
    args = parse()
    if args.gpus > 1 and not _launched():
        sys.exit(self_launch(sys.argv[1:], args.gpus))
    import torch
    import torch.nn.functional as F

    from mivod.utils import benchutil as BU
    BU.multi_rank_defaults()        # multi-rank: a stuck collective ends the job with a diagnosis

    import mivod.torch as hvd
    from mivod.models.resnet import resnet50, to_mixed_bf16
    from mivod.optim import FusedLARS, FusedSGD
    from mivod.parallel import collectives as C

    hvd.init()
    if hvd.size() != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {hvd.size()} ranks; "
              "reporting the actual world size", file=sys.stderr)
    rank, size = hvd.rank(), hvd.size()
    dev = hvd.device()
    assert dev.type == "cuda", "bench.py needs a GPU"
    torch.backends.cudnn.benchmark = True

    torch.manual_seed(1234 + rank)
    model = resnet50()
    model = to_mixed_bf16(model, channels_last=not args.no_channels_last).to(dev)
    lr = 0.1 * size
    if args.optimizer == "sgd":
        opt = FusedSGD(model.parameters(), lr=lr, momentum=0.9, weight_decay=5e-5)
    elif args.optimizer == "lars":
        opt = FusedLARS(model.parameters(), lr=lr, momentum=0.9, weight_decay=5e-5)
    else:
        opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=0.9, weight_decay=5e-5,
                              foreach=True)
    comp = hvd.Compression.by_name(args.compression)
    opt = hvd.DistributedOptimizer(opt, named_parameters=model.named_parameters(),
                                   compression=comp)
    hvd.broadcast_parameters(model.state_dict(), root_rank=0)
    hvd.broadcast_optimizer_state(opt, root_rank=0)

    mf = torch.contiguous_format if args.no_channels_last else torch.channels_last
    g = torch.Generator(device=dev)
    g.manual_seed(42 + rank)
    images = torch.rand(args.batch, 3, args.image, args.image, device=dev, generator=g)
    images = images.to(torch.bfloat16).contiguous(memory_format=mf)
    labels = torch.randint(0, 1000, (args.batch,), device=dev, generator=g)

    def step():
        out = model(images)
        loss = F.cross_entropy(out.float(), labels)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    t_w0 = time.perf_counter()
    if args.graph:
        if args.optimizer == "torch-sgd":
            raise SystemExit("--graph needs a mivod fused optimizer (sgd / lars)")
        step = hvd.make_graphed_step(step, opt, model=model, warmup=max(args.warmup, 1))
        if rank == 0:
            print(f"[bench] {max(args.warmup, 1)} eager warmup steps + HIP-graph capture done at "
                  f"{time.perf_counter() - t_w0:.1f}s", file=sys.stderr, flush=True)
        step()   # first replay (untimed)
    else:
        for i in range(args.warmup):
            loss = step()
            if rank == 0 and (i < 3 or i == args.warmup - 1):
                torch.cuda.synchronize()
                print(f"[bench] warmup step {i} done at {time.perf_counter() - t_w0:.1f}s",
                      file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    warm_s = time.perf_counter() - t_w0

    comm_stream = hvd.comm_stream()
    timing = []                       # (backward enqueued, comm stream drained) per step

    def timed_step():
        out = model(images)
        loss = F.cross_entropy(out.float(), labels)
        loss.backward()
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        opt.step()
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record(comm_stream)
        opt.zero_grad(set_to_none=True)
        timing.append((e0, e1))
        return loss

    run = step if args.graph else timed_step
    timed_comm = not args.graph and getattr(opt, "_mvd_comm", False)
    if timed_comm:
        opt.time_comm(True)          # timing events around every bucket collective
    stats0 = C.gpu_stats()
    C.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = run()
    torch.cuda.synchronize()
    C.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = C.max_over_ranks(elapsed)
    stats1 = C.gpu_stats()
    ms = elapsed / max(args.steps, 1) * 1000.0
    ips = args.batch * size * args.steps / elapsed
    plan = opt.bucket_plan()
    grad_bytes = sum(nb for _, nb, _ in plan)
    exposed = [max(0.0, a.elapsed_time(b)) for a, b in timing] if timing else []
    calls = (stats1.get("calls", 0) - stats0.get("calls", 0)) / max(args.steps, 1)
    measured = BU.comm_timing_record(opt.comm_timings() if timed_comm else [], args.steps, size)
    comm = {
        "buckets": len(plan),
        "grad_bytes_per_step": grad_bytes,
        "ring_wire_bytes_per_rank_per_step": int(2 * (size - 1) / size * grad_bytes),
        "collectives_per_step": round(calls, 2),
        "exposed_comm_ms": round(sum(exposed) / len(exposed), 3) if exposed else None,
        "exposed_comm_ms_max": round(max(exposed), 3) if exposed else None,
        **measured,
        "rccl": BU.rccl_info(),
    }
    if rank == 0:
        print(f"[bench] warmup {args.warmup} steps {warm_s:.1f}s; loss {float(loss.detach()):.4f}; "
              f"{ms:.2f} ms/step; buckets={len(opt.bucket_plan())}; peak HBM "
              f"{torch.cuda.max_memory_allocated(dev) / 2**30:.1f} GiB", file=sys.stderr)
        rec = make_record(args, size, ips, ms, _transport(size), comm)
        print(json.dumps(rec), flush=True)
    hvd.shutdown()


if __name__ == "__main__":
    main()
