#!/bin/bash
# Rehearse the multi-rank bench path (torch.distributed.run, N=2) on ONE GPU: both ranks
# share cuda:0 over the gloo wire (RCCL refuses two ranks per device).  Checks the code
# path (init, rings, bucket schedule, broadcasts, timing, JSON), not throughput.
set -u
mkdir -p gpurun_out
export MIVOD_TRANSPORT=gloo-gpu
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 --batch 64 > gpurun_out/rehearsal_resnet.log 2>&1 || { tail -30 gpurun_out/rehearsal_resnet.log; exit 1; }
grep '"metric"' gpurun_out/rehearsal_resnet.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29534 benchmarks/bench_bert.py --steps 3 --warmup 2 --batch 8 > gpurun_out/rehearsal_bert.log 2>&1 || { tail -30 gpurun_out/rehearsal_bert.log; exit 1; }
grep '"metric"' gpurun_out/rehearsal_bert.log
