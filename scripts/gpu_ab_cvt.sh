#!/bin/bash
# A/B on ONE box: round-3 kernels (compiler-selected bf16 pack conversion, stem at 2
# waves/SIMD) vs the round-2 sources (inline-asm conversion, stem 1 wave/SIMD):
# per-kernel profiles + 2 benches each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {   # $1 = tag
  TOP=70 TITLE="ResNet-50 bs2048 ($1)" timeout -k 10 600 bash scripts/gpu_prof_resnet.sh > gpurun_out/ab_$1_prof.log 2>&1 || { tail -20 gpurun_out/ab_$1_prof.log; exit 1; }
  cp gpurun_out/prof_summary.md gpurun_out/ab_$1.md
  for i in 1 2; do timeout -k 10 300 python bench.py > gpurun_out/ab_$1_b$i.log 2>&1 || { tail gpurun_out/ab_$1_b$i.log; exit 1; }; echo "$1: $(grep -o '"value": [0-9.]*' gpurun_out/ab_$1_b$i.log)"; done
}
run new
cp scripts/ab/mv_common.h.r2 csrc/kernels/mv_common.h
cp scripts/ab/mv_stem.hip.r2 csrc/kernels/mv_stem.hip
timeout -k 10 900 python -m mivod._build > gpurun_out/ab_build.log 2>&1 || { tail -20 gpurun_out/ab_build.log; exit 1; }
run old
run_new_again() { :; }
