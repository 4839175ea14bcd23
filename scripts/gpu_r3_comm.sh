#!/bin/bash
# Round 3: the comm-path changes on ONE GPU — multi-rank GPU tests (gloo-gpu / mesh
# over HIP IPC / world-1 RCCL), the 2-rank bench rehearsal with the new JSON
# fields, then the 1-GPU bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py tests/test_kernels_gpu.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r3c_pytest.log 2>&1; rc=$?
tail -25 gpurun_out/r3c_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 bash scripts/gpu_bench_rehearsal.sh > gpurun_out/r3c_rehearsal.log 2>&1 || { tail -30 gpurun_out/r3c_rehearsal.log; exit 1; }
cat gpurun_out/r3c_rehearsal.log
timeout -k 10 300 python bench.py > gpurun_out/r3c_bench.log 2>&1 || { tail -20 gpurun_out/r3c_bench.log; exit 1; }
grep '"metric"' gpurun_out/r3c_bench.log
