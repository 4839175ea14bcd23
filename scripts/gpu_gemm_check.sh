#!/bin/bash
# GEMM / fused conv-BN tests, then the 1-GPU bench with and without the fusion.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_resnet_paths_gpu.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/gemm_tests.log; exit 1; }
tail -2 gpurun_out/gemm_tests.log
for v in 1 0 1 0; do
  MIVOD_CONV_BN_FUSE=$v timeout -k 10 300 python bench.py --steps 10 --warmup 5 > gpurun_out/bench_fuse$v.log 2>&1 \
    || { echo "bench failed"; tail -20 gpurun_out/bench_fuse$v.log; exit 1; }
  echo "fuse=$v $(grep -o '"value": [0-9.]*' gpurun_out/bench_fuse$v.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_fuse$v.log)"
done
