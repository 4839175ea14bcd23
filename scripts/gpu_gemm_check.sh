#!/bin/bash
# GEMM microbench, GEMM / fused conv-BN tests, then the 1-GPU bench A/B of the
# backward fusion (MIVOD_CONV_BN_BWD_FUSE).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/micro_gemm1x1.py > gpurun_out/micro_gemm.log 2>&1 \
  || { echo "micro failed"; tail -30 gpurun_out/micro_gemm.log; exit 1; }
cat gpurun_out/micro_gemm.log
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_resnet_paths_gpu.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/gemm_tests.log; exit 1; }
tail -2 gpurun_out/gemm_tests.log
for v in ${BWD_AB:-1 0 1 0}; do
  MIVOD_CONV_BN_BWD_FUSE=$v timeout -k 10 300 python bench.py --steps 10 --warmup 5 > gpurun_out/bench_bwd$v.log 2>&1 \
    || { echo "bench failed"; tail -20 gpurun_out/bench_bwd$v.log; exit 1; }
  echo "bwdfuse=$v $(grep -o '"value": [0-9.]*' gpurun_out/bench_bwd$v.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_bwd$v.log)"
done
