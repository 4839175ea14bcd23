#!/bin/bash
# 224-row blocks on the 256-wide pipeline: GEMM + conv tests, micros, bench A/B vs 256-row blocks
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_conv_gpu.py tests/test_gemm_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g224_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/g224_pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED|Mismatch|Greatest" gpurun_out/g224_pytest.log | head -30; exit $rc; }
for v in 224 256; do
  MIVOD_G256_BM=$v timeout -k 10 300 python scripts/micro_conv3x3.py > gpurun_out/g224_conv_$v.log 2>&1 || { tail -20 gpurun_out/g224_conv_$v.log; exit 1; }
  MIVOD_G256_BM=$v timeout -k 10 300 python scripts/micro_gemm256.py > gpurun_out/g224_gemm_$v.log 2>&1 || { tail -20 gpurun_out/g224_gemm_$v.log; exit 1; }
  echo "== BM $v"; grep -v amdgpu.ids gpurun_out/g224_conv_$v.log | grep -v "^wgrad\|56"; grep -v amdgpu.ids gpurun_out/g224_gemm_$v.log
done
for v in 224 256 224 256; do MIVOD_G256_BM=$v timeout -k 10 300 python bench.py > gpurun_out/g224_bench.log 2>&1 || { tail gpurun_out/g224_bench.log; exit 1; }; echo "bench BM=$v: $(grep -o '"value": [0-9.]*' gpurun_out/g224_bench.log)"; done
