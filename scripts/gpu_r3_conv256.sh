#!/bin/bash
# conv256 (3x3 implicit GEMM on the 256x256 glds pipeline): conv tests, micro A/B, bench A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c256_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/c256_pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED|Mismatch|Greatest" gpurun_out/c256_pytest.log | head -30; exit $rc; }
for v in 1 0; do MIVOD_CONV256=$v timeout -k 10 300 python scripts/micro_conv3x3.py > gpurun_out/c256_micro_$v.log 2>&1 || { tail -20 gpurun_out/c256_micro_$v.log; exit 1; }; echo "== micro CONV256=$v"; grep -v amdgpu.ids gpurun_out/c256_micro_$v.log; done
for v in 1 0; do MIVOD_CONV256=$v timeout -k 10 300 python bench.py > gpurun_out/c256_bench_$v.log 2>&1 || { tail gpurun_out/c256_bench_$v.log; exit 1; }; echo "bench CONV256=$v: $(grep -o '"value": [0-9.]*' gpurun_out/c256_bench_$v.log)"; done
