#!/bin/bash
# conv256 + wgrad256<9>: conv tests, micro, bench A/B (all on / conv256 off / wgrad 3x3 off), profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c256_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/c256_pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED|Mismatch|Greatest" gpurun_out/c256_pytest.log | head -30; exit $rc; }
timeout -k 10 300 python scripts/micro_conv3x3.py > gpurun_out/c256_micro.log 2>&1 || { tail -20 gpurun_out/c256_micro.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c256_micro.log
for cfg in "X=1" "MIVOD_CONV256=0" "MIVOD_WGRAD256_3X3=0" "X=2"; do env $cfg timeout -k 10 300 python bench.py > gpurun_out/c256_bench.log 2>&1 || { tail gpurun_out/c256_bench.log; exit 1; }; echo "bench $cfg: $(grep -o '"value": [0-9.]*' gpurun_out/c256_bench.log)"; done
timeout -k 10 300 python scripts/micro_gemm256.py > gpurun_out/g256_micro.log 2>&1 && grep -v amdgpu.ids gpurun_out/g256_micro.log
TITLE="ResNet-50 bs2048 conv256 + wgrad256<9>" bash scripts/gpu_prof_resnet.sh
