#!/bin/bash
# gemm256 routing round 2: model-path tests, bench, vendor-kernel census, rocprof summary
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gemm_gpu.py tests/test_resnet_paths_gpu.py tests/test_conv_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g2_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/g2_pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/g2_pytest.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/g2_bench.log 2>&1 || { tail gpurun_out/g2_bench.log; exit 1; }
echo "bench: $(grep -o '"value": [0-9.]*' gpurun_out/g2_bench.log)"
timeout -k 10 400 python scripts/debug/find_vendor.py > gpurun_out/g2_vendor.log 2>&1 || { tail gpurun_out/g2_vendor.log; exit 1; }
grep "non-mivod" gpurun_out/g2_vendor.log
TOP=70 TITLE="ResNet-50 bs2048 round 3 (gemm256)" timeout -k 10 600 bash scripts/gpu_prof_resnet.sh > gpurun_out/g2_prof.log 2>&1 || { tail -20 gpurun_out/g2_prof.log; exit 1; }
cp gpurun_out/prof_summary.md gpurun_out/g2_prof.md; head -12 gpurun_out/g2_prof.md
