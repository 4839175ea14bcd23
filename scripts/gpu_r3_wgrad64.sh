#!/bin/bash
# wgrad64 (row-patch 64->64 3x3 weight gradient): conv tests, wgrad micro on/off, bench A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py -m gpu -x -q -k "wgrad" --timeout 200 --timeout-method thread > gpurun_out/w64_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/w64_pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/w64_pytest.log | head -30; exit $rc; }
for v in 1 0; do MIVOD_WGRAD64=$v timeout -k 10 300 python scripts/micro_conv3x3.py > gpurun_out/w64_micro_$v.log 2>&1 || { tail -20 gpurun_out/w64_micro_$v.log; exit 1; }; echo "WGRAD64=$v"; grep wgrad gpurun_out/w64_micro_$v.log; done
for v in 1 0; do MIVOD_WGRAD64=$v timeout -k 10 300 python bench.py > gpurun_out/w64_bench_$v.log 2>&1 || { tail gpurun_out/w64_bench_$v.log; exit 1; }; echo "bench WGRAD64=$v: $(grep -o '"value": [0-9.]*' gpurun_out/w64_bench_$v.log)"; done
