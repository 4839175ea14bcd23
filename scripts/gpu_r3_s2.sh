#!/bin/bash
# stride-2 3x3 data gradient: tests, micro, bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dgrad_s2_gpu.py tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s2_pytest.log 2>&1; rc=$?
tail -5 gpurun_out/s2_pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/s2_pytest.log | head -30; exit $rc; }
timeout -k 10 200 python scripts/micro_dgrad_s2.py > gpurun_out/s2_micro.log 2>&1 || { tail gpurun_out/s2_micro.log; exit 1; }
cat gpurun_out/s2_micro.log
timeout -k 10 300 python bench.py > gpurun_out/s2_bench.log 2>&1 || { tail gpurun_out/s2_bench.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/s2_bench.log
MIVOD_CONV3X3_DGRAD_S2=0 timeout -k 10 300 python bench.py > gpurun_out/s2_bench0.log 2>&1 || { tail gpurun_out/s2_bench0.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/s2_bench0.log
