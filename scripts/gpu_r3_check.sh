#!/bin/bash
# Round-3 checkpoint: full GPU tier, smoke, 1-GPU bench, rocprofv3 kernel summary.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c3_pytest.log 2>&1; rc=$?
tail -5 gpurun_out/c3_pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/c3_pytest.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c3_smoke.log 2>&1 || { tail gpurun_out/c3_smoke.log; exit 1; }
grep "smoke ok" gpurun_out/c3_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/c3_bench.log 2>&1 || { tail gpurun_out/c3_bench.log; exit 1; }
grep '"metric"' gpurun_out/c3_bench.log
TITLE="ResNet-50 bs2048 round 3 checkpoint" bash scripts/gpu_prof_resnet.sh
