#!/bin/bash
# Round 3 iteration check: selected GPU tests, 1-GPU bench x2, optional profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS="${TESTS:-tests/test_conv_gpu.py tests/test_kernels_gpu.py}"
timeout -k 10 700 python -u -m pytest $TESTS -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/q_pytest.log 2>&1; rc=$?
grep -E "windows|passed|failed|Error" gpurun_out/q_pytest.log | tail -12; [ $rc -ne 0 ] && { tail -40 gpurun_out/q_pytest.log; exit $rc; }
for i in 1 2; do timeout -k 10 300 python bench.py > gpurun_out/q_bench$i.log 2>&1 || { tail gpurun_out/q_bench$i.log; exit 1; }; echo "bench: $(grep -o '"value": [0-9.]*' gpurun_out/q_bench$i.log)"; done
if [ "${PROF:-0}" = "1" ]; then
  TOP=70 TITLE="${TITLE:-ResNet-50 bs2048}" timeout -k 10 600 bash scripts/gpu_prof_resnet.sh > gpurun_out/q_prof.log 2>&1 || { tail -20 gpurun_out/q_prof.log; exit 1; }
  head -8 gpurun_out/prof_summary.md
fi
