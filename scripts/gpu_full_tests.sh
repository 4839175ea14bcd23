#!/bin/bash
# Full GPU test tier (one process) + smoke
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "PASSED|FAILED|ERROR" gpurun_out/gpu_tests.log | tail -5; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
