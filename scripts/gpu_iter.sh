#!/bin/bash
# Iteration check on one GPU: the named GPU test files, then bench.py (optionally an A/B
# with one env setting).   TESTS="tests/a.py tests/b.py" AB="MIVOD_X=0" bash scripts/gpu_iter.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/it_pytest.log 2>&1; rc=$?
  tail -3 gpurun_out/it_pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED|Timeout" gpurun_out/it_pytest.log | head -30; exit $rc; }
fi
if [ -n "${MICRO:-}" ]; then
  timeout -k 10 300 python $MICRO > gpurun_out/it_micro.log 2>&1 || { tail gpurun_out/it_micro.log; exit 1; }
  cat gpurun_out/it_micro.log
fi
timeout -k 10 300 python bench.py > gpurun_out/it_bench.log 2>&1 || { tail gpurun_out/it_bench.log; exit 1; }
echo "bench: $(grep -o '"value": [0-9.]*' gpurun_out/it_bench.log)"
if [ -n "${AB:-}" ]; then
  env $AB timeout -k 10 300 python bench.py > gpurun_out/it_bench_ab.log 2>&1 || { tail gpurun_out/it_bench_ab.log; exit 1; }
  echo "bench $AB: $(grep -o '"value": [0-9.]*' gpurun_out/it_bench_ab.log)"
  timeout -k 10 300 python bench.py > gpurun_out/it_bench2.log 2>&1 || { tail gpurun_out/it_bench2.log; exit 1; }
  echo "bench again: $(grep -o '"value": [0-9.]*' gpurun_out/it_bench2.log)"
fi
exit 0
