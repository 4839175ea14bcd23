#!/bin/bash
# One GPU session: gpu tests, smoke, a short bench.  Stops at the first
# fault / abort / timeout (exit >= 124 or signal), tolerates plain test failures.
set -u
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 1 ] && [ $rc -ne 5 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
rocm-smi --showproductname > gpurun_out/smi.log 2>&1 || true
step pytest_gpu 900 python -m pytest tests -m gpu -x -q
step smoke 600 python -c "import __graft_entry__ as g; g.smoke()"
step bench1 1200 python bench.py --steps ${BENCH_STEPS:-20} --warmup ${BENCH_WARMUP:-10}
