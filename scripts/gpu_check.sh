#!/bin/bash
# One GPU session: gpu tests, smoke, a short bench, a rocprofv3 kernel profile.
# Stops at the first fault / abort / timeout (rc >= 124 or 2..), tolerates plain
# test failures (rc 1) and "no tests" (rc 5).
set -u
mkdir -p gpurun_out
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/gpurun_out/miopen_cache
mkdir -p "$MIOPEN_USER_DB_PATH" "$MIOPEN_CUSTOM_CACHE_DIR"
[ -d .miopen/db ] && cp -rn .miopen/db/. "$MIOPEN_USER_DB_PATH"/ 2>/dev/null
[ -d .miopen/cache ] && cp -rn .miopen/cache/. "$MIOPEN_CUSTOM_CACHE_DIR"/ 2>/dev/null
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if { [ $rc -ge 2 ] && [ $rc -ne 5 ]; }; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
rocm-smi --showproductname > gpurun_out/smi.log 2>&1 || true
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
  step smoke 600 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench1 1200 python bench.py --steps ${BENCH_STEPS:-20} --warmup ${BENCH_WARMUP:-10} ${BENCH_ARGS:-}
if [ "${PROFILE:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  step rocprof 1200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 5 ${BENCH_ARGS:-}
fi
