#!/bin/bash
# One GPU session: (optional) selected gpu tests, refresh the MIOpen find-db for
# new conv problems (NORMAL find on top of the shipped .miopen db), then A/B
# bench variants with that db.  Stops at the first fault / timeout.
#   TESTS="tests/test_pool_gpu.py"  VARIANTS="default nodgrad stem3"  bash scripts/gpu_ab.sh
set -u
mkdir -p gpurun_out/mio_new/db gpurun_out/mio_new/cache
cp -rn .miopen/db/. gpurun_out/mio_new/db/ && cp -rn .miopen/cache/. gpurun_out/mio_new/cache/
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/mio_new/db
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/gpurun_out/mio_new/cache
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -E '^\{|ms/step|passed|failed|Error|error' "gpurun_out/$name.log" | cut -c1-300 | tail -6
  if { [ $rc -ge 2 ] && [ $rc -ne 5 ]; } || [ $rc -eq 1 -a "$name" != pytest ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
if [ -n "${TESTS:-}" ]; then
  run pytest 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread $TESTS -m gpu
fi
if [ "${REFRESH:-1}" = 1 ]; then
  MIOPEN_FIND_MODE=NORMAL run refresh 600 python bench.py --steps 3 --warmup 2 ${BENCH_ARGS:-}
fi
for v in ${VARIANTS:-default}; do
  case $v in
    default) run b_default 300 python bench.py --steps 20 --warmup 10 ${BENCH_ARGS:-} ;;
    nodgrad) MIVOD_CONV_DGRAD_FWD=0 run b_nodgrad 300 python bench.py --steps 20 --warmup 10 ${BENCH_ARGS:-} ;;
    stem3) MIVOD_STEM_CHANNELS=3 run b_stem3 300 python bench.py --steps 20 --warmup 10 ${BENCH_ARGS:-} ;;
    prof) cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
          run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 5 ${BENCH_ARGS:-} ;;
  esac
done
