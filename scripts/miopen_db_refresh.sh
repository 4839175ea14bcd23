#!/bin/bash
# Rebuild the shipped MIOpen find-db / kernel cache (.miopen) for bench.py:
# run 1 populates a fresh db (naive direct-conv solvers disabled, as in bench.py),
# run 2 must then start fast.  Outputs land in gpurun_out/miopen_fresh/.
set -u
mkdir -p gpurun_out/miopen_fresh/db gpurun_out/miopen_fresh/cache
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_fresh/db
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/gpurun_out/miopen_fresh/cache
for i in 1 2; do
  timeout -k 10 500 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/miofresh_$i.log 2>&1
  rc=$?
  echo "run $i rc=$rc"; grep -E "^\{|\[bench\] warmup" gpurun_out/miofresh_$i.log | cut -c1-200
  [ $rc -ne 0 ] && exit $rc
done
ls -la gpurun_out/miopen_fresh/db gpurun_out/miopen_fresh/cache
