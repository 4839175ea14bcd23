#!/bin/bash
# Interleaved A/B of bench.py under an env switch:  VAR=MIVOD_BN_STATS_U A=4 B=8 TESTS="tests/x.py"
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    $TESTS -m gpu > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
  tail -1 gpurun_out/ab_pytest.log
fi
for i in 1 2; do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/ab_${v}_$i.log 2>&1 || exit 1
    echo "$VAR=$v run=$i $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/ab_${v}_$i.log | tr '\n' ' ')"
  done
done
