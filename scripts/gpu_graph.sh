#!/bin/bash
# HIP-graph step: tests, then eager vs graph bench at a small and the default batch.
set -u
mkdir -p gpurun_out
run() {  # run <log> <timeout> <cmd...>; stop on fault/timeout
  local log=$1 t=$2; shift 2
  echo "=== $log: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "=== $log rc=$rc"; tail -n 4 "gpurun_out/$log" | cut -c1-400
  if { [ $rc -ge 2 ] && [ $rc -ne 5 ]; }; then echo "STOP after $log (rc=$rc)"; exit $rc; fi
}
run graph_tests.log 300 python -u -m pytest tests/test_graphs_gpu.py -x -q --timeout 120 --timeout-method thread
for bs in ${GRAPH_BATCHES:-512 1024}; do
  run bench_eager_bs$bs.log 400 python bench.py --batch $bs --steps 20 --warmup 5
  run bench_graph_bs$bs.log 400 python bench.py --batch $bs --steps 20 --warmup 5 --graph
done
