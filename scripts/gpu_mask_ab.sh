#!/bin/bash
# BN add+ReLU backward: bitmask (mode 3) vs saved-output (mode 2) -- tests, interleaved
# A/B bench, and the micro benchmark kernel times.  Stops at the first failure.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_pool_gpu.py -m gpu > gpurun_out/mask_pytest.log 2>&1 || { tail -30 gpurun_out/mask_pytest.log; exit 1; }
tail -1 gpurun_out/mask_pytest.log
for i in 1 2; do
  for m in 0 1; do
    MIVOD_BN_MASK=$m timeout -k 10 300 python bench.py > gpurun_out/mask_b${m}_$i.log 2>&1 || exit 1
    echo "mask=$m run=$i $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/mask_b${m}_$i.log | tr '\n' ' ')"
  done
done
