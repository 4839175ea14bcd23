#!/bin/bash
# Round-2 GPU check: GPU test tier, 1-GPU bench, bench through mivod's RCCL comm
# (forced at world size 1), and a kernel-trace profile of the forced-RCCL bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/gputest.log 2>&1 || { echo "GPU tests failed"; tail -40 gpurun_out/gputest.log; exit 1; }
tail -3 gpurun_out/gputest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 5 > gpurun_out/bench.log 2>&1 \
  || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
MIVOD_FORCE_COLLECTIVES=1 timeout -k 10 300 python bench.py --steps 10 --warmup 5 \
  > gpurun_out/bench_forced.log 2>&1 || { echo "forced bench failed"; tail -30 gpurun_out/bench_forced.log; exit 1; }
tail -2 gpurun_out/bench_forced.log
MIVOD_FORCE_COLLECTIVES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_forced \
  -o run -- python bench.py --steps 5 --warmup 3 > gpurun_out/prof_forced.log 2>&1 \
  || { echo "profile failed"; tail -30 gpurun_out/prof_forced.log; exit 1; }
echo done
