#!/bin/bash
# rocprofv3 kernel trace of the 1-GPU ResNet-50 bench -> markdown summary
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 5 \
  > gpurun_out/prof.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/prof.log; exit 1; }
grep '"metric"' gpurun_out/prof.log
DB=$(ls gpurun_out/prof/*.db gpurun_out/prof/*/*.db 2>/dev/null | head -n 1)
python scripts/rocpd_summary.py "$DB" --steps 5 --per-step ${PER_STEP:-5} --top ${TOP:-45} --title "${TITLE:-ResNet-50 bs2048}" ${DETAIL:+--detail "$DETAIL"} > gpurun_out/prof_summary.md \
  || python scripts/rocpd_summary.py "$DB" --all --top ${TOP:-45} --title "${TITLE:-ResNet-50 bs2048} (whole trace)" > gpurun_out/prof_summary.md
head -60 gpurun_out/prof_summary.md
rm -rf gpurun_out/prof
