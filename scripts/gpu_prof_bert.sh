#!/bin/bash
# rocprofv3 kernel trace of the 1-GPU BERT-Large bench -> markdown summary
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/profb
timeout -k 10 500 rocprofv3 --kernel-trace -d gpurun_out/profb -o run -- python benchmarks/bench_bert.py --steps 5 --warmup 5 \
  > gpurun_out/profb.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/profb.log; exit 1; }
grep '"metric"' gpurun_out/profb.log | cut -c1-300
DB=$(ls gpurun_out/profb/*.db gpurun_out/profb/*/*.db 2>/dev/null | head -n 1)
python scripts/rocpd_summary.py "$DB" --steps 5 --marker "attn::fwd_kernel" --per-step ${PER_STEP:-24} --top 30 --title "${TITLE:-BERT-Large bs512 seq128}" > gpurun_out/profb_summary.md \
  || python scripts/rocpd_summary.py "$DB" --all --top 30 --title "${TITLE:-BERT-Large} (whole trace)" > gpurun_out/profb_summary.md
head -40 gpurun_out/profb_summary.md
rm -rf gpurun_out/profb
