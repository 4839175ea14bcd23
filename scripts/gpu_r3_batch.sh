#!/bin/bash
# Round-3 batch: the given GPU tests, bench A/B with one env setting, kernel profile.
#   TESTS="..." AB="MIVOD_X=0" TITLE="..." bash scripts/gpu_r3_batch.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS="${TESTS:-}" AB="${AB:-}" bash scripts/gpu_iter.sh || exit 1
TOP=${TOP:-60} TITLE="${TITLE:-batch profile}" bash scripts/gpu_prof_resnet.sh > /dev/null && cp gpurun_out/prof_summary.md gpurun_out/batch_prof.md || exit 1
echo batch done
