#!/bin/bash
# Two kernel profiles of the 1-GPU bench in one call, A/B on one env setting:
#   VAR=MIVOD_X A=1 B=0 bash scripts/gpu_prof_ab.sh   -> gpurun_out/prof_A.md, prof_B.md
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in $A $B; do
  env $VAR=$v TOP=${TOP:-70} TITLE="$VAR=$v" bash scripts/gpu_prof_resnet.sh > /dev/null || exit 1
  cp gpurun_out/prof_summary.md gpurun_out/prof_$v.md
  echo "$VAR=$v $(sed -n 3p gpurun_out/prof_$v.md)"
done
