#!/bin/bash
# BN kernel bandwidth under two values of an env switch (rocprofv3 kernel trace of
# scripts/micro_bn.py):  VAR=MIVOD_BN_APPLY_U A=2 B=4 bash scripts/gpu_micro_bn_ab.sh
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in $A $B; do
  rm -rf /tmp/prof_mbn_$v
  env $VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_mbn_$v -o run --output-format csv \
    -- python scripts/micro_bn.py > gpurun_out/mbn_$v.log 2>&1 || { tail -20 gpurun_out/mbn_$v.log; exit 1; }
  f=$(find /tmp/prof_mbn_$v -name "*kernel_trace.csv" | head -1)
  python scripts/micro_bn.py --parse "$f" > gpurun_out/mbn_${VAR}_$v.md || exit 1
done
paste -d' ' <(cut -d'|' -f2-5 gpurun_out/mbn_${VAR}_$A.md) <(cut -d'|' -f5,7 gpurun_out/mbn_${VAR}_$B.md)
