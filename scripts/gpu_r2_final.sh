#!/bin/bash
# Round-2 end check: full GPU tier, smoke, bench x2, kernel profile of the bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=5 -q --timeout 200 --timeout-method thread > gpurun_out/f_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/f_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f_smoke.log 2>&1 || exit 1
grep "smoke ok" gpurun_out/f_smoke.log
for i in 1 2; do timeout -k 10 300 python bench.py > gpurun_out/f_bench$i.log 2>&1 || exit 1; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/f_bench$i.log | tr '\n' ' '; echo; done
TITLE="${TITLE:-ResNet-50 bs2048 1xMI355X (round 2 final)}" timeout -k 10 600 bash scripts/gpu_prof_resnet.sh > gpurun_out/f_prof.log 2>&1 || { tail -5 gpurun_out/f_prof.log; exit 1; }
head -5 gpurun_out/prof_summary.md
