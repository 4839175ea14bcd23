#!/bin/bash
# Round-end style check: GPU tests, smoke, bench (3 runs), kernel profile of the bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/final_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/final_pytest.log; [ $rc -ge 2 ] && [ $rc -ne 5 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || exit 1
grep "smoke ok" gpurun_out/final_smoke.log
for i in 1 2 3; do timeout -k 10 300 python bench.py > gpurun_out/final_bench$i.log 2>&1 || exit 1; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/final_bench$i.log | tr '\n' ' '; echo; done
rm -rf /tmp/prof_final
timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/prof_final -o run --output-format csv -- python bench.py --steps 6 --warmup 3 > gpurun_out/final_prof.log 2>&1 || exit 1
f=$(find /tmp/prof_final -name "*kernel_trace.csv" | head -1)
python scripts/prof_summary.py "$f" --steps 5 --title "ResNet-50 bf16 bs2048 1xMI355X — bench.py default (round-1 final)" > gpurun_out/summary_final.md 2>&1
head -8 gpurun_out/summary_final.md
