#!/bin/bash
# Round 3 check: full GPU tier, smoke, 1-GPU bench x2, the 2-rank bench rehearsal (new
# comm JSON fields), the RCCL PreMulSum tail probe.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/v3_pytest.log 2>&1; rc=$?
tail -15 gpurun_out/v3_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v3_smoke.log 2>&1 || { tail gpurun_out/v3_smoke.log; exit 1; }
grep "smoke ok" gpurun_out/v3_smoke.log
for i in 1 2; do timeout -k 10 300 python bench.py > gpurun_out/v3_bench$i.log 2>&1 || { tail gpurun_out/v3_bench$i.log; exit 1; }; grep '"metric"' gpurun_out/v3_bench$i.log; done
timeout -k 10 500 bash scripts/gpu_bench_rehearsal.sh > gpurun_out/v3_rehearsal.log 2>&1 || { tail -30 gpurun_out/v3_rehearsal.log; exit 1; }
cat gpurun_out/v3_rehearsal.log
timeout -k 10 120 python scripts/debug/premul_tail.py > gpurun_out/v3_premul.log 2>&1; tail -40 gpurun_out/v3_premul.log
