#!/bin/bash
# Re-entry check: full GPU test tier, smoke, ResNet-50 bench x2, BERT-Large bench x1.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -q --timeout 200 --timeout-method thread > gpurun_out/v_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/v_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v_smoke.log 2>&1 || exit 1
grep "smoke ok" gpurun_out/v_smoke.log
for i in 1 2; do timeout -k 10 300 python bench.py > gpurun_out/v_bench$i.log 2>&1 || exit 1; grep '"metric"' gpurun_out/v_bench$i.log; done
timeout -k 10 400 python benchmarks/bench_bert.py > gpurun_out/v_bert.log 2>&1 || exit 1
grep '"metric"' gpurun_out/v_bert.log
[ "${VERIFY_PROF:-1}" = "1" ] || exit 0
TITLE="ResNet-50 bs2048 1xMI355X (round 2, BN3 fold)" timeout -k 10 600 bash scripts/gpu_prof_resnet.sh > gpurun_out/v_prof.log 2>&1 || { tail -5 gpurun_out/v_prof.log; exit 1; }
head -12 gpurun_out/prof_summary.md
