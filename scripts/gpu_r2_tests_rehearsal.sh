#!/bin/bash
# Full GPU test tier + smoke + 2-rank torch.distributed.run rehearsal of bench.py / bench_bert.py
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=5 -q --timeout 200 --timeout-method thread > gpurun_out/v_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/v_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v_smoke.log 2>&1 || exit 1
grep "smoke ok" gpurun_out/v_smoke.log
timeout -k 10 900 bash scripts/gpu_bench_rehearsal.sh || exit 1
