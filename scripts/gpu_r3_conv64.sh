#!/bin/bash
# conv64 (row-patch 64->64 3x3 kernel): tests, micro vs generic kernel vs MIOpen, bench, profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c64_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/c64_pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/c64_pytest.log | head -30; exit $rc; }
for v in 1 0; do MIVOD_CONV64=$v timeout -k 10 300 python scripts/micro_conv3x3.py > gpurun_out/c64_micro_$v.log 2>&1 || { tail -20 gpurun_out/c64_micro_$v.log; exit 1; }; echo "CONV64=$v"; head -9 gpurun_out/c64_micro_$v.log | grep -v amdgpu.ids; done
for v in 1 0; do MIVOD_CONV64=$v timeout -k 10 300 python bench.py > gpurun_out/c64_bench_$v.log 2>&1 || { tail gpurun_out/c64_bench_$v.log; exit 1; }; echo "bench CONV64=$v: $(grep -o '"value": [0-9.]*' gpurun_out/c64_bench_$v.log)"; done
TOP=70 TITLE="ResNet-50 bs2048 round 3 (conv64 row-patch kernel)" timeout -k 10 600 bash scripts/gpu_prof_resnet.sh > gpurun_out/c64_prof.log 2>&1 || { tail -20 gpurun_out/c64_prof.log; exit 1; }
cp gpurun_out/prof_summary.md gpurun_out/c64_prof.md; head -30 gpurun_out/c64_prof.md
