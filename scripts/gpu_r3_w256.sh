#!/bin/bash
# wgrad256 (1x1 weight gradient on the 256x256 pipeline): tests, micro on/off, bench A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_gemm_gpu.py -m gpu -x -q -k "wgrad or fold or gram or dual" --timeout 200 --timeout-method thread > gpurun_out/w256_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/w256_pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/w256_pytest.log | head -30; exit $rc; }
for v in 1 0; do MIVOD_WGRAD256=$v timeout -k 10 400 python scripts/micro_wgrad1x1.py > gpurun_out/w256_micro_$v.log 2>&1 || { tail -20 gpurun_out/w256_micro_$v.log; exit 1; }; echo "WGRAD256=$v"; grep -v amdgpu.ids gpurun_out/w256_micro_$v.log | tail -8; done
for v in 1 0; do MIVOD_WGRAD256=$v timeout -k 10 300 python bench.py > gpurun_out/w256_bench_$v.log 2>&1 || { tail gpurun_out/w256_bench_$v.log; exit 1; }; echo "bench WGRAD256=$v: $(grep -o '"value": [0-9.]*' gpurun_out/w256_bench_$v.log)"; done
