#!/bin/bash
# gemm256 (256x256 glds-pipelined NT GEMM): GEMM tests, micro vs CK / hipBLASLt, bench A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g256_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/g256_pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/g256_pytest.log | head -30; exit $rc; }
timeout -k 10 300 python scripts/micro_gemm256.py > gpurun_out/g256_micro.log 2>&1 || { tail -20 gpurun_out/g256_micro.log; exit 1; }
grep -v amdgpu.ids gpurun_out/g256_micro.log
for v in 1 0; do MIVOD_GEMM256=$v timeout -k 10 300 python bench.py > gpurun_out/g256_bench_$v.log 2>&1 || { tail gpurun_out/g256_bench_$v.log; exit 1; }; echo "bench GEMM256=$v: $(grep -o '"value": [0-9.]*' gpurun_out/g256_bench_$v.log)"; done
