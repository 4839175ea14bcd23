#!/bin/bash
# Round 3: convergence guard, Keras overlap (2 ranks on 1 GPU), multirank comm tests,
# stray elementwise kernels, BERT-Large config-5 bench (overlapped overflow guard).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_resnet_convergence_gpu.py tests/test_keras_gpu.py tests/test_multirank_gpu.py -m gpu -x -v -s --timeout 400 --timeout-method thread > gpurun_out/m_pytest.log 2>&1; rc=$?
grep -E "windows|PASSED|FAILED|SKIPPED|Error|passed|failed" gpurun_out/m_pytest.log | tail -30; [ $rc -ne 0 ] && { tail -40 gpurun_out/m_pytest.log; exit $rc; }
timeout -k 10 300 python scripts/debug/find_elementwise.py > gpurun_out/m_elementwise.log 2>&1 || { tail -20 gpurun_out/m_elementwise.log; exit 1; }
grep -v amdgpu.ids gpurun_out/m_elementwise.log | head -45
timeout -k 10 500 python benchmarks/bench_bert.py > gpurun_out/m_bert.log 2>&1 || { tail -20 gpurun_out/m_bert.log; exit 1; }
grep '"metric"' gpurun_out/m_bert.log | cut -c1-900
