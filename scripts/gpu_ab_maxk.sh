set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_conv_gpu.py tests/test_resnet_paths_gpu.py --maxfail=5 -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for v in 128 256 128 256; do
  MIVOD_BN_RECOMPUTE_MAXK=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ab_$v.log 2>&1 || { tail -20 gpurun_out/ab_$v.log; exit 1; }
  echo "RECOMPUTE_MAXK=$v $(grep -o '"value": [0-9.]*' gpurun_out/ab_$v.log)"
done
