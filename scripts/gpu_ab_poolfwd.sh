set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pool_gpu.py --maxfail=3 -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for v in 1 0 1 0; do
  MIVOD_POOL_FWD_BLOCK=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ab_$v.log 2>&1 || { tail -20 gpurun_out/ab_$v.log; exit 1; }
  echo "POOL_FWD_BLOCK=$v $(grep -o '"value": [0-9.]*' gpurun_out/ab_$v.log)"
done
