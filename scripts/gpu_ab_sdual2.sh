set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -k "dual or shortcut" --maxfail=5 -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for v in "1 128" "0 128" "1 256" "1 128" "0 128"; do
  set -- $v
  MIVOD_BN_SHORTCUT_DUAL=$1 MIVOD_GEMM_DUAL_BN=$2 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
  echo "DUAL=$1 BN=$2 $(grep -o '"value": [0-9.]*' gpurun_out/ab.log)"
done
