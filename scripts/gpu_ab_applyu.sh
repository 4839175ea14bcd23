set -o pipefail
mkdir -p gpurun_out
for v in 2 4 2 4; do
  MIVOD_BN_APPLY_U=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ab_$v.log 2>&1 || { tail -20 gpurun_out/ab_$v.log; exit 1; }
  echo "APPLY_U=$v $(grep -o '"value": [0-9.]*' gpurun_out/ab_$v.log)"
done
