set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/micro_wgrad1x1.py > gpurun_out/w1m.log 2>&1 || exit 1
for v in 1 0 1 0; do
  MIVOD_WGRAD1X1=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ab_$v.log 2>&1 || { tail -20 gpurun_out/ab_$v.log; exit 1; }
  echo "WGRAD1X1=$v $(grep -o '"value": [0-9.]*' gpurun_out/ab_$v.log)"
done
