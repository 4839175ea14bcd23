mkdir -p gpurun_out
for r in 1 2; do for nt in 0 1; do
  echo -n "NT=$nt run $r: "; MIVOD_BN_NT=$nt timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>&1 | grep -o '"ms_per_step": [0-9.]*' || exit 1
done; done
timeout -k 10 200 python -u -m pytest tests/test_bn_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1
