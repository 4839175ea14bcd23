mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pool_gpu.py tests/test_bn_gpu.py tests/test_gpu_hookpath.py tests/test_grad_tap.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
for r in 1 2; do for d in 0 1; do
  echo -n "DOWNSAMPLE_TAP=$d run $r: "; MIVOD_DOWNSAMPLE_TAP=$d timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>&1 | grep -o '"ms_per_step": [0-9.]*\|loss [0-9.a-z]*' | tr '\n' ' ' ; echo
done; done
