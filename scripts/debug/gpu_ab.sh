mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pool_gpu.py tests/test_attention_gpu.py tests/test_resnet_paths_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1
for r in 1 2 3; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>&1 | grep -o '"ms_per_step": [0-9.]*'; done
