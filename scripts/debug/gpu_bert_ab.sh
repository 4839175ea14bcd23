timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1
for r in 1 2; do timeout -k 10 300 python benchmarks/bench_bert.py --steps 10 --warmup 3 2>&1 | grep -o '"value": [0-9.]*'; done
