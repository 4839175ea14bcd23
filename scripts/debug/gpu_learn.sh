timeout -k 10 300 python -u -m pytest tests/test_graphs_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
timeout -k 10 300 python benchmarks/bench_graph_convnet.py 2>&1 | grep -v amdgpu
