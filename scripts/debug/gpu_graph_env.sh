mkdir -p gpurun_out
run() { echo "== $*"; env "$@" timeout -k 10 300 python bench.py --batch 512 --steps 10 --warmup 3 --graph 2>&1 | grep -o '"ms_per_step": [0-9.]*' || exit 1; }
timeout -k 10 300 python bench.py --batch 512 --steps 10 --warmup 3 2>&1 | grep -o '"ms_per_step": [0-9.]*'
run X=1
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
run DEBUG_HIP_FORCE_GRAPH_QUEUES=0
run DEBUG_HIP_FORCE_GRAPH_QUEUES=1
run DEBUG_HIP_GRAPH_BATCH_SIZE=1
run DEBUG_HIP_GRAPH_BATCH_SIZE=64
