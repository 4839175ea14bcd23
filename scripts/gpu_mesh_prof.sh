#!/bin/bash
# Kernel-trace profile of the xGMI mesh allreduce: 2 ranks share the GPU (HIP IPC),
# rank 0 runs directly under rocprofv3, rank 1 plainly.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PORT=$((20000 + RANDOM % 20000))
common="MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MIVOD_TRANSPORT=gloo-gpu MIVOD_MESH_MAX_MB=8 OMP_NUM_THREADS=1 PYTHONPATH=$PWD"
env $common RANK=1 LOCAL_RANK=1 timeout -k 10 240 python tests/mp_workers.py gpu_mesh_bench > gpurun_out/mesh_r1.log 2>&1 &
P1=$!
env $common RANK=0 LOCAL_RANK=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mesh -o run -- python tests/mp_workers.py gpu_mesh_bench > gpurun_out/mesh_r0.log 2>&1
RC0=$?
wait $P1
RC1=$?
echo "rank0 rc=$RC0 rank1 rc=$RC1"
grep -h "mesh allreduce\|OK" gpurun_out/mesh_r0.log gpurun_out/mesh_r1.log
exit $(( RC0 | RC1 ))
