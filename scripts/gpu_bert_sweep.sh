#!/bin/bash
# BERT-Large config-5 sweep: per-GPU batch, then hipBLASLt/rocBLAS GEMM selection via
# PyTorch TunableOp (tune once, then replay the tuned table).
set -u
mkdir -p gpurun_out
run() { local log=$1 t=$2; shift 2; echo "== $log"; timeout -k 10 "$t" "$@" > gpurun_out/$log 2>&1; local rc=$?;
        grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/$log | tr '\n' ' '; echo " rc=$rc";
        if [ $rc -ge 124 ]; then exit $rc; fi; }
for bs in 64 128 256; do run bert_bs$bs.log 400 python benchmarks/bench_bert.py --batch $bs --steps 10 --warmup 3; done
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_bert%d.csv
PYTORCH_TUNABLEOP_TUNING=1 run bert_tune_bs${TBS:-256}.log 900 python benchmarks/bench_bert.py --batch ${TBS:-256} --steps 3 --warmup 2
PYTORCH_TUNABLEOP_TUNING=0 run bert_tuned_bs${TBS:-256}.log 400 python benchmarks/bench_bert.py --batch ${TBS:-256} --steps 10 --warmup 3
